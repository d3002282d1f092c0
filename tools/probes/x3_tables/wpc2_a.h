// A/B table: two persistent workgroups per CU (4 MFMA + 2 loader waves each) for blocks 4 and 6
#define APNEAUQ_X3_LAYERS(X)                  \
  X(1, 128, 192, 5, 4, 2, 4, false, -8, 32, 1) \
  X(2, 192, 224, 3, 2, 1, 7, false, 4, 64, 1) \
  X(3, 224, 96, 7, 2, 2, 2, false, 2, 32, 2)  \
  X(4, 96, 256, 9, 2, 1, 8, false, 4, 32, 1)  \
  X(5, 256, 96, 9, 2, 2, 2, true, 2, 32, 2)
