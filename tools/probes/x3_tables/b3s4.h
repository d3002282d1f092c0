// A/B table (round 6): block 3 at 4-sample tiles (256 rows per weight fragment), 7 MFMA waves staging, no loader waves
#define APNEAUQ_X3_LAYERS(X) \
  X(1, 128, 192, 5, 4, 2, 4, false, -8, 0, 32, 1) \
  X(2, 192, 224, 3, 4, 1, 7, false, -7, 0, 32, 1) \
  X(3, 224, 96, 7, 4, 2, 2, false, 4, 4, 32, 1) \
  X(4, 96, 256, 9, 2, 1, 8, false, 4, 4, 32, 1) \
  X(5, 256, 96, 9, 4, 2, 2, true, 4, 4, 64, 1)
