// A/B table (round 5): one MFMA wave per SIMD, alternative tilings
#define APNEAUQ_X3_LAYERS(X)                     \
  X(1, 128, 192, 5, 5, 1, 4, false, 0, 0, 32, 1) \
  X(2, 192, 224, 3, 4, 2, 2, false, 0, 0, 32, 1) \
  X(3, 224, 96, 7, 4, 2, 2, false, 0, 0, 32, 1)  \
  X(4, 96, 256, 9, 4, 2, 2, false, 0, 0, 32, 1)  \
  X(5, 256, 96, 9, 4, 2, 2, true, 0, 0, 64, 1)
