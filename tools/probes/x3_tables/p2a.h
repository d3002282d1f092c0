// A/B table (round 5): two independent workgroups per CU (their barriers and epilogues desynchronise,
// each SIMD pairs waves of different workgroups), MFMA waves stage
#define APNEAUQ_X3_LAYERS(X)                     \
  X(1, 128, 192, 5, 2, 1, 4, false, 0, 0, 32, 2) \
  X(2, 192, 224, 3, 2, 2, 2, false, 0, 0, 32, 2) \
  X(3, 224, 96, 7, 4, 2, 2, false, 4, 4, 32, 1)  \
  X(4, 96, 256, 9, 2, 1, 4, false, 0, 0, 32, 2)  \
  X(5, 256, 96, 9, 4, 2, 2, true, 4, 4, 64, 1)
