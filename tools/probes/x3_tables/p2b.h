// A/B table (round 5): two workgroups per CU, Cout-96 blocks at 2-sample tiles, 64-channel chunks
#define APNEAUQ_X3_LAYERS(X)                     \
  X(1, 128, 192, 5, 2, 1, 4, false, 0, 0, 32, 2) \
  X(2, 192, 224, 3, 2, 2, 2, false, 0, 0, 64, 2) \
  X(3, 224, 96, 7, 2, 2, 2, false, 0, 0, 32, 2)  \
  X(4, 96, 256, 9, 2, 1, 4, false, 0, 0, 64, 2)  \
  X(5, 256, 96, 9, 2, 2, 2, true, 0, 0, 64, 2)
