// Kernel-argument structs of the fp32-faithful layer-wise inference kernels (x3_layers.hip), shared
// by the HIP translation unit and the host bindings (plain C++ types only).
#pragma once

namespace apneauq {
namespace x3 {

struct LayerArgs {
  const float* in;        // R_{l-1}: [samples_in][60][CIN] fp32 ReLU output (before BN and dropout)
  float* out;             // R_l [samples][60][COUT] fp32; block 6: masked sums [samples][2][COUT]
  const void* wfrag;      // [G][chunk][tap][ct][hi|lo][64 lanes][8] fp16
  long long w_gstride;    // 16-B fragments per weight group (0: one set shared by all groups)
  const float* bias;      // [G][COUT]
  const float* wscale;    // [G] 2^-sw (exact) undoing the host weight pre-scale
  int p_gstride;          // bias floats per weight group (0: shared; then wscale[0] too)
  const float* aff_in;    // [G][2][CIN] BN affine of block l-1 (scale | shift) x 1/(1-p_{l-1})
  int aff_gstride;        // floats per group (0: shared)
  // range-safe fp16 split (see x3_layers.hip sample_prescale): per-sample power-of-two prescale of the
  // staged activations from the sample's max of R_{l-1} and the affine's channel maxima
  const unsigned* smax_in;  // max of R_{l-1} per input sample (fp32 bits), indexed like the input rows
                            // (in_shared: window; else group * n_win + window); nullptr: no prescale
  const float* amax_in;     // [G][2] max_c |scale|, max_c |shift| of aff_in (aff_gstride 0: one pair)
  unsigned* smax_out;       // [G * n_win] max of R_l per sample (fp32 bits, atomicMax; nullptr: none)
  const float* gscale_in;   // [G] 2^-sa of aff_in's folded per-group prescale (aff_gstride 0: one), or
                            // nullptr
  double* stats;          // [G][16 slots][2][COUT] moment sums of R_l (nullptr: none)
  int n_win;              // windows per group
  int groups;
  int tiles_per_group;    // informational (the kernel derives its tiling from n_win, groups and its tile size)
  int total_tiles;
  int in_shared;          // input indexed by window only (block-1 output shared by all passes)
  int sign_in;            // the input carries block l-1's dropout mask in its sign bits (else: hashed here)
  int sign_out;           // draw block l's mask in the epilogue, stored as the sign bit (blocks 2..5)
  unsigned thr_in;        // 16-bit drop threshold of block l-1, whose mask the staging draws (0: no dropout)
  unsigned thr_out;       // 16-bit drop threshold of block l (block 6 only: its masked sums; 0: no dropout)
  int layer;              // 0-based index of this block (dropout streams: layer - 1 in, layer out)
  unsigned pass_base;     // dropout pass id of group 0
  unsigned window_offset;
  unsigned long long seed;
};

struct L1Args {
  const float* x;      // [n_win][60][4]
  const float* w;      // [G][7][4][128]
  const float* b;      // [G][128]
  float* out;          // [G][n_win][60][128]
  double* stats;       // [G][16][2][128] or nullptr
  unsigned* smax;      // [G][n_win] max of R_1 per sample (fp32 bits) or nullptr
  int n_win, groups, blocks_per_group;
};

struct AffArgs {
  const double* stats;   // [G][16][2][C] or nullptr (moving statistics)
  const float* gamma;    // [Gp][C] (p_gstride = 0: shared)
  const float* beta;
  float* mmean;
  float* mvar;
  float* aff;            // [G][2][C]
  float* amax;           // [G][2] out: max_c |aff scale|, max_c |aff shift| (nullptr: not written)
  float* gscale;         // [G] out (batch moments only): 2^-sa of the per-group prescale folded into aff
                         // (nullptr: none)
  int C, groups, p_gstride, update;
  int repeat;            // moving updates per stats group (block 1 moments are shared by all passes)
  double inv_count;
  float eps, momentum, dsc;
  int running;           // affine from the moving statistics; stats (if given) only bound the range (gscale)
};

struct HeadArgs {
  const float* sums;    // [samples][2][C]
  const float* aff;     // [G][2][C] (block-6 affine x 1/(1-p6))
  const float* dw;      // [Gp][C]
  const float* db;      // [Gp]
  float* out;           // [samples]
  int C, n_win, samples, aff_gstride, p_gstride, out_logits;
};

constexpr int kL1Win = 8;        // windows per block-1 workgroup
constexpr int kStatSlots = 16;   // interleaved moment-sum slots (workgroup % 16)

}  // namespace x3
}  // namespace apneauq
