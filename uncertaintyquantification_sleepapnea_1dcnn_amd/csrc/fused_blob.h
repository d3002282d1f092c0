// Parameter-blob layout shared by the fused whole-network kernels (fused_forward.hip: the reference
// no-pool CNN; fused_pooled.hip: the same CNN with MaxPool1D(2) after blocks 1-5).  Both read one
// model's packed parameters (ops/fused.py:pack_blob) from the same byte offsets.
#pragma once

namespace apneauq {
namespace fused {

// channel / kernel-size table of the default spec (cnn_baseline_train.py:59-86)
constexpr int C[7] = {4, 128, 192, 224, 96, 256, 96};
constexpr int KS[6] = {7, 5, 3, 7, 9, 9};

__host__ __device__ constexpr int ksteps(int l) { return (C[l] * KS[l] + 31) / 32; }
__host__ __device__ constexpr int wbytes(int l) { return ksteps(l) * (C[l + 1] / 16) * 1024; }
constexpr int kEpiRows = 8;  // per-channel [s, t' = b*s + t, lo, hi], then the same x 1/(1-rate) (ops/fused.py)
__host__ __device__ constexpr int ebytes(int l) { return ((kEpiRows * C[l + 1] * 4) + 15) / 16 * 16; }
__host__ __device__ constexpr int woff(int l) { return l == 0 ? 0 : woff(l - 1) + wbytes(l - 1); }
__host__ __device__ constexpr int eoff(int l) { return l == 0 ? woff(6) : eoff(l - 1) + ebytes(l - 1); }
constexpr int kDenseOff = eoff(6);
constexpr int kBlobBytes = kDenseOff + ((C[6] + 1) * 4 + 15) / 16 * 16;

// fp16x3 blob (fused_tiled_x3.hip, ops/fused.py:pack_blob_x3): per (k-step, channel tile) the hi and
// the lo fragment of W 2^sw (2 KiB), then the same epilogue rows (scale x 2^-sw) and dense head
__host__ __device__ constexpr int wbytes3(int l) { return 2 * wbytes(l); }
__host__ __device__ constexpr int woff3(int l) { return l == 0 ? 0 : woff3(l - 1) + wbytes3(l - 1); }
__host__ __device__ constexpr int eoff3(int l) { return l == 0 ? woff3(6) : eoff3(l - 1) + ebytes(l - 1); }
constexpr int kDenseOff3 = eoff3(6);
constexpr int kBlobBytes3 = kDenseOff3 + ((C[6] + 1) * 4 + 15) / 16 * 16;

}  // namespace fused
}  // namespace apneauq
