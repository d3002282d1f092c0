// Ablation timing of the fused inference kernel: build once per APNEAUQ_ABL value
// (see fused_forward.hip) and compare launch times to see where the kernel's cycles go.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DAPNEAUQ_ABL=<bits> -I<csrc> fused_ablation.hip -o abl_<bits>
//   ./abl_<bits> [mode=mcd|de] [n_win]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "fused_forward.hip"

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

static uint16_t to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return (uint16_t)((u + 0x7FFF + ((u >> 16) & 1)) >> 16);
}

int main(int argc, char** argv) {
  const bool mcd = argc < 2 || std::strcmp(argv[1], "de") != 0;
  const int n_win = argc > 2 ? std::atoi(argv[2]) : 16384;
  const int n_pass = mcd ? 50 : 1, n_member = mcd ? 1 : 8;
  const int blob_bytes = apneauq::fused_blob_bytes();
  std::vector<uint8_t> blob((size_t)blob_bytes * n_member);
  srand(7);
  for (int m = 0; m < n_member; ++m) {
    uint8_t* b = blob.data() + (size_t)m * blob_bytes;
    // weights: small bf16; epilogue/dense: sane fp32 (bias 0.01, scale 1, shift 0)
    const int wend = apneauq::fused::woff(6);
    for (int i = 0; i < wend / 2; ++i) {
      const uint16_t v = to_bf16(((rand() & 1023) - 512) / 8192.f);
      std::memcpy(b + 2 * i, &v, 2);
    }
    for (int l = 0; l < 6; ++l) {
      float* e = reinterpret_cast<float*>(b + apneauq::fused::eoff(l));
      const int co = apneauq::fused::C[l + 1];
      for (int c = 0; c < co; ++c) {
        e[c] = 1.f;                  // s
        e[co + c] = 0.01f;           // t' = b*s + t
        e[2 * co + c] = 0.f;         // lo (s >= 0: t)
        e[3 * co + c] = 1e30f;       // hi (+inf)
        for (int q = 0; q < 4; ++q) e[(4 + q) * co + c] = e[q * co + c] * 1.25f;  // MC-Dropout rows
      }
    }
    float* d = reinterpret_cast<float*>(b + apneauq::fused::kDenseOff);
    for (int c = 0; c <= 96; ++c) d[c] = 0.01f;
  }
  std::vector<uint16_t> x((size_t)n_win * 240);
  for (auto& v : x) v = to_bf16(((rand() & 1023) - 512) / 256.f);

  void *dx, *db;
  float* dout;
  CK(hipMalloc(&dx, x.size() * 2));
  CK(hipMalloc(&db, blob.size()));
  CK(hipMalloc(&dout, (size_t)n_member * n_pass * n_win * 4));
  CK(hipMemcpy(dx, x.data(), x.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(db, blob.data(), blob.size(), hipMemcpyHostToDevice));
  const unsigned thr[6] = {19661, 19661, 26214, 13107, 19661, 32768};
  const float dsc[6] = {1 / .7f, 1 / .7f, 1 / .6f, 1 / .8f, 1 / .7f, 2.f};
  auto run = [&]() {
    CK(apneauq::launch_fused_forward(dx, (const uint8_t*)db, blob_bytes, dout, n_win, n_pass, n_member, 0, 0, 2025ull,
                                     mcd ? 1 : 0, 0, thr, dsc, 0, nullptr));
  };
  run();
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 5;
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) run();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= iters;
  const double samples = (double)n_win * n_pass * n_member;
#ifdef APNEAUQ_STAMPS
  {
    run();
    CK(hipDeviceSynchronize());
    using namespace apneauq::fused;
    std::vector<unsigned long long> st((size_t)kStampWG * 4 * kStampN);
    std::vector<unsigned> cu(kStampWG);
    CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_stamps), st.size() * 8));
    CK(hipMemcpyFromSymbol(cu.data(), HIP_SYMBOL(g_stamp_cu), cu.size() * 4));
    char fn[256];
    std::snprintf(fn, sizeof fn, "gpurun_out/stamps_%s.bin", mcd ? "mcd" : "de");
    FILE* f = std::fopen(fn, "wb");
    if (f) {
      std::fwrite(cu.data(), 4, cu.size(), f);
      std::fwrite(st.data(), 8, st.size(), f);
      std::fclose(f);
    }
  }
#endif
  std::printf("{\"abl\": %d, \"mode\": \"%s\", \"ms\": %.3f, \"samples_per_s\": %.0f}\n", APNEAUQ_ABL, mcd ? "mcd" : "de", ms,
              samples / (ms * 1e-3));
  return 0;
}
