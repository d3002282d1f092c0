"""Probe build of the x3 layer kernels with per-wave phase stamps (and optional timing-only ablations):
patches a copy of csrc/x3_layers.hip in place, builds gpuprobe/<name>.so, restores the source.  Read
the stamps with tools/x3_prof_run.py.  The library source never carries these hooks.

    python tools/probes/x3_prof_build.py <name> [nohash] [nostats]
"""
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(ROOT, "uncertaintyquantification_sleepapnea_1dcnn_amd", "csrc", "x3_layers.hip")


def rep(s, a, b):
    assert a in s, a[:80]
    return s.replace(a, b)


def patch(s, abl):
    s = rep(s, "namespace apneauq {\nnamespace x3 {\n", """__device__ unsigned long long g_x3prof[8][16];
extern "C" void x3_prof_dump(unsigned long long* out) { hipMemcpyFromSymbol(out, HIP_SYMBOL(g_x3prof), sizeof(g_x3prof)); }
extern "C" void x3_prof_reset() {
  static unsigned long long z[8][16] = {};
  hipMemcpyToSymbol(HIP_SYMBOL(g_x3prof), z, sizeof(z));
}
#define PSTAMP() __builtin_amdgcn_s_memtime()
namespace apneauq {
namespace x3 {
""")
    s = rep(s, """      compute_chunk(c, smem + (it & 1) * kBufB, wcur, wnxt, []() {});
      if (c == NCH - 1) epilogue(tile);
      lds_barrier();
    }
    flush_stats(g_cur);
    return;""", """      unsigned long long q0 = PSTAMP();
      compute_chunk(c, smem + (it & 1) * kBufB, wcur, wnxt, []() {});
      unsigned long long q1 = PSTAMP();
      if (c == NCH - 1) epilogue(tile);
      unsigned long long q2 = PSTAMP();
      lds_barrier();
      pc += q1 - q0; pe += q2 - q1; pb += PSTAMP() - q2;
    }
    flush_stats(g_cur);
    if (lane == 0) {
      atomicAdd(&g_x3prof[A.layer][0], pc); atomicAdd(&g_x3prof[A.layer][1], pe);
      atomicAdd(&g_x3prof[A.layer][2], pb); atomicAdd(&g_x3prof[A.layer][3], PSTAMP() - pt0);
      atomicAdd(&g_x3prof[A.layer][4], 1ull);
    }
    return;""")
    s = rep(s, """    lds_barrier();
    load_a(wbase(t_begin), ah, al);
#pragma unroll 1
    for (int it = 0; it < total; ++it) {""", """    unsigned long long pt0 = PSTAMP(), pc = 0, pe = 0, pb = 0;
    lds_barrier();
    load_a(wbase(t_begin), ah, al);
#pragma unroll 1
    for (int it = 0; it < total; ++it) {""")
    s = rep(s, """        if (stager && it + 1 < total) store_chunk(chunk_tile(it + 1), (it + 1) % NCH, smem + ((it + 1) & 1) * kBufB, s0);
        lds_barrier();
        if (stager && it + 2 < total) load_chunk(chunk_tile(it + 2), (it + 2) % NCH, s0);
      }
      flush_stats(g_cur);
      return;""", """        unsigned long long q0 = PSTAMP();
        if (stager && it + 1 < total) store_chunk(chunk_tile(it + 1), (it + 1) % NCH, smem + ((it + 1) & 1) * kBufB, s0);
        unsigned long long q1 = PSTAMP();
        lds_barrier();
        unsigned long long q2 = PSTAMP();
        if (stager && it + 2 < total) load_chunk(chunk_tile(it + 2), (it + 2) % NCH, s0);
        ps += q1 - q0; pb += q2 - q1; pl += PSTAMP() - q2;
      }
      flush_stats(g_cur);
      if (lane == 0) {
        atomicAdd(&g_x3prof[A.layer][8], ps); atomicAdd(&g_x3prof[A.layer][9], pb);
        atomicAdd(&g_x3prof[A.layer][10], pl); atomicAdd(&g_x3prof[A.layer][11], PSTAMP() - pt0);
        atomicAdd(&g_x3prof[A.layer][12], 1ull);
      }
      return;""")
    s = rep(s, """      lds_barrier();
      if (stager && total > 1) load_chunk(chunk_tile(1), 1 % NCH, s0);
#pragma unroll 1
      for (int it = 0; it < total; ++it) {""", """      unsigned long long pt0 = PSTAMP(), ps = 0, pb = 0, pl = 0;
      lds_barrier();
      if (stager && total > 1) load_chunk(chunk_tile(1), 1 % NCH, s0);
#pragma unroll 1
      for (int it = 0; it < total; ++it) {""")
    s = rep(s, """    compute_chunk(c, buf, wcur, wnxt, [&]() {
      if (stager && it + 1 < total) store_chunk(chunk_tile(it + 1), (it + 1) % NCH, nbuf, s0);
    });
    if (c == NCH - 1) epilogue(tile);
    lds_barrier();
    if (stager && it + 2 < total) load_chunk(chunk_tile(it + 2), (it + 2) % NCH, s0);
  }
  flush_stats(g_cur);
}""", """    unsigned long long q0 = PSTAMP();
    compute_chunk(c, buf, wcur, wnxt, [&]() {
      if (stager && it + 1 < total) store_chunk(chunk_tile(it + 1), (it + 1) % NCH, nbuf, s0);
    });
    unsigned long long q1 = PSTAMP();
    if (c == NCH - 1) epilogue(tile);
    unsigned long long q2 = PSTAMP();
    lds_barrier();
    unsigned long long q3 = PSTAMP();
    if (stager && it + 2 < total) load_chunk(chunk_tile(it + 2), (it + 2) % NCH, s0);
    ppc += q1 - q0; ppe += q2 - q1; ppb += q3 - q2; ppl += PSTAMP() - q3;
  }
  flush_stats(g_cur);
  if (lane == 0) {
    atomicAdd(&g_x3prof[A.layer][0], ppc); atomicAdd(&g_x3prof[A.layer][1], ppe);
    atomicAdd(&g_x3prof[A.layer][2], ppb); atomicAdd(&g_x3prof[A.layer][3], PSTAMP() - ppt0);
    atomicAdd(&g_x3prof[A.layer][4], 1ull); atomicAdd(&g_x3prof[A.layer][5], ppl);
  }
}""")
    s = rep(s, """  if (stager) {
    load_chunk(t_begin, 0, s0);
    store_chunk(t_begin, 0, smem, s0);
  }
  lds_barrier();
  if (stager && total > 1) load_chunk(chunk_tile(1), 1 % NCH, s0);
  load_a(wbase(t_begin), ah, al);""", """  unsigned long long ppt0 = PSTAMP(), ppc = 0, ppe = 0, ppb = 0, ppl = 0;
  if (stager) {
    load_chunk(t_begin, 0, s0);
    store_chunk(t_begin, 0, smem, s0);
  }
  lds_barrier();
  if (stager && total > 1) load_chunk(chunk_tile(1), 1 % NCH, s0);
  load_a(wbase(t_begin), ah, al);""")
    if "nohash" in abl:  # timing only: the epilogue's mask is a cheap function of (t, channel)
        s = rep(s, "const unsigned b01 = dropout_bits2(key, t, co0), b23 = dropout_bits2(key, t, co0 + 2);",
                "const unsigned b01 = (key ^ (t * 0x9E3779B9u)) + co0, b23 = b01 * 3u;")
    if "nostats" in abl:  # timing only: no per-tile moment reductions
        s = rep(s, """      // reduce over the 16 rows of each lane group (lanes sharing h hold the same 4 channels)
      if (A.stats != nullptr) {""", """      if (A.stats != nullptr && s1[0] == 1234.5f) {""")
    return s


def main():
    name, abl = sys.argv[1], sys.argv[2:]
    orig = open(SRC).read()
    try:
        open(SRC, "w").write(patch(orig, abl))
        os.environ["APNEAUQ_SO_OUT"] = os.path.join(ROOT, "gpuprobe", name + ".so")
        sys.path.insert(0, ROOT)
        from uncertaintyquantification_sleepapnea_1dcnn_amd.csrc import build as b
        b.EXTRA.append("-DX3_PROF_BUILD")
        print(b.build(force=True, jobs=8))
    finally:
        open(SRC, "w").write(orig)


if __name__ == "__main__":
    main()
