// Building blocks of the persistent fused kernels (fused.hip: C3k2, detect_cls.hip: the Detect cls branch): one
// block keeps its convs' packed A fragments in LDS and runs a chain of conv stages per tile, the intermediates in LDS.
#pragma once
#include "common.h"

namespace fce {

// Barrier between two stages of one tile: the LDS writes published (lgkmcnt(0)), the global traffic left in flight
// (__syncthreads() also waits vmcnt(0), i.e. for the next tile's input prefetch and the tile's output stores)
__device__ __forceinline__ void stage_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ h4 h4_of(const float (&v)[4]) {
  return h4{(_Float16)fpin(v[0]), (_Float16)fpin(v[1]), (_Float16)fpin(v[2]), (_Float16)fpin(v[3])};
}

// One conv stage for the wave's MF pixel fragments (fragment f = wave + NW i) x CT cout tiles over NS K-steps,
// fully unrolled: A from the stage's LDS fragments ([ct][step][lane]), B = bl(i, step); then epi(i, ct, acc).
// Each output sums the K-steps in order with v_mfma_f32_16x16x32_f16 from zero: the unfused conv kernels' order.
template <int MF, int CT, int NS, typename BL, typename EPI>
__device__ __forceinline__ void mfma_stage(const h8* wl, BL bl, EPI epi) {
  f4 acc[MF][CT];
#pragma unroll
  for (int i = 0; i < MF; ++i)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) acc[i][ct] = f4{0.f, 0.f, 0.f, 0.f};
  // the fragments of step st + 1 are read while step st's MFMAs run (register double buffer; with the reads of a
  // step issued only after the previous step's MFMAs, every step waited out a full LDS round trip at two waves per
  // SIMD)
  h8 av[2][CT], bv[2][MF];
  auto load = [&](int st, h8 (&a)[CT], h8 (&b)[MF]) {
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) a[ct] = wl[(ct * NS + st) * 64];
#pragma unroll
    for (int i = 0; i < MF; ++i) b[i] = bl(i, st);
  };
  load(0, av[0], bv[0]);
#pragma unroll
  for (int st = 0; st < NS; ++st) {
    if (st + 1 < NS) load(st + 1, av[(st + 1) & 1], bv[(st + 1) & 1]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
        acc[i][ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av[st & 1][ct], bv[st & 1][i], acc[i][ct], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int i = 0; i < MF; ++i)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) epi(i, ct, acc[i][ct]);
}

// Copy one conv's packed fragments (conv_pack layout [cout tile][nalloc][64 lanes]) into LDS as [ct][step][lane]
// (the first ns steps of every cout tile), by all nt threads of the block
__device__ __forceinline__ void stage_copy_frags(h8* dst, const h8* src, int ct_n, int ns, int nalloc, int nt) {
  const int nfr = ct_n * ns * 64;
  for (int e0 = int(threadIdx.x); e0 < nfr; e0 += 4 * nt) {
    h8 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = e0 + u * nt;
      const int k = e >> 6, ct = k / ns, stp = k - ct * ns;
      if (e < nfr) v[u] = src[(size_t(ct) * nalloc + stp) * 64 + (e & 63)];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = e0 + u * nt;
      if (e < nfr) dst[e] = v[u];
    }
  }
}

// dense_geom's per-cout-tile fragment count of a (cin, k x k) conv
inline int stage_nalloc(int cin, int k) {
  const int nsteps = (k * k * (cin / 8) + 3) / 4;
  return ((nsteps + 7) & ~7) + 8;
}

}  // namespace fce
