// Fused C3k2 block (reference ultralytics/nn/modules/block.py C2f.forward :303-307 with C3k2's
// Bottleneck branch :1064-1084, Bottleneck.forward :474-476): for c3k = False and one repeat,
//
//   t = SiLU(cv1(x))            1x1, cin -> 2c          t = [a | b]
//   h = SiLU(m.cv1(b))          3x3, c -> c_mid
//   m = SiLU(m.cv2(h)) + b      3x3, c_mid -> c   (shortcut)
//   y = SiLU(cv2([a | b | m]))  1x1, 3c -> cout
//
// in ONE persistent kernel.  A block owns a contiguous run of TH x TW output tiles and keeps the four
// convs' packed A fragments and biases resident in LDS for its whole life (copied once); per tile
//   stage 1: cv1 over the tile + 2-pixel halo, its B operands (x) loaded straight from HBM into registers
//            while the PREVIOUS tile's stages 2-4 run (one read of x per tile, latency off the critical path),
//   stage 2: m.cv1 over the tile + 1-pixel halo, from the t image in LDS,
//   stage 3: m.cv2 + the residual b over the tile, into the m image in LDS,
//   stage 4: cv2 over [a | b | m] from LDS, y to HBM.
// t / h / m never leave LDS: the block is one read of x and one write of y (the four separate convs move
// x, t twice, h twice, m twice and [a | b | m] through HBM, n32's L2 block alone ~390 MB against ~157 MB).
// Every shape is a compile-time constant of the (cin, c, c_mid, cout, tile) instantiation: the stages' K loops
// unroll with no guards between MFMAs (a first version with runtime counts wrapped every MFMA in its own branch
// and ran 2.2x slower than the four convs); waves with fewer fragments compute clamped positions and skip
// the stores.
//
// Bitwise identical to the four unfused convs (conv_mfma_kernel and its variants): every stage walks
// the same K-steps of the same packed A fragments (conv_pack: chunk-major for cin % 32 == 0, else
// tap-major 8-channel chunks c = 4 s + lane / 16) with v_mfma_f32_16x16x32_f16 from zero, the B data
// are the same fp16 values (intermediates rounded to fp16 exactly where the unfused path stores them,
// zeros where it zero-pads), and the epilogue arithmetic is conv_epilogue's (bias, SiLU, residual add,
// fpin before every fp16 conversion).
#include <algorithm>

#include "mfma_stage.h"

namespace fce {

static __device__ __attribute__((aligned(16))) _Float16 g_c3_zero[8];

// compile-time geometry of one instantiation (LDS offsets in 16-byte units)
template <int CIN, int C, int CM, int COUT, int TH, int TW, int NW>
struct C3G {
  static constexpr int R2W = TW + 4, R2 = (TH + 4) * R2W;  // cv1 region: tile + 2-pixel halo
  static constexpr int R1W = TW + 2, R1 = (TH + 2) * R1W;  // m.cv1 region: tile + 1-pixel halo
  static constexpr int NC = TH * TW;
  static constexpr int NF1 = (R2 + 15) / 16, NF2 = (R1 + 15) / 16, NF4 = (NC + 15) / 16;
  static constexpr int MF1 = (NF1 + NW - 1) / NW, MF2 = (NF2 + NW - 1) / NW, MF4 = (NF4 + NW - 1) / NW;
  static constexpr int CT1 = 2 * C / 16, CT2 = (CM + 15) / 16, CT3 = (C + 15) / 16, CT4 = (COUT + 15) / 16;
  static constexpr bool F2 = C % 32 == 0, F3 = CM % 32 == 0;  // chunk-major K order of the 3x3s
  // K-steps exactly as dense_geom / conv_pack count them: (taps * cin / 8 + 3) / 4
  static constexpr int NS1 = CIN / 32, NS2 = (9 * (C / 8) + 3) / 4, NS3 = (9 * (CM / 8) + 3) / 4,
                       NS4 = (3 * C / 8 + 3) / 4;
  static constexpr int sT = (2 * C / 8) | 1, sH = (CM / 8) | 1, sM = (C / 8) | 1;
  static constexpr int W1 = CT1 * NS1 * 64, W2 = CT2 * NS2 * 64, W3 = CT3 * NS3 * 64, W4 = CT4 * NS4 * 64;
  static constexpr int OW2 = W1, OW3 = W1 + W2, OW4 = W1 + W2 + W3, OB = W1 + W2 + W3 + W4;
  static constexpr int B2 = CT1 * 16, B3 = B2 + CT2 * 16, B4 = B3 + CT3 * 16, NB = B4 + CT4 * 16;  // floats
  static constexpr int OT = OB + NB / 4, OH = OT + R2 * sT, OM = OH + R1 * sH, TOTAL = OM + NC * sM;
  static constexpr size_t LDS = size_t(TOTAL) * 16;
  static_assert(CIN % 32 == 0 && C % 8 == 0 && CM % 8 == 0 && COUT % 8 == 0, "c3k2 fused: channel alignment");
};

struct C3k2Args {
  const _Float16* x;
  int xcs;
  _Float16* y;
  int ycs;
  int H, W, tiles_x, tiles_y, ntiles;
  const h8* w[4];     // packed A fragments (conv_pack layout: [cout tile][nalloc][64 lanes])
  int nalloc[4];      // fragments stored per cout tile
  const float* b[4];  // biases (BN folded)
  int diag;           // FCE_C3K2_DIAG: block 0 prints its per-stage clocks
};

// SiLU(acc + bias) of lane group grp's 4 couts of tile ct (the bias from the block's LDS copy: a global load in
// an epilogue would make it wait for the next tile's x prefetch, vmcnt retiring in issue order)
__device__ __forceinline__ void c3_act(const float* bias, int ct, int grp, const f4& acc, float (&v)[4]) {
  const int co0 = ct * 16 + grp * 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = silu(acc[j] + bias[co0 + j]);
}

// (tap, 8-channel chunk, real step) of K-step st for lane group grp: chunk-major steps (cin % 32 == 0) are
// (32-channel chunk st / 9, tap st % 9); otherwise the tap-major 8-channel chunks k = 4 st + grp
template <bool FAST, int CPT>
__device__ __forceinline__ void c3_kstep(int st, int grp, int& tap, int& cc, bool& ok) {
  if (FAST) {
    tap = st % 9;
    cc = (st / 9) * 4 + grp;
    ok = true;
  } else {
    const int k = st * 4 + grp;
    tap = k / CPT;
    cc = k - tap * CPT;
    ok = tap < 9;
  }
}

__device__ __forceinline__ void c3_tile(const C3k2Args& a, int TH, int TW, int t, int& n, int& y0, int& x0) {
  const int tx = t % a.tiles_x;
  t /= a.tiles_x;
  const int ty = t % a.tiles_y;
  n = t / a.tiles_y;
  y0 = ty * TH;
  x0 = tx * TW;
}

template <int CIN, int C, int CM, int COUT, int TH, int TW, int NW, bool YB>
__global__ __launch_bounds__(NW * 64, 2) void c3k2_fused_kernel(C3k2Args a) {
  using G = C3G<CIN, C, CM, COUT, TH, TW, NW>;
  extern __shared__ __attribute__((aligned(16))) h8 sm[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, col = lane & 15, grp = lane >> 4;
  const int NG = gridDim.x, bi = blockIdx.x;
  const int t_begin = int(int64_t(bi) * a.ntiles / NG), t_end = int(int64_t(bi + 1) * a.ntiles / NG);
  if (t_begin >= t_end) return;  // block-uniform

  // stage-1 B operands of tile t: x at the cv1 region's positions (zero line outside the image / region)
  h8 xb[G::MF1][G::NS1];
  auto load_x = [&](int t) {
    int n, y0, x0;
    c3_tile(a, TH, TW, t, n, y0, x0);
    const _Float16* zl = g_c3_zero;
#pragma unroll
    for (int i = 0; i < G::MF1; ++i) {
      const int q = (wave + NW * i) * 16 + col;
      const int r = q / G::R2W, cq = q - r * G::R2W;
      const int iy = y0 - 2 + r, ix = x0 - 2 + cq;
      const bool in = q < G::R2 && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
      const _Float16* src = a.x + (in ? nhwc_off(n, iy, ix, a.H, a.W, a.xcs) + grp * 8 : 0);
#pragma unroll
      for (int s = 0; s < G::NS1; ++s) xb[i][s] = *reinterpret_cast<const h8*>(in ? src + s * 32 : zl);
    }
  };
  load_x(t_begin);
  // the four convs' fragments and biases -> LDS, once per block
  {
    const int wofs[4] = {0, G::OW2, G::OW3, G::OW4}, cts[4] = {G::CT1, G::CT2, G::CT3, G::CT4};
    const int nss[4] = {G::NS1, G::NS2, G::NS3, G::NS4}, couts[4] = {2 * C, CM, C, COUT};
    const int bofs[4] = {0, G::B2, G::B3, G::B4};
    float* bias = reinterpret_cast<float*>(sm + G::OB);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      stage_copy_frags(sm + wofs[s], a.w[s], cts[s], nss[s], a.nalloc[s], NW * 64);
      for (int e = int(threadIdx.x); e < cts[s] * 16; e += NW * 64) bias[bofs[s] + e] = e < couts[s] ? a.b[s][e] : 0.f;
    }
  }
  __syncthreads();

  const float* bias = reinterpret_cast<const float*>(sm + G::OB);
  _Float16* T = reinterpret_cast<_Float16*>(sm + G::OT);
  _Float16* Hh = reinterpret_cast<_Float16*>(sm + G::OH);
  _Float16* Mm = reinterpret_cast<_Float16*>(sm + G::OM);
  const h8* Tin = sm + G::OT;
  const h8* Hin = sm + G::OH;
  const h8* Min = sm + G::OM;
  // diagnostics (FCE_C3K2_DIAG=1): block 0, wave 0 sums s_memtime clocks per stage over its tiles and prints them
  uint64_t clk[6] = {0, 0, 0, 0, 0, 0}, tprev = a.diag ? __builtin_amdgcn_s_memtime() : 0;
  auto tick = [&](int k) {
    if (a.diag) {
      const uint64_t tn = __builtin_amdgcn_s_memtime();
      clk[k] += tn - tprev;
      tprev = tn;
    }
  };

  for (int t = t_begin; t < t_end; ++t) {
    int n, y0, x0;
    c3_tile(a, TH, TW, t, n, y0, x0);
    // ---------------- stage 1: t = cv1(x) over the cv1 region (B operands already in registers)
    {
      auto bl = [&](int i, int st) -> h8 { return xb[i][st]; };
      auto epi = [&](int i, int ct, const f4& acc) {
        const int q = (wave + NW * i) * 16 + col;
        if (q >= G::R2) return;
        const int r = q / G::R2W, cq = q - r * G::R2W;
        const int iy = y0 - 2 + r, ix = x0 - 2 + cq;
        float v[4];
        c3_act(bias, ct, grp, acc, v);
        h4 o = h4_of(v);
        if (!(iy >= 0 && iy < a.H && ix >= 0 && ix < a.W)) o = h4{0, 0, 0, 0};  // the 3x3s' zero padding of b
        *reinterpret_cast<h4*>(T + (q * G::sT) * 8 + ct * 16 + grp * 4) = o;
      };
      mfma_stage<G::MF1, G::CT1, G::NS1>(sm + lane, bl, epi);
    }
    tick(0);
    if (t + 1 < t_end) load_x(t + 1);  // in flight during stages 2-4
    tick(1);
    stage_barrier();
    // ---------------- stage 2: h = m.cv1(b) over the m.cv1 region (3x3 from the t image)
    {
      int pb[G::MF2];
#pragma unroll
      for (int i = 0; i < G::MF2; ++i) {
        const int q = min((wave + NW * i) * 16 + col, G::R1 - 1);  // clamped: waves past the last fragment
        const int r = q / G::R1W, cq = q - r * G::R1W;
        pb[i] = r * G::R2W + cq;  // tap (0, 0) of output (r, cq): R2 position (r + 1 - 1, cq + 1 - 1)
      }
      auto bl = [&](int i, int st) -> h8 {
        int tap, cc;
        bool ok;
        c3_kstep<G::F2, C / 8>(st, grp, tap, cc, ok);
        const int ky = tap / 3, kx = tap - ky * 3;
        return ok ? Tin[(pb[i] + ky * G::R2W + kx) * G::sT + C / 8 + cc] : h8{0, 0, 0, 0, 0, 0, 0, 0};
      };
      auto epi = [&](int i, int ct, const f4& acc) {
        const int q = (wave + NW * i) * 16 + col;
        if (q >= G::R1 || ct * 16 + grp * 4 >= CM) return;  // past the region / a partial cout tile
        const int r = q / G::R1W, cq = q - r * G::R1W;
        const int iy = y0 - 1 + r, ix = x0 - 1 + cq;
        float v[4];
        c3_act(bias + G::B2, ct, grp, acc, v);
        h4 o = h4_of(v);
        if (!(iy >= 0 && iy < a.H && ix >= 0 && ix < a.W)) o = h4{0, 0, 0, 0};
        *reinterpret_cast<h4*>(Hh + (q * G::sH) * 8 + ct * 16 + grp * 4) = o;
      };
      mfma_stage<G::MF2, G::CT2, G::NS2>(sm + G::OW2 + lane, bl, epi);
    }
    tick(2);
    stage_barrier();
    // ---------------- stage 3: m = m.cv2(h) + b over the tile (3x3 from the h image)
    {
      int pb[G::MF4];
#pragma unroll
      for (int i = 0; i < G::MF4; ++i) {
        const int q = min((wave + NW * i) * 16 + col, G::NC - 1);
        const int r = q / TW, cq = q - r * TW;
        pb[i] = r * G::R1W + cq;
      }
      auto bl = [&](int i, int st) -> h8 {
        int tap, cc;
        bool ok;
        c3_kstep<G::F3, CM / 8>(st, grp, tap, cc, ok);
        const int ky = tap / 3, kx = tap - ky * 3;
        return ok ? Hin[(pb[i] + ky * G::R1W + kx) * G::sH + cc] : h8{0, 0, 0, 0, 0, 0, 0, 0};
      };
      auto epi = [&](int i, int ct, const f4& acc) {
        const int q = (wave + NW * i) * 16 + col;
        const int co0 = ct * 16 + grp * 4;
        if (q >= G::NC || co0 >= C) return;
        const int r = q / TW, cq = q - r * TW;
        float v[4];
        c3_act(bias + G::B3, ct, grp, acc, v);
        const h4 rv = *reinterpret_cast<const h4*>(T + (((r + 2) * G::R2W + cq + 2) * G::sT) * 8 + C + co0);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = fpin(v[j] + (float)rv[j]);
        *reinterpret_cast<h4*>(Mm + (q * G::sM) * 8 + co0) = h4_of(v);
      };
      mfma_stage<G::MF4, G::CT3, G::NS3>(sm + G::OW3 + lane, bl, epi);
    }
    tick(3);
    stage_barrier();
    // ---------------- stage 4: y = cv2([a | b | m]) over the tile, to HBM
    {
      int pt[G::MF4], pm[G::MF4];
#pragma unroll
      for (int i = 0; i < G::MF4; ++i) {
        const int q = min((wave + NW * i) * 16 + col, G::NC - 1);
        const int r = q / TW, cq = q - r * TW;
        pt[i] = ((r + 2) * G::R2W + cq + 2) * G::sT;
        pm[i] = q * G::sM - 2 * C / 8;
      }
      auto bl = [&](int i, int st) -> h8 {
        const int cc = st * 4 + grp;  // 1x1 (either K order): the 8-channel chunk of [a | b | m]
        if (cc >= 3 * C / 8) return h8{0, 0, 0, 0, 0, 0, 0, 0};
        return cc < 2 * C / 8 ? Tin[pt[i] + cc] : Min[pm[i] + cc];
      };
      // YB: y through a per-image buffer resource, every lane storing (store_h4_or_drop), so the next tile's
      // stage 1 waits for its x prefetch only, not for these stores; otherwise branched global stores
      const uint32_t img = uint32_t(a.H) * uint32_t(a.W) * uint32_t(a.ycs);
      const __amdgpu_buffer_rsrc_t yr = out_rsrc(a.y + int64_t(n) * img, img * 2u);
      auto epi = [&](int i, int ct, const f4& acc) {
        const int q = (wave + NW * i) * 16 + col;
        const int r = q / TW, cq = q - r * TW;
        const int iy = y0 + r, ix = x0 + cq;
        const bool ok = q < G::NC && ct * 16 + grp * 4 < COUT && iy < a.H && ix < a.W;
        if (!YB && !ok) return;
        float v[4];
        c3_act(bias + G::B4, ct, grp, acc, v);
        const int off = (iy * a.W + ix) * a.ycs + ct * 16 + grp * 4;
        if constexpr (YB) store_h4_or_drop(yr, ok, uint32_t(off) * 2u, h4_of(v));
        else *reinterpret_cast<h4*>(a.y + int64_t(n) * img + off) = h4_of(v);
      };
      mfma_stage<G::MF4, G::CT4, G::NS4>(sm + G::OW4 + lane, bl, epi);
    }
    tick(4);
    stage_barrier();  // stage 4's reads of t / m before the next tile's stage 1 overwrites them
    tick(5);
  }
  if (a.diag && blockIdx.x == 0 && threadIdx.x == 0) {
    const unsigned long long nt = (unsigned long long)(t_end - t_begin);
    printf("c3k2 fused diag: %llu tiles, clocks per tile: stage1 %llu, x-issue %llu, stage2 %llu, stage3 %llu, "
           "stage4 %llu, last barrier %llu\n", nt, (unsigned long long)clk[0] / nt, (unsigned long long)clk[1] / nt,
           (unsigned long long)clk[2] / nt, (unsigned long long)clk[3] / nt, (unsigned long long)clk[4] / nt,
           (unsigned long long)clk[5] / nt);
  }
}

// ============================================================================ host
// the instantiated channel configurations (cin, c, c_mid, cout): the n / s scales' C3k2 blocks with c3k = False
// whose four weight sets fit the LDS beside a tile (n L2 / L4 / L18, s L2); per configuration two tiles: 8 x 16
// with 4 waves (two blocks per CU) for maps >= 128 wide, 4 x 40 with 8 waves (one block per CU) below
struct C3Inst {
  int cin, c, cm, cout;
};
static constexpr C3Inst kC3Insts[] = {{32, 16, 8, 64}, {64, 32, 16, 128}, {32, 32, 16, 64}};

template <int CIN, int C, int CM, int COUT, int TH, int TW, int NW, bool YB>
static int c3_launch(const C3k2Args& a0, int H, int W, int N, hipStream_t s) {
  using G = C3G<CIN, C, CM, COUT, TH, TW, NW>;
  static_assert(G::LDS <= 160 * 1024, "c3k2 fused: LDS over 160 KiB");
  auto k = c3k2_fused_kernel<CIN, C, CM, COUT, TH, TW, NW, YB>;
  static const bool big = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
  if (!big && G::LDS > 64 * 1024) return fail(FCE_ERR_HIP, "c3k2 fused: cannot opt in to >64 KiB LDS");
  C3k2Args a = a0;
  a.tiles_x = (W + TW - 1) / TW;
  a.tiles_y = (H + TH - 1) / TH;
  const int64_t tiles = int64_t(a.tiles_x) * a.tiles_y * N;
  if (tiles == 0) return FCE_OK;
  FCE_CHECK(tiles < (int64_t(1) << 30), "c3k2 fused: grid too large");
  a.ntiles = int(tiles);
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
  }
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, NW * 64, G::LDS) != hipSuccess || occ < 1) occ = 1;
  {
    static const int cap = [] {  // FCE_C3K2_OCC=k (experiment): at most k resident blocks per CU
      const char* e = getenv("FCE_C3K2_OCC");
      return e ? atoi(e) : 0;
    }();
    if (cap > 0) occ = std::min(occ, cap);
  }
  const int grid = int(std::min<int64_t>(a.ntiles, int64_t(cus) * occ));
  FCE_LAUNCH(k, dim3(unsigned(grid)), dim3(NW * 64), G::LDS, s, a);
  return launch_status("c3k2_fused_kernel");
}

// FCE_C3K2_TILE="8,16,4" / "4,40,8" forces one of the two tiles (tests, tuning); otherwise by map width.  Any other
// value is an error (it once fell back to the choice by width silently).  Round 5 measured 16x16 (4 or 8 waves),
// 8x32, 4x40 with 4 waves and a y tile staged through LDS for 16-byte stores: none faster
template <int CIN, int C, int CM, int COUT>
static int c3_launch_cfg(const C3k2Args& a, int H, int W, int N, hipStream_t s) {
  const char* env = getenv("FCE_C3K2_TILE");  // read per call: tests switch it within one process
  bool wide = W >= 128;
  if (env && *env) {
    if (strcmp(env, "8,16,4") == 0) wide = true;
    else if (strcmp(env, "4,40,8") == 0) wide = false;
    else return fail(FCE_ERR_INVALID, "FCE_C3K2_TILE: only \"8,16,4\" or \"4,40,8\"");
  }
  // y stores: through a buffer resource, every lane storing, for the cout-64 blocks (n L2 73.1 against 75.7 us,
  // L18 44.1 against 44.5); branched global stores for cout 128 (n L4 53.4 against 56.0 us;
  // profiles/r05_c3k2_ystore_ab.txt).  FCE_C3K2_YSTORE=buf / global forces one (A/B runs); any other value is an error
  const char* yst = getenv("FCE_C3K2_YSTORE");
  bool yb = COUT <= 64;
  if (yst && *yst) {
    if (strcmp(yst, "buf") == 0) yb = true;
    else if (strcmp(yst, "global") == 0) yb = false;
    else return fail(FCE_ERR_INVALID, "FCE_C3K2_YSTORE: only \"buf\" or \"global\"");
  }
  if (wide) return yb ? c3_launch<CIN, C, CM, COUT, 8, 16, 4, true>(a, H, W, N, s) : c3_launch<CIN, C, CM, COUT, 8, 16, 4, false>(a, H, W, N, s);
  return yb ? c3_launch<CIN, C, CM, COUT, 4, 40, 8, true>(a, H, W, N, s) : c3_launch<CIN, C, CM, COUT, 4, 40, 8, false>(a, H, W, N, s);
}

static int c3_inst(const fce_c3k2_desc& d) {
  for (int i = 0; i < int(sizeof(kC3Insts) / sizeof(kC3Insts[0])); ++i)
    if (kC3Insts[i].cin == d.cin && kC3Insts[i].c == d.c && kC3Insts[i].cm == d.c_mid && kC3Insts[i].cout == d.cout)
      return i;
  return -1;
}

bool c3k2_fused_ok(const fce_c3k2_desc& d) { return c3_inst(d) >= 0; }

int c3k2_fused(const fce_c3k2_desc& d, const fce_tensor& x, const fce_tensor& y, hipStream_t s) {
  const int inst = c3_inst(d);
  FCE_CHECK(inst >= 0, "c3k2 fused: unsupported channel configuration");
  FCE_CHECK(x.layout == FCE_NHWC && y.layout == FCE_NHWC && x.dtype == FCE_F16 && y.dtype == FCE_F16,
            "c3k2 fused: NHWC f16 views");
  FCE_CHECK(x.c == d.cin && y.c == d.cout && x.n == y.n && x.h == y.h && x.w == y.w, "c3k2 fused: shape mismatch");
  FCE_CHECK(x.cstride % 8 == 0 && x.coff % 8 == 0 && y.cstride % 4 == 0 && y.coff % 4 == 0,
            "c3k2 fused: aligned channel slices");
  for (int i = 0; i < 4; ++i) FCE_CHECK(d.w[i] && d.b[i], "c3k2 fused: null weights");
  C3k2Args a{};
  a.x = static_cast<const _Float16*>(x.data) + x.coff;
  a.xcs = x.cstride;
  a.y = static_cast<_Float16*>(y.data) + y.coff;
  a.ycs = y.cstride;
  a.H = x.h;
  a.W = x.w;
  const int cins[4] = {d.cin, d.c, d.c_mid, 3 * d.c}, ks[4] = {1, 3, 3, 1};
  for (int i = 0; i < 4; ++i) {
    a.w[i] = static_cast<const h8*>(d.w[i]);
    a.b[i] = d.b[i];
    a.nalloc[i] = stage_nalloc(cins[i], ks[i]);
  }
  {
    const char* de = getenv("FCE_C3K2_DIAG");
    a.diag = de && atoi(de) != 0;
  }
  switch (inst) {
    case 0: return c3_launch_cfg<32, 16, 8, 64>(a, x.h, x.w, x.n, s);
    case 1: return c3_launch_cfg<64, 32, 16, 128>(a, x.h, x.w, x.n, s);
    default: return c3_launch_cfg<32, 32, 16, 64>(a, x.h, x.w, x.n, s);
  }
}

}  // namespace fce
