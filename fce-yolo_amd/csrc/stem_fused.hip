// The network's first two convs in one kernel (reference yolo11*.yaml backbone rows 0-1: Conv(3, c0, 3, 2) ->
// Conv(c0, c1, 3, 2); conv.py:39-89 with the BN folded): the stem's c0-channel output at half resolution -- the
// largest activation of the forward (n32 at 640: 105 MB written and read back) -- never leaves LDS.
//
// A persistent block walks a contiguous run of row groups (SR2 output rows of the second conv of one image); per group:
//   stage 1: the 4 SR2 + 3 input rows of the 3 channels (loaded into registers during the previous group) -> LDS as fp16 (stem_mfma_kernel's staging: f32 inputs
//            rounded, u8 inputs fp16(v / 255) as im.half() / 255 does), 16-byte zero pads each side;
//   stage 2: the stem over the 2 SR2 + 1 rows those outputs read (rows outside the image zero) -> LDS, stem_mfma_kernel's
//            arithmetic (B = the lane group's 8 gathered (ci, ky, kx) values, one v_mfma_f32_16x16x32_f16 per 16 couts
//            from zero, bias, SiLU, fp16), stored with the zero column either side and even / odd columns apart, so
//            the stride-2 taps of 16 consecutive outputs read 16 consecutive positions;
//   stage 3: the second conv (3x3 stride 2, c0 -> c1) from LDS: the K-steps of its packed fragments (tap-major
//            8-channel chunks, conv_pack's order for c0 % 32 != 0) with v_mfma_f32_16x16x32_f16 from zero, bias,
//            SiLU, fp16 NHWC stores (conv_epilogue's arithmetic).
// Bitwise equal to the two separate convs (tests/test_gpu.py::test_fused_stem_bitwise_equal_to_two_convs).
#include <algorithm>
#include <type_traits>

#include "mfma_stage.h"

namespace fce {

struct Stem2Args {
  const void* x;  // NCHW, 3 channels, fp16 / f32 / u8
  int N, H, W;    // input
  int Hs, Ws;     // stem output
  int Ho, Wo;     // second conv output
  const h8* w0;   // stem MFMA fragments: (c0 / 16) x 64 lanes (conv_pack's stem image, after the fp32 table)
  const float* b0;
  const h8* w1;   // second conv packed fragments [c1 / 16][nalloc][64]
  int nalloc1;
  const float* b1;
  _Float16* y;
  int ycs;
};

template <int C0, int C1, int SR2>
struct StG {
  static constexpr int IR = 4 * SR2 + 3;  // staged input rows
  static constexpr int NS = 2 * SR2 + 1;  // stem rows
  static constexpr int K1 = C0 / 8, sS = K1 | 1;  // stem chunks per position, LDS units per position (odd)
  static constexpr int RC0 = C0 / 16, CT1 = C1 / 16;
  // second conv K-steps as conv_pack orders them: chunk-major (32-channel chunk, tap) for c0 % 32 == 0, else
  // tap-major 8-channel chunks
  static constexpr bool CM = C0 % 32 == 0;
  static constexpr int NS1 = CM ? 9 * (C0 / 32) : (9 * K1 + 3) / 4;
  static_assert(C0 % 16 == 0 && C1 % 16 == 0, "stem fused: channel configuration");
};

// 8 consecutive input elements, raw (a prefetch register image: converted to fp16 only when written to LDS, so the
// conversion never waits on a load that is still in flight)
template <typename T>
struct StRaw {
  h8 v;
  __device__ __forceinline__ void load(const T* p) { v = *reinterpret_cast<const h8*>(p); }
  __device__ __forceinline__ void zero() { v = h8{0, 0, 0, 0, 0, 0, 0, 0}; }
  __device__ __forceinline__ h8 half8() const { return v; }
};
template <>
struct StRaw<float> {
  f4 a, b;
  __device__ __forceinline__ void load(const float* p) {
    a = reinterpret_cast<const f4*>(p)[0];
    b = reinterpret_cast<const f4*>(p)[1];
  }
  __device__ __forceinline__ void zero() { a = b = f4{0.f, 0.f, 0.f, 0.f}; }
  __device__ __forceinline__ h8 half8() const {  // stem_mfma_kernel: f32 inputs rounded to fp16
    return h8{(_Float16)a[0], (_Float16)a[1], (_Float16)a[2], (_Float16)a[3],
              (_Float16)b[0], (_Float16)b[1], (_Float16)b[2], (_Float16)b[3]};
  }
};
template <>
struct StRaw<uint8_t> {
  uint2 v;
  __device__ __forceinline__ void load(const uint8_t* p) { v = *reinterpret_cast<const uint2*>(p); }
  __device__ __forceinline__ void zero() { v = uint2{0u, 0u}; }
  __device__ __forceinline__ h8 half8() const {  // fp16(v / 255), as im.half() / 255 (stem_mfma_kernel's u8 path)
    h8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const unsigned u = ((j < 4 ? v.x : v.y) >> ((j & 3) * 8)) & 255u;
      o[j] = (_Float16)(float)(_Float16)((float)u / 255.0f);
    }
    return o;
  }
};

// Persistent: block b owns the contiguous run of row groups [g_begin, g_end) (a group = SR2 output rows of one image)
// and loads the next group's input rows into registers while the current group's stem and second conv run.
template <typename T, int C0, int C1, int SR2, int NW, int NXE>
__global__ __launch_bounds__(NW * 64, 1) void stem_fused_kernel(Stem2Args a) {
  using G = StG<C0, C1, SR2>;
  constexpr int NT = NW * 64;
  extern __shared__ __attribute__((aligned(16))) _Float16 ssm[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, col = lane & 15, grp = lane >> 4;
  const int tid = threadIdx.x;
  const int rows = (a.Ho + SR2 - 1) / SR2, ngroups = a.N * rows;
  const int NG = gridDim.x, bi = blockIdx.x;
  const int g_begin = int(int64_t(bi) * ngroups / NG), g_end = int(int64_t(bi + 1) * ngroups / NG);
  if (g_begin >= g_end) return;  // block-uniform
  const int WP = a.W + 16, CW = WP / 8;
  const int npos = a.Ws + 2, half = (npos + 1) / 2;  // stem positions: columns -1 .. Ws, even then odd
  _Float16* IN = ssm;                                  // [3][IR][WP]
  h8* S = reinterpret_cast<h8*>(ssm + 3 * G::IR * WP);  // [NS][npos][sS]
  const int ne = 3 * G::IR * CW;
  const T* x = static_cast<const T*>(a.x);
  StRaw<T> xr[NXE];
  auto load_in = [&](int g) {
    const int n = g / rows, iy0 = 4 * (g - n * rows) * SR2 - 3;  // first staged input row: 2 (2 oy0 - 1) - 1
#pragma unroll
    for (int k = 0; k < NXE; ++k) {
      const int e = tid + k * NT;
      const int cr = e / CW, q = e - cr * CW;
      const int ci = cr / G::IR, r = cr - ci * G::IR;
      const int iy = iy0 + r, ix0 = (q - 1) * 8;
      if (e < ne && iy >= 0 && iy < a.H && q >= 1 && ix0 < a.W)
        xr[k].load(x + ((int64_t(n) * 3 + ci) * a.H + iy) * a.W + ix0);
      else
        xr[k].zero();
    }
  };
  load_in(g_begin);
  // stem lane constants: the 8 k values (ci, ky, kx) of lane group grp -> offset from the window origin (k >= 27:
  // tap (0, 0, 0) again, zero weights, as stem_mfma_kernel)
  int koff[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int kq = 8 * grp + j, ci = kq / 9, t = kq - ci * 9;
    koff[j] = kq < 27 ? (ci * G::IR + t / 3) * WP + (t % 3) : 0;
  }
  h8 af[G::RC0];
  float bz0[G::RC0][4];
#pragma unroll
  for (int r = 0; r < G::RC0; ++r) {
    af[r] = a.w0[r * 64 + lane];
#pragma unroll
    for (int j = 0; j < 4; ++j) bz0[r][j] = a.b0[r * 16 + grp * 4 + j];
  }
  // second conv: the wave's A fragments for every K-step, biases
  h8 a1[G::CT1][G::NS1];
  float bz1[G::CT1][4];
#pragma unroll
  for (int ct = 0; ct < G::CT1; ++ct) {
#pragma unroll
    for (int st = 0; st < G::NS1; ++st) a1[ct][st] = a.w1[(size_t(ct) * a.nalloc1 + st) * 64 + lane];
#pragma unroll
    for (int j = 0; j < 4; ++j) bz1[ct][j] = a.b1[ct * 16 + grp * 4 + j];
  }
  const int fps = (a.Ws + 15) / 16, fpo = (a.Wo + 15) / 16;
  constexpr int FMAX = (SR2 * 10 + NW - 1) / NW;  // second-conv fragments per wave (st_launch checks fpo <= 10)
  for (int g = g_begin; g < g_end; ++g) {
    const int n = g / rows, oy0 = (g - n * rows) * SR2;
    const uint32_t yimg = uint32_t(a.Ho) * uint32_t(a.Wo) * uint32_t(a.ycs);
    const __amdgpu_buffer_rsrc_t yr = out_rsrc(a.y + int64_t(n) * yimg, yimg * 2u);
    const int sy0 = 2 * oy0 - 1;  // first stem row
    // ---------------- input rows (prefetched) -> LDS, the next group's in flight
#pragma unroll
    for (int k = 0; k < NXE; ++k) {
      const int e = tid + k * NT;
      if (e < ne) {
        const int cr = e / CW, q = e - cr * CW;
        *reinterpret_cast<h8*>(IN + cr * WP + q * 8) = xr[k].half8();
      }
    }
    if (g + 1 < g_end) load_in(g + 1);
    stage_barrier();
    // ---------------- stem rows -> S (zero outside the image and in the two pad columns)
    for (int rr = 0; rr < G::NS; ++rr) {
      const int sy = sy0 + rr;
      h8* Srow = S + rr * npos * G::sS;
      if (sy < 0 || sy >= a.Hs) {
        for (int e = tid; e < npos * G::K1; e += NT) Srow[(e / G::K1) * G::sS + e % G::K1] = h8{0, 0, 0, 0, 0, 0, 0, 0};
        continue;
      }
      if (tid < 2 * G::K1) {  // columns -1 and Ws
        const int c = tid / G::K1 ? a.Ws + 1 : 0;
        const int p = (c & 1) ? half + (c >> 1) : (c >> 1);
        Srow[p * G::sS + tid % G::K1] = h8{0, 0, 0, 0, 0, 0, 0, 0};
      }
      for (int fx = wave; fx < fps; fx += NW) {
        const int ox = fx * 16 + col;
        const int base = (2 * rr) * WP + 2 * min(ox, a.Ws - 1) + 7;
        h8 b;
#pragma unroll
        for (int j = 0; j < 8; ++j) b[j] = IN[base + koff[j]];
        const int c = ox + 1, p = (c & 1) ? half + (c >> 1) : (c >> 1);
        _Float16* so = reinterpret_cast<_Float16*>(Srow + p * G::sS);
#pragma unroll
        for (int r = 0; r < G::RC0; ++r) {
          const f4 d = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[r], b, f4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
          if (ox < a.Ws) {
            h4 o;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float t = d[j] + bz0[r][j];
              o[j] = (_Float16)silu(t);
            }
            *reinterpret_cast<h4*>(so + r * 16 + grp * 4) = o;
          }
        }
      }
    }
    stage_barrier();
    // ---------------- the second conv from S -> y
    // A static FMAX fragments per wave (W <= 640: at most 10 per output row), every one issuing its stores (dropped
    // past the map / for a wave's spare fragment): with a runtime trip count the stores were maybe-absent to hipcc's
    // waitcnt pass, and the next group's wait for its input prefetch (issued before them) also waited for them.
#pragma unroll
    for (int i = 0; i < FMAX; ++i) {
      const int f = wave + NW * i;
      const int r1 = f / fpo, fx = f - r1 * fpo;
      const int oy = oy0 + r1;
      const bool wv = f < SR2 * fpo && oy < a.Ho;  // wave-uniform
      const int ox = fx * 16 + col, oxc = min(ox, a.Wo - 1);
      f4 acc[G::CT1];
#pragma unroll
      for (int ct = 0; ct < G::CT1; ++ct) acc[ct] = f4{0.f, 0.f, 0.f, 0.f};
      if (wv) {
#pragma unroll
        for (int st = 0; st < G::NS1; ++st) {
          int tap, cc;
          bool ok;
          if (G::CM) {  // chunk-major: step = (32-channel chunk) * 9 + tap
            tap = st % 9;
            cc = (st / 9) * 4 + grp;
            ok = true;
          } else {  // tap-major 8-channel chunk c = 4 st + grp
            const int c = st * 4 + grp;
            tap = c / G::K1;
            cc = c - tap * G::K1;
            ok = c < 9 * G::K1;
          }
          h8 b = h8{0, 0, 0, 0, 0, 0, 0, 0};
          if (ok) {
            const int ky = tap / 3, kx = tap - ky * 3;
            const int cp = 2 * oxc + kx, p = (cp & 1) ? half + (cp >> 1) : (cp >> 1);
            b = S[((2 * r1 + ky) * npos + p) * G::sS + cc];
          }
#pragma unroll
          for (int ct = 0; ct < G::CT1; ++ct) acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[ct][st], b, acc[ct], 0, 0, 0);
        }
      }
      const bool ok = wv && ox < a.Wo;
      const uint32_t off = uint32_t((oy * a.Wo + ox) * a.ycs + grp * 4) * 2u;
#pragma unroll
      for (int ct = 0; ct < G::CT1; ++ct) {
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = silu(acc[ct][j] + bz1[ct][j]);
        store_h4_or_drop(yr, ok, off + uint32_t(ct * 32), h4_of(v));
      }
    }
    stage_barrier();  // the second conv's reads of S and the stem's of IN before the next group overwrites them
  }
}

// ============================================================================ host
// (c0, c1) instantiated: the n scale's 3 -> 16 -> 32 and the s scale's 3 -> 32 -> 64 (m at 1280 and l's 64-channel
// stem do not fit the LDS tile / the register-resident fragments: their two convs stay separate).
// FCE_STEM2_SR = 1 / 2 output rows per group, FCE_STEM2_NW = 4 / 8 waves: n default 2 rows x 8 waves (n32 pipelined
// bench 38.5k images/s against 38.1k with 1 row / 4 waves and 37.7k unfused, profiles/r05_stem_ab.txt), s 1 x 4 (two
// rows of the 32-channel stem image do not fit 160 KiB; eight waves spill at the 256-register cap).
static constexpr int kStemInsts[][2] = {{16, 32}, {32, 64}};

bool stem_fused_ok(const fce_stem2_desc& d) {
  for (const auto& s : kStemInsts)
    if (s[0] == d.c0 && s[1] == d.c1) return true;
  return false;
}

// the planned input size fits the kernel: the register image of the staged rows is sized for W <= 640 (and the
// LDS tile with it); the executor keeps the two convs otherwise
bool stem_fused_fits(const fce_stem2_desc& d, int h, int w) { return stem_fused_ok(d) && h > 0 && w % 8 == 0 && w <= 640; }

template <typename T, int C0, int C1, int SR2, int NW>
static int st_launch(const Stem2Args& a, hipStream_t s) {
  using G = StG<C0, C1, SR2>;
  constexpr int NXE_MAX = (3 * G::IR * (640 + 16) / 8 + NW * 64 - 1) / (NW * 64);  // register image sized for W <= 640
  const int ne = 3 * G::IR * (a.W + 16) / 8;
  FCE_CHECK(ne <= NXE_MAX * NW * 64, "stem fused: input wider than the prefetch register image (W <= 640)");
  FCE_CHECK((a.Wo + 15) / 16 <= 10, "stem fused: output wider than the per-wave fragment count (W <= 640)");
  const size_t lds = size_t(3) * G::IR * (a.W + 16) * sizeof(_Float16) + size_t(G::NS) * (a.Ws + 2) * G::sS * 16;
  FCE_CHECK(lds <= 160 * 1024, "stem fused: input too wide for the LDS tile");
  auto k = stem_fused_kernel<T, C0, C1, SR2, NW, NXE_MAX>;
  static const bool big = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
  if (!big && lds > 64 * 1024) return fail(FCE_ERR_HIP, "stem fused: cannot opt in to >64 KiB LDS");
  const int64_t groups = int64_t(a.N) * ((a.Ho + SR2 - 1) / SR2);
  FCE_CHECK(groups > 0 && groups < (int64_t(1) << 31), "stem fused: grid size");
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
  }
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k, NW * 64, lds) != hipSuccess || occ < 1) occ = 1;
  const int grid = int(std::min<int64_t>(groups, int64_t(cus) * occ));
  FCE_LAUNCH(k, dim3(unsigned(grid)), dim3(NW * 64), lds, s, a);
  return launch_status("stem_fused_kernel");
}

template <typename T>
static int st_dispatch(const Stem2Args& a, int c0, hipStream_t s) {
  const char* e = getenv("FCE_STEM2_SR");  // read per call: tests switch it
  const char* w = getenv("FCE_STEM2_NW");
  const int sr = e && *e ? atoi(e) : (c0 == 16 ? 2 : 1), nw = w && *w ? atoi(w) : (c0 == 16 ? 8 : 4);
  if (c0 == 16) {
    if (sr == 1 && nw == 4) return st_launch<T, 16, 32, 1, 4>(a, s);
    if (sr == 1 && nw == 8) return st_launch<T, 16, 32, 1, 8>(a, s);
    if (sr == 2 && nw == 4) return st_launch<T, 16, 32, 2, 4>(a, s);
    if (sr == 2 && nw == 8) return st_launch<T, 16, 32, 2, 8>(a, s);
  } else {
    if (sr == 1 && nw == 4) return st_launch<T, 32, 64, 1, 4>(a, s);
    if (sr == 1 && nw == 8) return st_launch<T, 32, 64, 1, 8>(a, s);
  }
  return fail(FCE_ERR_INVALID, "FCE_STEM2_SR / FCE_STEM2_NW: 1 or 2 rows (1 for c0 32), 4 or 8 waves");
}

int stem_fused(const fce_stem2_desc& d, const fce_tensor& x, const fce_tensor& y, hipStream_t s) {
  FCE_CHECK(stem_fused_ok(d), "stem fused: unsupported channel configuration");
  FCE_CHECK(x.layout == FCE_NCHW && x.c == 3 && x.coff == 0 && x.cstride == 3, "stem fused: dense NCHW 3-channel input");
  FCE_CHECK(x.w % 8 == 0 && x.w <= 640, "stem fused: input width a multiple of 8, at most 640");
  FCE_CHECK(y.layout == FCE_NHWC && y.dtype == FCE_F16 && y.c == d.c1 && y.cstride % 4 == 0 && y.coff % 4 == 0,
            "stem fused: NHWC f16 output view");
  Stem2Args a{};
  a.x = x.data;
  a.N = x.n;
  a.H = x.h;
  a.W = x.w;
  a.Hs = (x.h - 1) / 2 + 1;
  a.Ws = (x.w - 1) / 2 + 1;
  a.Ho = (a.Hs - 1) / 2 + 1;
  a.Wo = (a.Ws - 1) / 2 + 1;
  FCE_CHECK(y.n == x.n && y.h == a.Ho && y.w == a.Wo, "stem fused: output size mismatch");
  a.w0 = reinterpret_cast<const h8*>(static_cast<const char*>(d.w[0]) + size_t(3) * 9 * d.c0 * sizeof(float));
  a.b0 = d.b[0];
  a.w1 = static_cast<const h8*>(d.w[1]);
  a.nalloc1 = stage_nalloc(d.c0, 3);
  a.b1 = d.b[1];
  a.y = static_cast<_Float16*>(y.data) + y.coff;
  a.ycs = y.cstride;
  if (x.dtype == FCE_F16) return st_dispatch<_Float16>(a, d.c0, s);
  if (x.dtype == FCE_F32) return st_dispatch<float>(a, d.c0, s);
  if (x.dtype == FCE_U8) return st_dispatch<uint8_t>(a, d.c0, s);
  return fail(FCE_ERR_INVALID, "stem fused: input dtype");
}

}  // namespace fce
