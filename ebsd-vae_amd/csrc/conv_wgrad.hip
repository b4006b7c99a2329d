// Weight / bias gradients of the 3x3 convs (autograd's convolution_backward weight and
// bias outputs for latice/model.py:95,102-104,148), on the fp32 MFMA
// (v_mfma_f32_16x16x4_f32).
//
//   dWc[co][ci][tap] = sum_{b,p} gy[b,p,co] * act(src)[b, p + d(tap), ci]
//   db[co]           = sum_{b,p} gy[b,p,co]
//
// GEMM view: M = co, N = ci, K = pixels (B*H*W, up to 4.2M), one accumulator per tap.
// The K reduction is split over "slices" (contiguous runs of pixel tiles); each block
// writes its slice's partial tile and ebsdvae_wgrad_reduce sums the slices in a fixed
// order -> bitwise reproducible gradients (no float atomics).
//
// Per block: a co tile (32 or 64) x ci tile of 32; 2 or 4 waves, each co32 x ci16 x 9 taps
// = 18 accumulators of 16x16 (72 regs).  Per k-step of 4 pixels: 2 A reads (gy) and 9 B
// reads (shifted activations) feed 18 MFMAs.  LDS tiles: gy [128 px][co] with stride
// CO_T+16 (== 16 mod 32 -> the two 16-lane pixel rows of an A fragment are bank-disjoint),
// activation halo [(TH+2)(TW+2)][32] with stride 48 (same reason).  The activation is
// recomputed from the producer's saved pre-norm output (InstanceNorm + LeakyReLU
// [+ pool/upsample]) while staging, exactly as in the forward.
#include <utility>

#include "common.h"
#include "../../include/ebsdvae.h"

namespace ev {

constexpr int WG_PT = 128;   // pixels per tile
constexpr int WG_AS = 48;    // activation halo channel stride (32 + 16)

struct WgGeom {
  int TH, TW, NI, ntx, nty, tiles, slices, tps, lTW, ltpx;
};

// tile width of the split kernels' 32-channel layers: 16 (4x16 tiles, 108 halo pixels per
// 64) stages 20 % fewer activation pixels than 2x32 (136) and measured 4-5 % faster on the
// 128x128 layers (tools/conv_micro.py wgrad32, wgrad32u); EBSDVAE_WG_TW=32|8 for A/B timing
static int wg_tw_pref() {
  static const int v = [] {
    const char* e = getenv("EBSDVAE_WG_TW");
    const int t = e ? atoi(e) : 16;
    return (t == 8 || t == 32) ? t : 16;
  }();
  return v;
}

// target block count of a weight-gradient launch (slices x co tiles x ci tiles).  Every
// slice writes a full partial dW that the batched reduce re-reads, so fewer, longer slices
// cut that traffic (512 measured 0.2 ms/step faster than 1024; 256 leaves half the CUs'
// block slots empty); EBSDVAE_WG_BLOCKS overrides the split kernels' target (A/B timing)
static int wg_block_target(int pt) {
  static const int v = [] {
    const char* e = getenv("EBSDVAE_WG_BLOCKS");
    const int t = e ? atoi(e) : 512;   // 2 blocks per CU x 256 CUs: one wave of blocks
    return (t >= 64 && t <= 8192) ? t : 512;
  }();
  return pt == 64 ? v : 1024;
}

// pt = pixels per tile (128 for fp32, 64 for the split-bf16 kernels)
static bool wg_geom(int B, int H, int W, int cin, int cout, WgGeom* g, int pt = WG_PT) {
  if (B <= 0 || H <= 0 || W <= 0 || cin <= 0 || cout <= 0) return false;
  const int twmax = pt == 64 && cout == 32 ? wg_tw_pref() : 32;
  g->TW = W < twmax ? W : twmax;
  if (H * g->TW >= pt) {
    g->TH = pt / g->TW;
    g->NI = 1;
  } else {
    g->TH = H;
    g->NI = pt / (H * W);
    if (g->NI * H * W != pt) return false;
  }
  if (W % g->TW || H % g->TH) return false;
  if (g->NI * (g->TH + 2) * (g->TW + 2) > 224) return false;   // KH = 7 halo items / thread
  g->ntx = W / g->TW;
  g->lTW = __builtin_ctz(g->TW);
  g->ltpx = __builtin_ctz(g->TH * g->TW);
  if ((1 << g->lTW) != g->TW || (1 << g->ltpx) != g->TH * g->TW) return false;
  g->nty = H / g->TH;
  const long imgs = (B + g->NI - 1) / g->NI;
  g->tiles = (int)(imgs * g->ntx * g->nty);
  // aim for ~2048 blocks (slices x co tiles x ci tiles), >= 4 tiles per slice
  // 8x8 maps (two-image tiles) use 32-wide co tiles: the 64-wide variant exceeds 256 VGPRs
  const int co_t = cout == 1 ? 1 : (cout == 32 || g->TW == 8 ? cout / 32 : cout / 64);
  const int ci_t = cin == 1 ? 1 : (cout == 1 ? 1 : cin / 32);
  if (co_t <= 0 || ci_t <= 0) return false;
  const int want = wg_block_target(pt) / (co_t * ci_t);
  int tps = 4;
  while ((g->tiles + tps - 1) / tps > (want > 1 ? want : 1)) tps *= 2;
  g->tps = tps;
  g->slices = (g->tiles + tps - 1) / tps;
  return true;
}

// the pipelined two-piece kernel (wgrad_pipe_kernel) on 8x8 tiles; EBSDVAE_WG_PIPE=0 selects
// wgrad_split_kernel instead (A/B timing)
static bool wg_pipe() {
  static const bool v = [] {
    const char* e = getenv("EBSDVAE_WG_PIPE");
    return !(e && e[0] == '0');
  }();
  return v;
}
// output channels per block of the pipelined kernel: 32 (cout 32), 128 (8-wave blocks, one per
// CU, for cout % 128 == 0) or 64 (cout 64; every cout % 64 == 0 with EBSDVAE_WG_CO128=0).  Alone
// the wide blocks stage 1.28x fewer elements per FLOP and run 7-8 % faster (128->128 @32 232 ->
// 215 us, 64->128 @32 116 -> 107 us).  In round 2's step they were ~0.1 ms slower (a 112-KB
// block owns its CU and crowded out the input-gradient chain beside it); with round 3's
// schedule (kernel-attached forks, fused network end) the step is 0.07 ms faster with them
// (two pairs, same box), so they are the default.
static int wg_pipe_cot(int cout) {
  static const bool wide = [] {
    const char* e = getenv("EBSDVAE_WG_CO128");
    return !(e && e[0] == '0');
  }();
  return cout == 32 ? 32 : ((wide && cout % 128 == 0) ? 128 : 64);
}
// input channels per block of the pipelined kernel: 64 for co 64 blocks where cin % 64 == 0
// (co 64 x ci 64, 8 waves: gy is read once per layer instead of twice; 64->64 @64 236 -> 221 us,
// round 5), else 32.  A co 128 x ci 64 block (waves of co 64 x ci 16) needs 144 accumulator
// VGPRs and spilled 132-208 B per lane: 2x slower (wgrad128 195 -> 400 us), not used.
// EBSDVAE_WG_CI64=0: always 32 (A/B); =2 also the co 128 x ci 64 blocks (experiment)
static int wg_pipe_ci64_mode() {
  static const int v = [] {
    const char* e = getenv("EBSDVAE_WG_CI64");
    return e ? atoi(e) : 1;
  }();
  return v;
}
static int wg_pipe_cit(int cin, int cout) {
  const int m = wg_pipe_ci64_mode();
  if (m <= 0 || cout == 32 || cin % 64) return 32;
  return (m >= 2 || wg_pipe_cot(cout) == 64) ? 64 : 32;
}
static bool wg_pipe_geom(int B, int H, int W, int cin, int cout, WgGeom* g) {
  if (B <= 0 || H <= 0 || W <= 0 || cin <= 0 || cout <= 0) return false;
  if (H % 8 || W % 8 || cin % 32 || !(cout == 32 || cout % 64 == 0)) return false;
  if (((H / 8) & (H / 8 - 1)) || ((W / 8) & (W / 8 - 1))) return false;   // tile_at shifts
  // per-image byte ranges of the source / gradient buffer descriptors: 32-bit
  if (!ev_buf_bytes_ok(4LL * H * W * (cin > cout ? cin : cout) * 4)) return false;
  g->TW = 8; g->TH = 8; g->NI = 1;
  g->ntx = W / 8; g->nty = H / 8;
  g->lTW = 3; g->ltpx = 6;
  g->tiles = (int)((long)B * g->ntx * g->nty);
  const int cot = wg_pipe_cot(cout), cit = wg_pipe_cit(cin, cout);
  const int co_t = cout == 32 ? 1 : cout / cot;
  // 8-wave blocks fill a CU alone: half the block target keeps one wave of blocks
  const bool eight = cot == 128 || cit == 64;
  const int want = wg_block_target(64) / (eight ? 2 : 1) / (co_t * (cin / cit));
  int tps = 4;
  while ((g->tiles + tps - 1) / tps > (want > 1 ? want : 1)) tps *= 2;
  g->tps = tps;
  g->slices = (g->tiles + tps - 1) / tps;
  return true;
}

// 1-D grid of wgrad_pipe_kernel: 8 x ceil(slices / 8) x (co tiles x ci tiles) blocks
static dim3 wg_pipe_grid(const WgGeom& g, int cin, int cout) {
  const int nm = (cout == 32 ? 1 : cout / wg_pipe_cot(cout)) * (cin / wg_pipe_cit(cin, cout));
  return dim3(8 * ((g.slices + 7) / 8) * nm);
}

EV_DEVINL void tile_origin(int t, const WgGeom& g, int& b0, int& y0, int& x0) {
  const int per_img = g.ntx * g.nty;
  const int ib = t / per_img, r = t - ib * per_img;
  b0 = ib * g.NI;
  y0 = (r / g.ntx) * g.TH;
  x0 = (r % g.ntx) * g.TW;
}

// ------------------------------------------------------------------ generic (cin % 32 == 0)
// Tile geometry is a compile-time function of TW (the tile width, min(W, 32)): 128 pixels
// as 4x32, 8x16 or 2 images of 8x8.  With it, and the k-step loop fully unrolled, every
// LDS operand address is a per-lane base register plus an immediate offset.
template <int TW>
struct WgTile {
  static constexpr int TH = TW == 32 ? 4 : 8;
  static constexpr int NI = TW == 8 ? 2 : 1;
  static constexpr int HP = TH + 2, WP = TW + 2;
  static constexpr int HALO = NI * HP * WP;   // 204 / 180 / 200 pixels
  static constexpr int IPX = TH * TW;         // pixels per image in the tile
  static_assert(NI * IPX == WG_PT, "128-pixel tiles");
  static_assert(HALO * 8 <= 7 * 256, "7 halo float4 items per thread");
};

// Software-pipelined over the slice's pixel tiles: the NEXT tile's gy rows and raw
// activation halo (+ its InstanceNorm stats) are loaded into registers while the MFMAs of
// the current tile run; the transform (InstanceNorm + LeakyReLU [+ upsample]) is applied
// when they are written to LDS.  The bias gradient is summed from the same gy registers.
// MODE is never NORM_POOL here: pool-fed layers pass the pooled activation that their
// forward conv materialised (RAW).
template <int NWCO, int KSPLIT, int MODE, int TW>
__global__ __launch_bounds__(256, 2) void wgrad_kernel(
    const float* __restrict__ src, const float2* __restrict__ sstats,
    const float* __restrict__ gy, float* __restrict__ wpart, float* __restrict__ bpart, int B,
    int H, int W, int Cin, int Cout, WgGeom g) {
  using T = WgTile<TW>;
  constexpr int CO_T = NWCO * 32;
  constexpr int GS = CO_T + 16;
  constexpr int QG = CO_T / 4;      // float4 channel groups of a gy pixel
  constexpr int KG = CO_T / 8;      // gy float4 items per thread per tile
  constexpr int KH = 7;             // halo float4 items per thread per tile (upper bound)
  constexpr bool NORM = (MODE == ACT_NORM || MODE == ACT_NORM_UP);
  constexpr bool UPS = (MODE == ACT_UP || MODE == ACT_NORM_UP);
  static_assert(NWCO * 2 * KSPLIT == 4, "4 waves per block");
  static_assert(MODE != ACT_NORM_POOL, "pool-fed layers use the materialised activation");
  constexpr int SPR = TW / (4 * KSPLIT);        // k-steps per tile row
  constexpr int ROW_UNROLL = 1;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* lg = smem;                 // [128][GS]
  float* la = smem + WG_PT * GS;    // [halo px][48]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wco = wave % NWCO, wci = (wave / NWCO) & 1, wk = wave / (2 * NWCO);
  const int slice = blockIdx.x, co0 = blockIdx.y * CO_T, ci0 = blockIdx.z * 32;
  const int l16 = lane & 15, kq = lane >> 4;
  const int Hs = UPS ? H / 2 : H, Ws = UPS ? W / 2 : W;
  const int qh = tid & 7;           // this thread's 4-channel group of every halo pixel
  const int qg = tid % QG;          // this thread's 4-channel group of every gy pixel
  const bool do_bias = blockIdx.z == 0;

  f32x4 acc[2][9];
#pragma unroll
  for (int f = 0; f < 2; ++f)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[f][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  double bs[4] = {0.0, 0.0, 0.0, 0.0};   // bias partial of channels co0 + 4*qg + 0..3

  const int per_img = g.ntx * g.nty;
  const int t_beg = slice * g.tps;
  const int t_end = min(t_beg + g.tps, g.tiles);
  float4 rg[KG], rh[KH];
  float2 st[T::NI][4];
  int cb0 = 0, cy0 = 0, cx0 = 0;   // origin of the tile held in registers
  auto load_stats = [&](int b0) {
#pragma unroll
    for (int i = 0; i < T::NI; ++i) {
      const int gb = min(b0 + i, B - 1);
      const float2* sp = sstats + (size_t)gb * Cin + ci0 + qh * 4;
      st[i][0] = sp[0]; st[i][1] = sp[1]; st[i][2] = sp[2]; st[i][3] = sp[3];
    }
  };
  auto issue = [&](int t) {
    const int ib = t / per_img, rr = t - ib * per_img;
    const int ty = rr / g.ntx;
    const int b0 = ib * T::NI, y0 = ty * T::TH, x0 = (rr - ty * g.ntx) * TW;
    cb0 = b0; cy0 = y0; cx0 = x0;
#pragma unroll
    for (int k = 0; k < KG; ++k) {
      const int px = (tid + 256 * k) / QG;
      const int img = px / T::IPX, rem = px % T::IPX;
      const int r = rem / TW, c = rem % TW;
      const int gb = b0 + img;
#ifdef EV_WG_NOLOAD   // timing experiment only (wrong results)
      rg[k] = make_float4((float)r, (float)c, 1.f, 0.f);
#else
      if (T::NI == 1 || gb < B)
        rg[k] = ld4(gy + (((size_t)gb * H + y0 + r) * W + x0 + c) * Cout + co0 + qg * 4);
#endif
    }
#pragma unroll
    for (int k = 0; k < KH; ++k) {
      const int pix = (tid + 256 * k) >> 3;
      const int img = pix / (T::HP * T::WP), rem = pix % (T::HP * T::WP);
      const int hh = rem / T::WP, ww = rem % T::WP;
      const int gh = y0 + hh - 1, gw = x0 + ww - 1, gb = b0 + img;
      if (pix < T::HALO && gb < B && gh >= 0 && gh < H && gw >= 0 && gw < W) {
        const int sh = UPS ? (gh >> 1) : gh, sw = UPS ? (gw >> 1) : gw;
#ifdef EV_WG_NOLOAD
        rh[k] = make_float4((float)sh, (float)sw, 1.f, 0.f);
#else
        rh[k] = ld4(src + (((size_t)gb * Hs + sh) * Ws + sw) * Cin + ci0 + qh * 4);
#endif
      }
    }
    if (NORM && T::NI == 1) load_stats(b0);
  };
  auto store = [&]() {
    // two-image tiles fetch their stats here (L2-resident) to stay within 256 VGPRs
    if (NORM && T::NI > 1) load_stats(cb0);
    float4 tb = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int k = 0; k < KG; ++k) {
      const int px = (tid + 256 * k) / QG;
      float4 v = rg[k];
      if (T::NI > 1 && cb0 + px / T::IPX >= B) v = make_float4(0.f, 0.f, 0.f, 0.f);
      tb.x += v.x; tb.y += v.y; tb.z += v.z; tb.w += v.w;
      st4(lg + px * GS + qg * 4, v);
    }
    bs[0] += (double)tb.x; bs[1] += (double)tb.y; bs[2] += (double)tb.z; bs[3] += (double)tb.w;
#pragma unroll
    for (int k = 0; k < KH; ++k) {
      const int pix = (tid + 256 * k) >> 3;
      if (pix < T::HALO) {
        const int img = pix / (T::HP * T::WP), rem = pix % (T::HP * T::WP);
        const int hh = rem / T::WP, ww = rem % T::WP;
        const int gh = cy0 + hh - 1, gw = cx0 + ww - 1, gb = cb0 + img;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (gb < B && gh >= 0 && gh < H && gw >= 0 && gw < W) {
          v = rh[k];
          if (NORM) {
            const bool second = T::NI > 1 && img > 0;
            v = make_float4(normact(v.x, second ? st[T::NI - 1][0] : st[0][0]),
                            normact(v.y, second ? st[T::NI - 1][1] : st[0][1]),
                            normact(v.z, second ? st[T::NI - 1][2] : st[0][2]),
                            normact(v.w, second ? st[T::NI - 1][3] : st[0][3]));
          }
        }
        st4(la + pix * WG_AS + qh * 4, v);
      }
    }
  };

  // per-lane operand bases; the k-step's own offset is a compile-time immediate
  const float* aP = lg + (kq + 4 * wk) * GS + wco * 32 + l16;
  const float* bP = la + (kq + 4 * wk) * WG_AS + wci * 16 + l16;

  if (t_beg < t_end) issue(t_beg);
  for (int t = t_beg; t < t_end; ++t) {
    __syncthreads();
    store();
    __syncthreads();
    if (t + 1 < t_end) issue(t + 1);
    // one iteration per tile row: its k-steps are unrolled with immediate offsets
#pragma unroll ROW_UNROLL
    for (int row = 0; row < T::NI * T::TH; ++row) {
      const int img = row / T::TH, r = row % T::TH;
      const float* ap = aP + row * TW * GS;
      const float* bp = bP + (img * T::HP + r) * T::WP * WG_AS;
#pragma unroll
      for (int jj = 0; jj < SPR; ++jj) {
        const int c = 4 * KSPLIT * jj;
        const float a0 = ap[c * GS];
        const float a1 = ap[c * GS + 16];
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
          const float bv = bp[(c + (tap / 3) * T::WP + tap % 3) * WG_AS];
          acc[0][tap] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, bv, acc[0][tap], 0, 0, 0);
          acc[1][tap] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, bv, acc[1][tap], 0, 0, 0);
        }
      }
    }
  }
  __syncthreads();
  if (KSPLIT == 2) {   // fold the second K half into the first through LDS
    float* xs = smem + (size_t)(wave - 2 * NWCO) * 72 * 64;
    if (wk == 1) {
#pragma unroll
      for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int tap = 0; tap < 9; ++tap)
#pragma unroll
          for (int r = 0; r < 4; ++r) xs[((f * 9 + tap) * 4 + r) * 64 + lane] = acc[f][tap][r];
    }
    __syncthreads();
    if (wk == 0) {
      xs = smem + (size_t)wave * 72 * 64;
#pragma unroll
      for (int f = 0; f < 2; ++f)
#pragma unroll
        for (int tap = 0; tap < 9; ++tap)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[f][tap][r] += xs[((f * 9 + tap) * 4 + r) * 64 + lane];
    }
    __syncthreads();
  }
  // partial layout [slice][tap][co][ci]
  const int ci = ci0 + wci * 16 + l16;
  if (wk == 0) {
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int tap = 0; tap < 9; ++tap)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int co = co0 + wco * 32 + f * 16 + kq * 4 + r;
          wpart[(((size_t)slice * 9 + tap) * Cout + co) * Cin + ci] = acc[f][tap][r];
        }
  }
  if (do_bias) {   // threads sharing a channel group fold their sums in a fixed order
    double* xb = reinterpret_cast<double*>(smem);
#pragma unroll
    for (int i = 0; i < 4; ++i) xb[i * 256 + tid] = bs[i];
    __syncthreads();
    if (tid < CO_T) {
      const int q = tid >> 2, i = tid & 3;
      double sum = 0.0;
      for (int m = q; m < 256; m += QG) sum += xb[i * 256 + m];
      bpart[(size_t)slice * Cout + co0 + tid] = (float)sum;
    }
  }
}

// ------------------------------------------------------------------ split-bf16 (NP pieces)
// Same blocking, slices and register prefetch as wgrad_kernel, on v_mfma_f32_16x16x32_bf16
// with every operand split into NP bf16 pieces (products of total order < NP, see
// conv_split.hip).  K = pixels: both operands are staged pixel-major (NHWC, as loaded) in
// per-piece LDS images and read k-major with the hardware transpose read
// ds_read_b64_tr_b16 (lane 4q+p of a 16-lane group addresses row q, columns 4p..4p+3 and
// receives one column of the 4 rows).  Element j of a lane group g's fragment is pixel
//     32 s + (j < 4 ? 4g + j : 16 + 4g + j - 4)
// of the tile, which with row strides of 160 / 96 B keeps every transposed read
// conflict-free; the tap shift is a per-lane row offset into the activation halo, so any
// shift stays 8-byte aligned.
template <int TW, int PT>
struct WgTileP {
  static constexpr int TH = PT == 128 ? (TW == 32 ? 4 : 8) : (TW == 32 ? 2 : (TW == 16 ? 4 : 8));
  static constexpr int NI = (PT == 128 && TW == 8) ? 2 : 1;
  static constexpr int HP = TH + 2, WP = TW + 2;
  static constexpr int HALO = NI * HP * WP;
  static constexpr int IPX = TH * TW;
  static_assert(NI * IPX == PT, "tile pixels");
};

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8w __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4* lds_s16x4_ptr;

EV_DEVINL bf16x8w tr_frag(const char* r0, const char* r1) {
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_ptr)(r0));
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_ptr)(r1));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8w, v);
}

template <int NP>
EV_DEVINL void store_pieces(char* base, size_t piece_stride, float4 v) {
  typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
  if constexpr (NP == NP_F16) {   // fp16 bit patterns in the 16-bit piece slots
    unsigned h01, l01, h23, l23;
    split_f16x2(v.x, v.y, h01, l01);
    split_f16x2(v.z, v.w, h23, l23);
    typedef unsigned u2 __attribute__((ext_vector_type(2)));
    *reinterpret_cast<u2*>(base) = u2{h01, h23};
    *reinterpret_cast<u2*>(base + piece_stride) = u2{l01, l23};
    return;
  }
  const float e[4] = {v.x, v.y, v.z, v.w};
  constexpr int NPC = npc(NP);
  bf4 pc[NPC];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if constexpr (NP == NP_F16) {   // fp16 bit patterns in the 16-bit piece slots
      const _Float16 h0 = (_Float16)e[c];
      const _Float16 h1 = (_Float16)(e[c] - (float)h0);
      pc[0][c] = __builtin_bit_cast(__bf16, h0);
      pc[1][c] = __builtin_bit_cast(__bf16, h1);
    } else {
      float r = e[c];
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const __bf16 h = (__bf16)r;
        pc[i][c] = h;
        r -= (float)h;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NPC; ++i) *reinterpret_cast<bf4*>(base + i * piece_stride) = pc[i];
}

template <int NP>
EV_DEVINL f32x4 mfma16_piece(bf16x8w a, bf16x8w b, f32x4 c) {
  if constexpr (NP == NP_F16)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

constexpr int WGS_ASB = 96;   // activation image row stride (32 ch x 2 B + 32 B)

// End of a split weight-gradient block (both kernels below): fold the second K half into
// the first through LDS (KSPLIT 2), store the slice's partial dW tile [slice][tap][co][ci]
// (16x16 C/D: col = ci = lane & 15, row = co) with the gradient scale undone, and the bias
// partial from the per-thread gy sums (ci tile 0 only).  LDS is free on entry.
// FCO = 16-co fragments per wave (co tile of a wave 16 FCO), NWCI = ci-waves of 16 channels
// (block ci tile 16 NWCI); the defaults are the co 32 x ci 16 waves of 32-channel ci tiles.
template <int NWCO, int KSPLIT, bool F16, int FCO = 2, int NWCI = 2>
EV_DEVINL void wgrad_split_finish(f32x4 (&acc)[FCO][9], const double (&bs)[4], char* wsm,
                                  float* __restrict__ wpart, float* __restrict__ bpart, int slice,
                                  int co0, int ci0, int Cin, int Cout, float gsc, bool do_bias) {
  constexpr int CO_T = NWCO * 16 * FCO;
  constexpr int QG = CO_T / 4;
  constexpr int NTH = NWCO * NWCI * KSPLIT * 64;   // threads per block
  constexpr int NACC = FCO * 9 * 4;                // accumulator floats per lane
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wco = wave % NWCO, wci = (wave / NWCO) % NWCI, wk = wave / (NWCI * NWCO);
  if (KSPLIT == 2) {
    float* xs = reinterpret_cast<float*>(wsm) + (size_t)(wave - NWCI * NWCO) * NACC * 64;
    if (wk == 1) {
#pragma unroll
      for (int f = 0; f < FCO; ++f)
#pragma unroll
        for (int tap = 0; tap < 9; ++tap)
#pragma unroll
          for (int r = 0; r < 4; ++r) xs[((f * 9 + tap) * 4 + r) * 64 + lane] = acc[f][tap][r];
    }
    __syncthreads();
    if (wk == 0) {
      xs = reinterpret_cast<float*>(wsm) + (size_t)wave * NACC * 64;
#pragma unroll
      for (int f = 0; f < FCO; ++f)
#pragma unroll
        for (int tap = 0; tap < 9; ++tap)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[f][tap][r] += xs[((f * 9 + tap) * 4 + r) * 64 + lane];
    }
    __syncthreads();
  }
  const int ci = ci0 + wci * 16 + (lane & 15);
  if (wk == 0) {
#pragma unroll
    for (int f = 0; f < FCO; ++f)
#pragma unroll
      for (int tap = 0; tap < 9; ++tap)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int co = co0 + wco * 16 * FCO + f * 16 + (lane >> 4) * 4 + r;
          // the slice partials are read once, by the batched reduction: non-temporal
          __builtin_nontemporal_store(F16 ? acc[f][tap][r] * (1.f / gsc) : acc[f][tap][r],
                                      wpart + (((size_t)slice * 9 + tap) * Cout + co) * Cin + ci);
        }
  }
  if (do_bias) {
    double* xb = reinterpret_cast<double*>(wsm);
#pragma unroll
    for (int i = 0; i < 4; ++i) xb[i * NTH + tid] = bs[i];
    __syncthreads();
    if (tid < CO_T) {
      const int qq = tid >> 2, i = tid & 3;
      double sum = 0.0;
      for (int m = qq; m < NTH; m += QG) sum += xb[i * NTH + m];
      bpart[(size_t)slice * Cout + co0 + tid] = (float)sum;
    }
  }
}

template <int NP, int NWCO, int KSPLIT, int MODE, int TW, int PT>
__global__ __launch_bounds__(256, 2) void wgrad_split_kernel(
    const float* __restrict__ src, const float2* __restrict__ sstats,
    const float* __restrict__ gy, float* __restrict__ wpart, float* __restrict__ bpart, int B,
    int H, int W, int Cin, int Cout, WgGeom g, const float* __restrict__ gmax, int gmT) {
  using T = WgTileP<TW, PT>;
  constexpr int NPC = npc(NP);
  constexpr bool F16 = NP == NP_F16;
  constexpr int CO_T = NWCO * 32;
  constexpr int GSB = CO_T * 2 + 32;      // gy image row stride (bytes)
  constexpr int QG = CO_T / 4;
  constexpr int KG = PT * CO_T / 4 / 256; // gy float4 items per thread per tile
  constexpr int KH = (T::HALO * 8 + 255) / 256;
  constexpr int KSTEPS = PT / 32;
  constexpr size_t GY_PIECE = (size_t)PT * GSB;
  constexpr size_t ACT_PIECE = (size_t)T::HALO * WGS_ASB;
  constexpr bool NORM = (MODE == ACT_NORM || MODE == ACT_NORM_UP);
  constexpr bool UPS = (MODE == ACT_UP || MODE == ACT_NORM_UP);
  static_assert(NWCO * 2 * KSPLIT == 4, "4 waves per block");
  static_assert(KG >= 1, "gy items");
  static_assert(MODE != ACT_NORM_POOL, "pool-fed layers use the materialised activation");
  extern __shared__ __attribute__((aligned(16))) char wsm[];
  char* gimg = wsm;                         // [NP][PT][GSB]
  char* aimg = wsm + NPC * GY_PIECE;        // [NP][HALO][96]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wco = wave % NWCO, wci = (wave / NWCO) & 1, wk = wave / (2 * NWCO);
  const int slice = blockIdx.x, co0 = blockIdx.y * CO_T, ci0 = blockIdx.z * 32;
  const int Hs = UPS ? H / 2 : H, Ws = UPS ? W / 2 : W;
  const int qh = tid & 7;
  const int qg = tid % QG;
  const bool do_bias = blockIdx.z == 0;

  f32x4 acc[2][9];
#pragma unroll
  for (int f = 0; f < 2; ++f)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[f][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  double bs[4] = {0.0, 0.0, 0.0, 0.0};

  const int per_img = g.ntx * g.nty;
  const int t_beg = slice * g.tps;
  const int t_end = min(t_beg + g.tps, g.tiles);
  // F16: the slice's gy is scaled by 2^k from the maximum over the images it covers
  // (a common scale: the accumulators sum over all of them), undone at the partial store
  int gshift = 0;
  if constexpr (F16) {
    static_assert(T::NI == 1, "one image per tile");
    if (t_beg < t_end) gshift = f16_gshift(gmax, gmT, t_beg / per_img, (t_end - 1) / per_img);
  }
  const float gsc = ldexpf(1.f, gshift);
  float4 rg[KG], rh[KH];
  float2 st[T::NI][4];
  int cb0 = 0, cy0 = 0, cx0 = 0;
  auto load_stats = [&](int b0) {
#pragma unroll
    for (int i = 0; i < T::NI; ++i) {
      const int gb = min(b0 + i, B - 1);
      const float2* sp = sstats + (size_t)gb * Cin + ci0 + qh * 4;
      st[i][0] = sp[0]; st[i][1] = sp[1]; st[i][2] = sp[2]; st[i][3] = sp[3];
    }
  };
  auto issue = [&](int t) {
    const int ib = t / per_img, rr = t - ib * per_img;
    const int ty = rr / g.ntx;
    const int b0 = ib * T::NI, y0 = ty * T::TH, x0 = (rr - ty * g.ntx) * TW;
    cb0 = b0; cy0 = y0; cx0 = x0;
#pragma unroll
    for (int k = 0; k < KG; ++k) {
      const int px = (tid + 256 * k) / QG;
      const int img = px / T::IPX, rem = px % T::IPX;
      const int r = rem / TW, c = rem % TW;
      const int gb = b0 + img;
#ifdef EV_WG_NOLOAD   // timing experiment only (wrong results)
      rg[k] = make_float4((float)r, (float)c, 1.f, 0.f);
#else
      if (T::NI == 1 || gb < B)
        rg[k] = ld4(gy + (((size_t)gb * H + y0 + r) * W + x0 + c) * Cout + co0 + qg * 4);
#endif
    }
#pragma unroll
    for (int k = 0; k < KH; ++k) {
      const int pix = (tid + 256 * k) >> 3;
      const int img = pix / (T::HP * T::WP), rem = pix % (T::HP * T::WP);
      const int hh = rem / T::WP, ww = rem % T::WP;
      const int gh = y0 + hh - 1, gw = x0 + ww - 1, gb = b0 + img;
      if (pix < T::HALO && gb < B && gh >= 0 && gh < H && gw >= 0 && gw < W) {
        const int sh = UPS ? (gh >> 1) : gh, sw = UPS ? (gw >> 1) : gw;
#ifdef EV_WG_NOLOAD
        rh[k] = make_float4((float)sh, (float)sw, 1.f, 0.f);
#else
        rh[k] = ld4(src + (((size_t)gb * Hs + sh) * Ws + sw) * Cin + ci0 + qh * 4);
#endif
      }
    }
    if (NORM && T::NI == 1) load_stats(b0);
  };
  auto store = [&]() {
    if (NORM && T::NI > 1) load_stats(cb0);
    float4 tb = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int k = 0; k < KG; ++k) {
      const int px = (tid + 256 * k) / QG;
      float4 v = rg[k];
      if (T::NI > 1 && cb0 + px / T::IPX >= B) v = make_float4(0.f, 0.f, 0.f, 0.f);
      tb.x += v.x; tb.y += v.y; tb.z += v.z; tb.w += v.w;
      if constexpr (F16) v = make_float4(v.x * gsc, v.y * gsc, v.z * gsc, v.w * gsc);
      store_pieces<NP>(gimg + px * GSB + qg * 8, GY_PIECE, v);
    }
    bs[0] += (double)tb.x; bs[1] += (double)tb.y; bs[2] += (double)tb.z; bs[3] += (double)tb.w;
#pragma unroll
    for (int k = 0; k < KH; ++k) {
      const int pix = (tid + 256 * k) >> 3;
      if (pix < T::HALO) {
        const int img = pix / (T::HP * T::WP), rem = pix % (T::HP * T::WP);
        const int hh = rem / T::WP, ww = rem % T::WP;
        const int gh = cy0 + hh - 1, gw = cx0 + ww - 1, gb = cb0 + img;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (gb < B && gh >= 0 && gh < H && gw >= 0 && gw < W) {
          v = rh[k];
          if (NORM) {
            const bool second = T::NI > 1 && img > 0;
            v = make_float4(normact(v.x, second ? st[T::NI - 1][0] : st[0][0]),
                            normact(v.y, second ? st[T::NI - 1][1] : st[0][1]),
                            normact(v.z, second ? st[T::NI - 1][2] : st[0][2]),
                            normact(v.w, second ? st[T::NI - 1][3] : st[0][3]));
          }
        }
        store_pieces<NP>(aimg + pix * WGS_ASB + qh * 8, ACT_PIECE, v);
      }
    }
  };

  // per-lane transposed-read geometry: lane 4q+p of group gq addresses row q, columns 4p..
  const int gq = lane >> 4, i16 = lane & 15, q = i16 >> 2, p4 = i16 & 3;
  const int acol = (wco * 32 + 4 * p4) * 2;          // gy image column bytes (+ f*32)
  const int bcol = (wci * 16 + 4 * p4) * 2;          // act image column bytes

  if (t_beg < t_end) issue(t_beg);
  for (int t = t_beg; t < t_end; ++t) {
    __syncthreads();
#ifndef EV_WG_NOSTORE   // timing experiment only: no staging (and so no loads; wrong results)
    store();
#endif
    __syncthreads();
    if (t + 1 < t_end) issue(t + 1);
#pragma unroll
    for (int s = wk; s < KSTEPS; s += KSPLIT) {
      const int px0 = 32 * s + 4 * gq + q, px1 = px0 + 16;   // rows of read 0 / read 1
      bf16x8w a[NPC][2];
#pragma unroll
      for (int i = 0; i < NPC; ++i)
#pragma unroll
        for (int f = 0; f < 2; ++f)
          a[i][f] = tr_frag(gimg + i * GY_PIECE + px0 * GSB + acol + f * 32,
                            gimg + i * GY_PIECE + px1 * GSB + acol + f * 32);
      int hp0, hp1;
      {
        const int im0 = px0 / T::IPX, rm0 = px0 % T::IPX;
        const int im1 = px1 / T::IPX, rm1 = px1 % T::IPX;
        hp0 = (im0 * T::HP + rm0 / TW) * T::WP + rm0 % TW;
        hp1 = (im1 * T::HP + rm1 / TW) * T::WP + rm1 % TW;
      }
      bf16x8w b[NPC];
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int toff = (tap / 3) * T::WP + tap % 3;
#ifdef EV_WG_ONEB   // timing experiment only: one activation fragment per k-step (wrong results)
        if (tap == 0)
#endif
#pragma unroll
        for (int i = 0; i < NPC; ++i)
          b[i] = tr_frag(aimg + i * ACT_PIECE + (hp0 + toff) * WGS_ASB + bcol,
                         aimg + i * ACT_PIECE + (hp1 + toff) * WGS_ASB + bcol);
#ifdef EV_WG_NOMFMA   // timing experiment only (wrong results)
#pragma unroll
        for (int f = 0; f < 2; ++f)
#pragma unroll
          for (int i = 0; i < NPC; ++i) acc[f][tap][i & 3] += (float)a[i][f][0] * (float)b[i][1];
        if (false)
#endif
#pragma unroll
        for (int f = 0; f < 2; ++f) {
          f32x4 c = acc[f][tap];
          if constexpr (NP == 3) {
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][f], b[1], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[NP - 1][f], b[0], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][f], b[NP - 1], c, 0, 0, 0);
          }
          c = mfma16_piece<NP>(a[1][f], b[0], c);
          c = mfma16_piece<NP>(a[0][f], b[1], c);
          c = mfma16_piece<NP>(a[0][f], b[0], c);
          acc[f][tap] = c;
        }
      }
    }
  }
  __syncthreads();
  wgrad_split_finish<NWCO, KSPLIT, F16>(acc, bs, wsm, wpart, bpart, slice, co0, ci0, Cin, Cout, gsc,
                                        do_bias);
}

// f(integral_constant<int, 0>()), ..., f(integral_constant<int, N-1>()): compile-time indices
// for register arrays and slot tests inside fully unrolled loops
template <class F, int... I>
EV_DEVINL void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>()), ...);
}
template <int N, class F>
EV_DEVINL void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>());
}

// ------------------------------------------------------------------ pipelined split-fp16
// wgrad_split_kernel's operand images, transposed reads and MFMA sequence on 8x8 pixel tiles
// (100 halo pixels per 64, the fewest staged of the 64-pixel shapes), software-pipelined
// over the slice's tiles with two LDS image sets: while the k-steps of tile t read one set,
// tile t+1 is transformed, split and written into the other item by item BETWEEN the taps,
// and each item's register is refilled with tile t+2's load as soon as it has been staged
// (a whole tile of MFMA work covers every load).  One barrier per tile.  The serial kernel
// spends most of its time there: without its staging it runs 2.3-2.7x faster, without its
// loads 1.3x (tools/micro_variants.sh, EV_WG_NOSTORE / EV_WG_NOLOAD).
// NWCO = 4 (co 128 x ci 32, 8 waves, one block per CU by LDS): the activation halo of a tile
// is staged once per 128 output channels instead of once per 64 (EBSDVAE_WG_CO128).
// NWCI = 4 (ci tile 64; round 5): with FCO = 4 (waves of co 64 x ci 16, 144 accumulator
// registers) a co 128 x ci 64 block stages 0.64x the values per MAC of co 128 x ci 32 and reads
// each B fragment for twice the MFMAs; with FCO = 2 a co 64 x ci 64 block reads gy once per
// layer instead of twice (EBSDVAE_WG_CI64=0: the ci 32 blocks, A/B)
// Staging-store order of the 8-B piece stores (ds_write_b64: 4 groups of 16 contiguous lanes,
// banks (a/4) mod 32).  With 8 float4 items per pixel (32-channel images, 96-B rows) a group
// stores two pixels, and consecutive pixels (rows 24 dwords apart) overlap in 8 banks: 2-way on
// every store.  Swapping bits 0 and 1 of the pixel rank gives each group the pixels p, p + 2
// (48 dwords apart = 16 mod 32): conflict-free.  Wider images store one pixel per group.
template <int Q>
EV_DEVINL int wg_store_perm(int r) {
  if constexpr (Q == 8) return (r & ~3) | ((r >> 1) & 1) | ((r & 1) << 1);
  return r;
}

template <int NP, int NWCO, int KSPLIT, int MODE, int NWCI = 2, int FCO = 2>
__global__ __launch_bounds__(NWCO * NWCI * KSPLIT * 64, NWCO * NWCI * KSPLIT >= 8 ? 1 : 2) void wgrad_pipe_kernel(
    const float* __restrict__ src, const float2* __restrict__ sstats,
    const float* __restrict__ gy, float* __restrict__ wpart, float* __restrict__ bpart, int B,
    int H, int W, int Cin, int Cout, WgGeom g, const float* __restrict__ gmax, int gmT) {
  constexpr int TW = 8, PT = 64;
  using T = WgTileP<TW, PT>;               // one image, 8x8 pixels, 10x10 halo
  constexpr int NPC = npc(NP);
  constexpr bool F16 = NP == NP_F16;
  constexpr int CO_T = NWCO * 16 * FCO;
  constexpr int CI_T = NWCI * 16;
  constexpr int GSB = CO_T * 2 + 32;       // gy image row stride (bytes)
  constexpr int ASB = CI_T * 2 + 32;       // activation image row stride: 96 / 160 B
  constexpr int QG = CO_T / 4;
  constexpr int QH = CI_T / 4;             // float4 channel groups of a halo pixel
  constexpr int NTH = NWCO * NWCI * KSPLIT * 64;   // threads per block
  constexpr int KG = PT * CO_T / 4 / NTH;  // gy float4 items per thread per tile
  constexpr int KH = (T::HALO * QH + NTH - 1) / NTH;
  constexpr int NIT = KG + KH;
  constexpr int KSTEPS = PT / 32;
  constexpr int NSLOT = (KSTEPS / KSPLIT) * 9;   // (k-step, tap) slots per wave and tile
  constexpr int GY_PIECE = PT * GSB;
  constexpr int ACT_PIECE = T::HALO * ASB;
  constexpr int BUF = NPC * (GY_PIECE + ACT_PIECE);
  constexpr bool NORM = (MODE == ACT_NORM || MODE == ACT_NORM_UP);
  constexpr bool UPS = (MODE == ACT_UP || MODE == ACT_NORM_UP);
  // gy is read once per (co tile, slice): non-temporal loads for co <= 64 blocks, so the L2 keeps
  // the activation halo rows neighbouring tiles re-read (64->64 @64 220 -> 208 us, 32->32 @128
  // upsampled 265 -> 258 us; step within noise).  co 128 blocks measured
  // slower with it (round 4).
  constexpr int kGyPol = CO_T <= 64 ? 2 : 0;
  static_assert(T::NI == 1 && T::HP == 10 && T::WP == 10, "8x8 tiles");
  static_assert(NWCO * NWCI * KSPLIT == 4 || NWCO * NWCI * KSPLIT == 8, "4 or 8 waves per block");
  static_assert((NWCI == 2 || NWCI == 4) && (FCO == 2 || FCO == 4), "wave / block tiles");
  static_assert(NTH % QG == 0 && NTH % QH == 0, "item channel groups fixed per thread");
  static_assert(KSTEPS % KSPLIT == 0 && NIT <= NSLOT, "item slots");
  static_assert(MODE != ACT_NORM_POOL, "pool-fed layers use the materialised activation");
  extern __shared__ __attribute__((aligned(16))) char wsm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wco = wave % NWCO, wci = (wave / NWCO) % NWCI, wk = wave / (NWCI * NWCO);
  // XCD-aware block order (1-D grid, wg_pipe_grid): blocks L and L + 8 share an XCD, so the
  // nm = (co tiles) x (ci tiles) blocks of one slice take consecutive L / 8 on ONE XCD and
  // read the slice's gy and activation rows while they are in that XCD's L2
  const int nco = Cout / CO_T, nm = nco * (Cin / CI_T);
  const int xcd = blockIdx.x & 7, wq = blockIdx.x >> 3, m = wq % nm;
  const int slice = (wq / nm) * 8 + xcd;
  if (slice >= g.slices) return;   // grid padding (whole block, before any barrier)
  const int co0 = (m % nco) * CO_T, ci0 = (m / nco) * CI_T;
  const int Hs = UPS ? H / 2 : H, Ws = UPS ? W / 2 : W;
  const int qh = tid % QH, qg = tid % QG;

  f32x4 acc[FCO][9];
#pragma unroll
  for (int f = 0; f < FCO; ++f)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[f][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  double bs[4] = {0.0, 0.0, 0.0, 0.0};

  const int per_img = g.ntx * g.nty;
  const int t_beg = slice * g.tps;
  const int t_end = min(t_beg + g.tps, g.tiles);
  int gshift = 0;   // F16: the slice's gy scale 2^k (see wgrad_split_kernel)
  if constexpr (F16)
    if (t_beg < t_end) gshift = f16_gshift(gmax, gmT, t_beg / per_img, (t_end - 1) / per_img);
  const float gsc = ldexpf(1.f, gshift);

  // tile-invariant item geometry: gy item k = pixel (gr, gc) of the tile, channels qg*4..;
  // halo item k = halo pixel hp (row hh, column ww), channels qh*4.. of the ci tile
  int gyo[KG], glo[KG];
#pragma unroll
  for (int k = 0; k < KG; ++k) {
    const int px = wg_store_perm<QG>((tid + NTH * k) / QG), r = px / TW, c = px % TW;
    gyo[k] = (r * W + c) * Cout + co0 + qg * 4;
    glo[k] = px * GSB + qg * 8;
  }
  int hdr[KH], hdc[KH], hlo[KH];   // row / column relative to the tile origin (-1 .. 8)
  int hbo[KH];                     // byte offset of the item relative to the tile's source origin
  const int srow = Ws * Cin * 4;   // bytes per source row
#pragma unroll
  for (int k = 0; k < KH; ++k) {
    const int pix = wg_store_perm<QH>((tid + NTH * k) / QH);
    hdr[k] = pix < T::HALO ? pix / T::WP - 1 : -(1 << 20);   // dead item: never in range
    hdc[k] = pix % T::WP - 1;
    hlo[k] = pix * ASB + qh * 8;
    // UPS: (y0 + dr) >> 1 == y0 / 2 + (dr >> 1) for even y0 (arithmetic shift = floor)
    hbo[k] = pix < T::HALO ? (UPS ? (hdr[k] >> 1) * srow + (hdc[k] >> 1) * Cin * 4
                                  : hdr[k] * srow + hdc[k] * Cin * 4) + (ci0 + qh * 4) * 4
                           : (int)0x80000000;   // dead item: out of range, never staged
  }
  const int gimg_bytes = H * W * Cout * 4, simg_bytes = Hs * Ws * Cin * 4;

  float4 rg[KG], rh[KH];
  float2 st_l[4], st_s[4];         // NORM: stats of the loading / the staging tile's image
  int lb = 0, ly = 0, lx = 0;      // tile whose data the item registers receive
  int sb = 0, sy = 0, sx = 0;      // tile being staged from them
  // ntx and nty are powers of two (wg_pipe_geom): shifts, no runtime integer division
  const int lgx = 31 - __builtin_clz(g.ntx), lgp = lgx + 31 - __builtin_clz(g.nty);
  auto tile_at = [&](int t, int& b0, int& y0, int& x0) EV_LAMBDA_INLINE {
    const int rr = t & ((1 << lgp) - 1);
    b0 = t >> lgp; y0 = (rr >> lgx) * T::TH; x0 = (rr & (g.ntx - 1)) * TW;
  };
  // buffer loads with 32-bit offsets into the loading tile's image (scalar descriptor base,
  // tile-uniform offset + a per-lane constant): rows above / below the image and dead items
  // fall outside the descriptor's range and read 0 without a memory access; the left / right
  // halo columns read a neighbouring row's pixel, which the staging zeroes (in_img)
  __amdgpu_buffer_rsrc_t rgy, rsrc;
  int gtoff = 0, stoff = 0;
  auto set_tile = [&]() EV_LAMBDA_INLINE {
    rgy = __builtin_amdgcn_make_buffer_rsrc((void*)(gy + (size_t)lb * H * W * Cout), 0, gimg_bytes,
                                            0x00020000);
    rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)(src + (size_t)lb * Hs * Ws * Cin), 0,
                                             simg_bytes, 0x00020000);
    gtoff = (ly * W + lx) * Cout * 4;
    stoff = UPS ? (ly >> 1) * srow + (lx >> 1) * Cin * 4 : ly * srow + lx * Cin * 4;
  };
  auto load_stats = [&]() EV_LAMBDA_INLINE {
    set_tile();
    if constexpr (NORM) {   // as {rstd, -mean*rstd}: one FMA + LeakyReLU per value
      const float2* sp = sstats + (size_t)lb * Cin + ci0 + qh * 4;
      st_l[0] = norm_fs(sp[0]); st_l[1] = norm_fs(sp[1]); st_l[2] = norm_fs(sp[2]); st_l[3] = norm_fs(sp[3]);
    }
  };
  auto in_img = [&](int k, int y0, int x0) EV_LAMBDA_INLINE {
    return (unsigned)(y0 + hdr[k]) < (unsigned)H && (unsigned)(x0 + hdc[k]) < (unsigned)W;
  };
  auto issue_item = [&](auto j_c) EV_LAMBDA_INLINE {
    constexpr int j = decltype(j_c)::value;
    if constexpr (j < KG) {
      rg[j] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                             rgy, gtoff + gyo[j] * 4, 0, kGyPol));
    } else {
      // unconditional (the staging zeroes what lies outside the image): with every load
      // issued, the compiler's vmcnt waits count exactly one tile's loads
      constexpr int k = j - KG;
      rh[k] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                             rsrc, stoff + hbo[k], 0, 0));
    }
  };
  float4 tb;   // this thread's gy sum of the staging tile (bias)
  auto store_item = [&](auto j_c, char* buf) EV_LAMBDA_INLINE {
    constexpr int j = decltype(j_c)::value;
    if constexpr (j < KG) {
      float4 v = rg[j];
      tb.x += v.x; tb.y += v.y; tb.z += v.z; tb.w += v.w;
      if constexpr (F16) v = make_float4(v.x * gsc, v.y * gsc, v.z * gsc, v.w * gsc);
      store_pieces<NP>(buf + glo[j], GY_PIECE, v);
    } else {
      constexpr int k = j - KG;
      if (hdr[k] > -2) {   // live item
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (in_img(k, sy, sx)) {
          v = rh[k];
          if (NORM)
            v = make_float4(normact_fs(v.x, st_s[0]), normact_fs(v.y, st_s[1]),
                            normact_fs(v.z, st_s[2]), normact_fs(v.w, st_s[3]));
        }
        store_pieces<NP>(buf + NPC * GY_PIECE + hlo[k], ACT_PIECE, v);
      }
    }
  };
  auto all_items = [&](auto fn) EV_LAMBDA_INLINE { static_for<NIT>(fn); };
  auto shift = [&]() EV_LAMBDA_INLINE {   // the loaded tile becomes the staging tile
    sb = lb; sy = ly; sx = lx;
#pragma unroll
    for (int i = 0; i < 4; ++i) st_s[i] = st_l[i];
  };

  // per-lane transposed-read geometry (wgrad_split_kernel)
  const int gq = lane >> 4, i16 = lane & 15, q = i16 >> 2, p4 = i16 & 3;
  const int acol = (wco * 16 * FCO + 4 * p4) * 2;
  const int bcol = (wci * 16 + 4 * p4) * 2;

  if (t_beg < t_end) {
    // prologue: tile t_beg staged into set 0, tile t_beg+1 (clamped) in the registers
    tile_at(t_beg, lb, ly, lx);
    load_stats();
    all_items([&](auto j) EV_LAMBDA_INLINE { issue_item(j); });
    shift();
    tb = make_float4(0.f, 0.f, 0.f, 0.f);
    all_items([&](auto j) EV_LAMBDA_INLINE { store_item(j, wsm); });
    bs[0] += (double)tb.x; bs[1] += (double)tb.y; bs[2] += (double)tb.z; bs[3] += (double)tb.w;
    tile_at(min(t_beg + 1, t_end - 1), lb, ly, lx);
    load_stats();
    all_items([&](auto j) EV_LAMBDA_INLINE { issue_item(j); });
  }
  __syncthreads();
  for (int t = t_beg; t < t_end; ++t) {
    const int cur = (t - t_beg) & 1;
    const char* gimg = wsm + cur * BUF;
    const char* aimg = gimg + NPC * GY_PIECE;
    char* nbuf = wsm + (1 - cur) * BUF;
    // the registers hold tile t+1: staged into the other set during this tile (surplus
    // copies of the last tile land in a set nobody reads), refilled with tile t+2
    shift();
    tile_at(min(t + 2, t_end - 1), lb, ly, lx);
    load_stats();
    tb = make_float4(0.f, 0.f, 0.f, 0.f);
    static_for<KSTEPS / KSPLIT>([&](auto si_c) EV_LAMBDA_INLINE {
      constexpr int si = decltype(si_c)::value;
      const int s = wk + si * KSPLIT;
      const int px0 = 32 * s + 4 * gq + q, px1 = px0 + 16;
      bf16x8w a[NPC][FCO];
#pragma unroll
      for (int i = 0; i < NPC; ++i)
#pragma unroll
        for (int f = 0; f < FCO; ++f)
          a[i][f] = tr_frag(gimg + i * GY_PIECE + px0 * GSB + acol + f * 32,
                            gimg + i * GY_PIECE + px1 * GSB + acol + f * 32);
      const int hp0 = (px0 / TW) * T::WP + px0 % TW, hp1 = (px1 / TW) * T::WP + px1 % TW;
      static_for<9>([&](auto tap_c) EV_LAMBDA_INLINE {
        constexpr int tap = decltype(tap_c)::value;
        constexpr int toff = (tap / 3) * T::WP + tap % 3;
        bf16x8w b[NPC];
#pragma unroll
        for (int i = 0; i < NPC; ++i)
          b[i] = tr_frag(aimg + i * ACT_PIECE + (hp0 + toff) * ASB + bcol,
                         aimg + i * ACT_PIECE + (hp1 + toff) * ASB + bcol);
#pragma unroll
        for (int f = 0; f < FCO; ++f) {
          f32x4 c = acc[f][tap];
#ifdef EV_WGP_NOMFMA   // timing experiment only (wrong results)
          c[0] += (float)a[0][f][0] * (float)b[0][0] + (float)a[1][f][1] * (float)b[1][1];
#else
          c = mfma16_piece<NP>(a[1][f], b[0], c);
          c = mfma16_piece<NP>(a[0][f], b[1], c);
          c = mfma16_piece<NP>(a[0][f], b[0], c);
#endif
          acc[f][tap] = c;
        }
        // this slot's share of the staging: item j at slot j * NSLOT / NIT
        all_items([&](auto j_c) EV_LAMBDA_INLINE {
          constexpr int j = decltype(j_c)::value;
#ifndef EV_WGP_NOSTAGE   // timing experiment only (wrong results)
          if constexpr (si * 9 + tap == (j * NSLOT) / NIT) {
            store_item(j_c, nbuf);
            issue_item(j_c);
          }
#endif
        });
      });
    });
    if (t + 1 < t_end) {
      bs[0] += (double)tb.x; bs[1] += (double)tb.y; bs[2] += (double)tb.z; bs[3] += (double)tb.w;
    }
    __syncthreads();
  }
  wgrad_split_finish<NWCO, KSPLIT, F16, FCO, NWCI>(acc, bs, wsm, wpart, bpart, slice, co0, ci0, Cin,
                                                   Cout, gsc, ci0 == 0);
}

// ------------------------------------------------------------------ cin == 1 (first conv)
// taps become the N dimension: B[k=px][j=tap] = x[px + d(tap)] (j < 9), 16x16x4 MFMA.
__global__ __launch_bounds__(128) void wgrad_cin1_kernel(
    const float* __restrict__ src, const float2* __restrict__ sstats, int smode,
    const float* __restrict__ gy, float* __restrict__ wpart, float* __restrict__ bpart, int B,
    int H, int W, int Cout, WgGeom g) {
  constexpr int GS = 48;  // 32 co + 16
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* lg = smem;
  float* la = smem + WG_PT * GS;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;  // wave = co half
  const int slice = blockIdx.x;
  const int HP = g.TH + 2, WP = g.TW + 2, halo = g.NI * HP * WP;
  const int l16 = lane & 15, kq = lane >> 4;
  const int tapj = l16 < 9 ? l16 : 0;
  const int tkh = tapj / 3, tkw = tapj % 3;
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  double bsum = 0.0;
  const int t_beg = slice * g.tps, t_end = min(t_beg + g.tps, g.tiles);
  const int tpx = g.TH * g.TW;
  for (int t = t_beg; t < t_end; ++t) {
    int b0, y0, x0;
    tile_origin(t, g, b0, y0, x0);
    __syncthreads();
    for (int i = tid; i < WG_PT * 8; i += 128) {
      const int px = i >> 3, q = i & 7;
      const int img = px >> g.ltpx, rem = px & (tpx - 1);
      const int r = rem >> g.lTW, c = rem & (g.TW - 1);
      const int gb = b0 + img;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (gb < B) v = ld4(gy + (((size_t)gb * H + y0 + r) * W + x0 + c) * Cout + q * 4);
      st4(lg + px * GS + q * 4, v);
    }
    for (int i = tid; i < halo; i += 128) {
      const int img = i / (HP * WP), rem = i - img * (HP * WP);
      const int hh = rem / WP, ww = rem - hh * WP;
      const int gh = y0 + hh - 1, gw = x0 + ww - 1, gb = b0 + img;
      float v = 0.f;
      if (gb < B && gh >= 0 && gh < H && gw >= 0 && gw < W)
        v = load_act1(src, sstats, smode, gb, gh, gw, 0, H, W, 1);
      la[i] = v;
    }
    __syncthreads();
    if (tid < 32) {
      float ts = 0.f;
      for (int px = 0; px < WG_PT; ++px) ts += lg[px * GS + tid];
      bsum += (double)ts;
    }
    for (int s = 0; s < WG_PT / 4; ++s) {
      const int px = 4 * s + kq;
      const int img = px >> g.ltpx, rem = px & (tpx - 1);
      const int r = rem >> g.lTW, c = rem & (g.TW - 1);
      const float a = lg[px * GS + wave * 16 + l16];
      const float bv = l16 < 9 ? la[(img * HP + r + tkh) * WP + c + tkw] : 0.f;
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv, acc, 0, 0, 0);
    }
  }
  if (l16 < 9) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = wave * 16 + kq * 4 + r;
      wpart[((size_t)slice * 9 + l16) * Cout + co] = acc[r];   // Cin == 1
    }
  }
  if (tid < 32) bpart[(size_t)slice * Cout + tid] = (float)bsum;
}

// ------------------------------------------------------------------ cout == 1 (last conv)
// dW[ci][tap] = sum_q g[q - d(tap)] * a[q][ci]:  A[i=tap][k=q] = shifted g (halo tile),
// B[k=q][j=ci] = unshifted activation tile.  2 waves = ci halves (cin == 32).
__global__ __launch_bounds__(128) void wgrad_cout1_kernel(
    const float* __restrict__ src, const float2* __restrict__ sstats, int smode,
    const float* __restrict__ g1, float* __restrict__ wpart, float* __restrict__ bpart, int B,
    int H, int W, int Cin, WgGeom g) {
  constexpr int AS = 48;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* la = smem;                  // [128 px][48]
  float* lgh = smem + WG_PT * AS;    // g halo
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int slice = blockIdx.x;
  const int HP = g.TH + 2, WP = g.TW + 2, halo = g.NI * HP * WP;
  const int l16 = lane & 15, kq = lane >> 4;
  const int tapi = l16 < 9 ? l16 : 0;
  const int tkh = tapi / 3, tkw = tapi % 3;
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  double bsum = 0.0;
  const int t_beg = slice * g.tps, t_end = min(t_beg + g.tps, g.tiles);
  const int tpx = g.TH * g.TW;
  for (int t = t_beg; t < t_end; ++t) {
    int b0, y0, x0;
    tile_origin(t, g, b0, y0, x0);
    __syncthreads();
    for (int i = tid; i < WG_PT * 8; i += 128) {
      const int px = i >> 3, q = i & 7;
      const int img = px >> g.ltpx, rem = px & (tpx - 1);
      const int r = rem >> g.lTW, c = rem & (g.TW - 1);
      const int gb = b0 + img;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (gb < B) v = load_act4(src, sstats, smode, gb, y0 + r, x0 + c, q * 4, H, W, Cin);
      st4(la + px * AS + q * 4, v);
    }
    for (int i = tid; i < halo; i += 128) {
      const int img = i / (HP * WP), rem = i - img * (HP * WP);
      const int hh = rem / WP, ww = rem - hh * WP;
      const int gh = y0 + hh - 1, gw = x0 + ww - 1, gb = b0 + img;
      float v = 0.f;
      if (gb < B && gh >= 0 && gh < H && gw >= 0 && gw < W) v = g1[((size_t)gb * H + gh) * W + gw];
      lgh[i] = v;
    }
    __syncthreads();
    if (tid == 0) {
      float ts = 0.f;
      for (int img = 0; img < g.NI; ++img)
        for (int r = 0; r < g.TH; ++r)
          for (int c = 0; c < g.TW; ++c) ts += lgh[(img * HP + r + 1) * WP + c + 1];
      bsum += (double)ts;
    }
    for (int s = 0; s < WG_PT / 4; ++s) {
      const int px = 4 * s + kq;
      const int img = px >> g.ltpx, rem = px & (tpx - 1);
      const int r = rem >> g.lTW, c = rem & (g.TW - 1);
      // g[q - d(tap)] with d(tap) = (kh-1, kw-1): halo coordinate (r+1-(kh-1), c+1-(kw-1))
      const float a = l16 < 9 ? lgh[(img * HP + r + 2 - tkh) * WP + c + 2 - tkw] : 0.f;
      const float bv = la[px * AS + wave * 16 + l16];
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv, acc, 0, 0, 0);
    }
  }
  // acc: row i = tap = kq*4 + r, col j = ci
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int tap = kq * 4 + r;
    if (tap < 9) wpart[((size_t)slice * 9 + tap) * Cin + wave * 16 + l16] = acc[r];  // Cout == 1
  }
  if (tid == 0) bpart[slice] = (float)bsum;
}

// ------------------------------------------------------------------ slice reduction
// Level 1: grid (element blocks, G slice groups); thread (e, g) sums slices
// [g*S/G, (g+1)*S/G) in double (fixed order) -> work[g][e].  Level 2: thread per element
// sums the G groups in order and scatters into the parameter-gradient layout.
// Elements are [tap][co][ci] weights followed by the cout biases.
__global__ void wgrad_reduce1_kernel(const float* __restrict__ wpart, const float* __restrict__ bpart,
                                     int S, int G, double* __restrict__ work, int nw, int cout) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int g = blockIdx.y;
  const int E = nw + cout;
  if (e >= E) return;
  const int k0 = (int)((long)g * S / G), k1 = (int)((long)(g + 1) * S / G);
  double s = 0.0;
  if (e < nw) {
#pragma unroll 8
    for (int k = k0; k < k1; ++k) s += (double)wpart[(size_t)k * nw + e];
  } else {
    const int co = e - nw;
    for (int k = k0; k < k1; ++k) s += (double)bpart[(size_t)k * cout + co];
  }
  work[(size_t)g * E + e] = s;
}

__global__ void wgrad_reduce2_kernel(const double* __restrict__ work, int G, float* __restrict__ dw,
                                     float* __restrict__ db, int cin, int cout, int kind) {
  const int nw = 9 * cout * cin;
  const int E = nw + cout;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  double s = 0.0;
  for (int g = 0; g < G; ++g) s += work[(size_t)g * E + e];
  if (e < nw) {
    const int t = e / (cout * cin), rem = e - t * (cout * cin);
    const int co = rem / cin, ci = rem - co * cin;
    size_t idx;
    if (kind == 0) idx = ((size_t)co * cin + ci) * 9 + t;
    else idx = ((size_t)ci * cout + co) * 9 + (8 - t);
    dw[idx] = (float)s;
  } else if (db) {
    db[e - nw] = (float)s;
  }
}

// batched reduction: blockIdx.z = layer (descriptor array passed by value)
// batched reduction: blockIdx.x runs over every layer's element blocks back to back
// (blk0[i] = first block of layer i), so small layers cost no idle blocks
struct WgReduceBatch {
  ebsdvae_wgrad_reduce_desc d[EBSDVAE_MAX_WGRAD_BATCH];
  size_t work_off[EBSDVAE_MAX_WGRAD_BATCH];   // in doubles
  int G[EBSDVAE_MAX_WGRAD_BATCH];
  int blk0[EBSDVAE_MAX_WGRAD_BATCH + 1];     // level-2 element blocks
  int r1blk0[EBSDVAE_MAX_WGRAD_BATCH + 1];   // level-1 (slice group x element) blocks
  int n;
};

EV_DEVINL int wg_layer_of(const WgReduceBatch& rb, int blk) {
  int i = 0;
  while (i + 1 < rb.n && blk >= rb.blk0[i + 1]) ++i;
  return i;
}

// level 1: blockIdx.x runs over (layer, slice group g, element block) with no idle blocks:
// layer L owns blocks [r1blk0[L], r1blk0[L+1]), G[L] x eblocks of them
__global__ void wgrad_reduce1_batch_kernel(const WgReduceBatch rb, double* __restrict__ work) {
  int L = 0;
  while (L + 1 < rb.n && (int)blockIdx.x >= rb.r1blk0[L + 1]) ++L;
  const ebsdvae_wgrad_reduce_desc& q = rb.d[L];
  const int G = rb.G[L];
  const int nw = 9 * q.cin * q.cout, E = nw + q.cout;
  const int eb = (E + 255) / 256;
  const int r = blockIdx.x - rb.r1blk0[L];
  const int g = r / eb;
  const int e = (r - g * eb) * blockDim.x + threadIdx.x;
  if (g >= G || e >= E) return;
  const int S = q.slices;
  const int k0 = (int)((long)g * S / G), k1 = (int)((long)(g + 1) * S / G);
  double s = 0.0;
  if (e < nw) {
#pragma unroll 8
    for (int k = k0; k < k1; ++k) s += (double)__builtin_nontemporal_load(q.wpart + (size_t)k * nw + e);
  } else {
    const int co = e - nw;
    for (int k = k0; k < k1; ++k) s += (double)q.bpart[(size_t)k * q.cout + co];
  }
  work[rb.work_off[L] + (size_t)g * E + e] = s;
}

__global__ void wgrad_reduce2_batch_kernel(const WgReduceBatch rb, const double* __restrict__ work) {
  const int L = wg_layer_of(rb, blockIdx.x);
  const ebsdvae_wgrad_reduce_desc& q = rb.d[L];
  const int G = rb.G[L];
  const int cin = q.cin, cout = q.cout;
  const int nw = 9 * cout * cin, E = nw + cout;
  const int e = (blockIdx.x - rb.blk0[L]) * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const double* w = work + rb.work_off[L];
  double s = 0.0;
  for (int g = 0; g < G; ++g) s += w[(size_t)g * E + e];
  if (e < nw) {
    const int t = e / (cout * cin), rem = e - t * (cout * cin);
    const int co = rem / cin, ci = rem - co * cin;
    size_t idx;
    if (q.kind == 0) idx = ((size_t)co * cin + ci) * 9 + t;
    else idx = ((size_t)ci * cout + co) * 9 + (8 - t);
    q.dw[idx] = (float)s;
  } else if (q.db) {
    q.db[e - nw] = (float)s;
  }
}

// slice groups of the level-1 reduction: about 2^19 threads per layer, at least EV_RED_GMIN
// groups (2: the 128-channel layers' level 1 writes and level 2 reads 4x fewer doubles than
// with 8; their reduce1 / reduce2 batch 95 -> 77 / 27 -> 24 us)
#ifndef EV_RED_GMIN
#define EV_RED_GMIN 2
#endif
static int reduce_groups(int slices, int cin, int cout) {
  const int E = 9 * cin * cout + cout;
  int G = 524288 / E;
  if (G < EV_RED_GMIN) G = EV_RED_GMIN;
  if (G > 64) G = 64;
  if (G > slices) G = slices;
  return G;
}

static size_t wg_lds(int variant, const WgGeom& g, int co_t) {
  const size_t halo = (size_t)g.NI * (g.TH + 2) * (g.TW + 2);
  if (variant == 0) return (WG_PT * (co_t + 16) + halo * WG_AS) * sizeof(float);
  if (variant == 1) return (WG_PT * 48 + halo) * sizeof(float);
  return (WG_PT * 48 + halo) * sizeof(float);
}

template <int NWCO, int KSPLIT, int MODE, int TW>
static void launch_wg_tw(dim3 grid, size_t lds, hipStream_t s, const float* src, const float* st,
                         const float* gy, float* wpart, float* bpart, int B, int H, int W, int cin,
                         int cout, const WgGeom& g) {
  auto k = wgrad_kernel<NWCO, KSPLIT, MODE, TW>;
  static bool once = false;
  if (!once) {
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    once = true;
  }
  hipLaunchKernelGGL(k, grid, dim3(256), lds, s, src, (const float2*)st, gy, wpart, bpart, B, H, W,
                     cin, cout, g);
}

template <int NWCO, int KSPLIT, int MODE>
static void launch_wg(dim3 grid, size_t lds, hipStream_t s, const float* src, const float* st,
                      const float* gy, float* wpart, float* bpart, int B, int H, int W, int cin,
                      int cout, const WgGeom& g) {
  if (g.TW == 32)
    launch_wg_tw<NWCO, KSPLIT, MODE, 32>(grid, lds, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g);
  else if (g.TW == 16)
    launch_wg_tw<NWCO, KSPLIT, MODE, 16>(grid, lds, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g);
  else if constexpr (NWCO == 1)   // 8x8 maps always take the 32-wide co tile
    launch_wg_tw<NWCO, KSPLIT, MODE, 8>(grid, lds, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g);
}

template <int NP, int NWCO, int KSPLIT, int MODE, int TW, int PT>
static void launch_wgs_tw(dim3 grid, hipStream_t s, const float* src, const float* st,
                          const float* gy, float* wpart, float* bpart, int B, int H, int W, int cin,
                          int cout, const WgGeom& g, const float* gmax, int gmT) {
  using T = WgTileP<TW, PT>;
  constexpr int CO_T = NWCO * 32;
  const size_t lds_img = (size_t)npc(NP) * ((size_t)PT * (CO_T * 2 + 32) + (size_t)T::HALO * WGS_ASB);
  const size_t lds_fold = KSPLIT == 2 ? (size_t)2 * 72 * 64 * 4 : 0;
  const size_t lds_bias = 256 * 4 * 8;
  size_t lds = lds_img;
  if (lds < lds_fold) lds = lds_fold;
  if (lds < lds_bias) lds = lds_bias;
  auto k = wgrad_split_kernel<NP, NWCO, KSPLIT, MODE, TW, PT>;
  static bool once = false;
  if (!once) {
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    once = true;
  }
  hipLaunchKernelGGL(k, grid, dim3(256), lds, s, src, (const float2*)st, gy, wpart, bpart, B, H, W,
                     cin, cout, g, gmax, gmT);
}

template <int NP, int NWCO, int KSPLIT, int MODE>
static void launch_wgs(dim3 grid, hipStream_t s, const float* src, const float* st, const float* gy,
                       float* wpart, float* bpart, int B, int H, int W, int cin, int cout,
                       const WgGeom& g, const float* gmax, int gmT) {
  constexpr int PT = 64;
  if (g.TW == 32)
    launch_wgs_tw<NP, NWCO, KSPLIT, MODE, 32, PT>(grid, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g, gmax, gmT);
  else if (g.TW == 16)
    launch_wgs_tw<NP, NWCO, KSPLIT, MODE, 16, PT>(grid, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g, gmax, gmT);
  else if constexpr (NWCO == 1)
    launch_wgs_tw<NP, NWCO, KSPLIT, MODE, 8, PT>(grid, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g, gmax, gmT);
}

template <int NP, int NWCO, int KSPLIT, int MODE, int NWCI = 2, int FCO = 2>
static void launch_wgp(dim3 grid, hipStream_t s, const float* src, const float* st, const float* gy,
                       float* wpart, float* bpart, int B, int H, int W, int cin, int cout,
                       const WgGeom& g, const float* gmax, int gmT) {
  constexpr int CO_T = NWCO * 16 * FCO, CI_T = NWCI * 16;
  constexpr int NTH = NWCO * NWCI * KSPLIT * 64;
  const size_t lds_img = 2 * (size_t)npc(NP) * ((size_t)64 * (CO_T * 2 + 32) + (size_t)100 * (CI_T * 2 + 32));
  const size_t lds_fold = KSPLIT == 2 ? (size_t)NWCO * NWCI * FCO * 36 * 64 * 4 : 0;
  size_t lds = lds_img;
  if (lds < lds_fold) lds = lds_fold;
  if (lds < (size_t)NTH * 4 * 8) lds = (size_t)NTH * 4 * 8;
  auto k = wgrad_pipe_kernel<NP, NWCO, KSPLIT, MODE, NWCI, FCO>;
  static bool once = false;
  if (!once) {
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    once = true;
  }
  hipLaunchKernelGGL(k, grid, dim3(NTH), lds, s, src, (const float2*)st, gy, wpart, bpart, B, H, W,
                     cin, cout, g, gmax, gmT);
}

template <int NP>
static void dispatch_wgp(int mode, bool narrow, dim3 grid, hipStream_t s, const float* src,
                         const float* st, const float* gy, float* wpart, float* bpart, int B, int H,
                         int W, int cin, int cout, const WgGeom& g, const float* gmax, int gmT) {
  if (narrow) {
    switch (mode) {
      case ACT_RAW: launch_wgp<NP, 1, 2, ACT_RAW>(grid, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g, gmax, gmT); break;
      case ACT_NORM: launch_wgp<NP, 1, 2, ACT_NORM>(grid, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g, gmax, gmT); break;
      case ACT_UP: launch_wgp<NP, 1, 2, ACT_UP>(grid, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g, gmax, gmT); break;
      default: launch_wgp<NP, 1, 2, ACT_NORM_UP>(grid, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g, gmax, gmT); break;
    }
  } else if (wg_pipe_cit(cin, cout) == 64 && wg_pipe_cot(cout) == 128) {   // co 128 x ci 64
    switch (mode) {
      case ACT_RAW: launch_wgp<NP, 2, 1, ACT_RAW, 4, 4>(grid, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g, gmax, gmT); break;
      case ACT_NORM: launch_wgp<NP, 2, 1, ACT_NORM, 4, 4>(grid, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g, gmax, gmT); break;
      case ACT_UP: launch_wgp<NP, 2, 1, ACT_UP, 4, 4>(grid, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g, gmax, gmT); break;
      default: launch_wgp<NP, 2, 1, ACT_NORM_UP, 4, 4>(grid, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g, gmax, gmT); break;
    }
  } else if (wg_pipe_cit(cin, cout) == 64) {   // co 64 x ci 64
    switch (mode) {
      case ACT_RAW: launch_wgp<NP, 2, 1, ACT_RAW, 4, 2>(grid, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g, gmax, gmT); break;
      case ACT_NORM: launch_wgp<NP, 2, 1, ACT_NORM, 4, 2>(grid, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g, gmax, gmT); break;
      case ACT_UP: launch_wgp<NP, 2, 1, ACT_UP, 4, 2>(grid, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g, gmax, gmT); break;
      default: launch_wgp<NP, 2, 1, ACT_NORM_UP, 4, 2>(grid, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g, gmax, gmT); break;
    }
  } else if (wg_pipe_cot(cout) == 128) {
    switch (mode) {
      case ACT_RAW: launch_wgp<NP, 4, 1, ACT_RAW>(grid, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g, gmax, gmT); break;
      case ACT_NORM: launch_wgp<NP, 4, 1, ACT_NORM>(grid, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g, gmax, gmT); break;
      case ACT_UP: launch_wgp<NP, 4, 1, ACT_UP>(grid, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g, gmax, gmT); break;
      default: launch_wgp<NP, 4, 1, ACT_NORM_UP>(grid, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g, gmax, gmT); break;
    }
  } else {
    switch (mode) {
      case ACT_RAW: launch_wgp<NP, 2, 1, ACT_RAW>(grid, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g, gmax, gmT); break;
      case ACT_NORM: launch_wgp<NP, 2, 1, ACT_NORM>(grid, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g, gmax, gmT); break;
      case ACT_UP: launch_wgp<NP, 2, 1, ACT_UP>(grid, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g, gmax, gmT); break;
      default: launch_wgp<NP, 2, 1, ACT_NORM_UP>(grid, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g, gmax, gmT); break;
    }
  }
}

template <int NP>
static void dispatch_wgs(int mode, bool narrow, dim3 grid, hipStream_t s, const float* src,
                         const float* st, const float* gy, float* wpart, float* bpart, int B, int H,
                         int W, int cin, int cout, const WgGeom& g, const float* gmax, int gmT) {
  if (narrow) {
    switch (mode) {
      case ACT_RAW: launch_wgs<NP, 1, 2, ACT_RAW>(grid, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g, gmax, gmT); break;
      case ACT_NORM: launch_wgs<NP, 1, 2, ACT_NORM>(grid, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g, gmax, gmT); break;
      case ACT_UP: launch_wgs<NP, 1, 2, ACT_UP>(grid, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g, gmax, gmT); break;
      default: launch_wgs<NP, 1, 2, ACT_NORM_UP>(grid, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g, gmax, gmT); break;
    }
  } else {
    switch (mode) {
      case ACT_RAW: launch_wgs<NP, 2, 1, ACT_RAW>(grid, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g, gmax, gmT); break;
      case ACT_NORM: launch_wgs<NP, 2, 1, ACT_NORM>(grid, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g, gmax, gmT); break;
      case ACT_UP: launch_wgs<NP, 2, 1, ACT_UP>(grid, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g, gmax, gmT); break;
      default: launch_wgs<NP, 2, 1, ACT_NORM_UP>(grid, s, src, st, gy, wpart, bpart, B, H, W, cin, cout, g, gmax, gmT); break;
    }
  }
}

static bool wgs_geom_ok(const WgGeom& g, int pt) {
  if (pt == 128)
    return (g.TW == 32 && g.TH == 4) || (g.TW == 16 && g.TH == 8 && g.NI == 1) ||
           (g.TW == 8 && g.TH == 8 && g.NI == 2);
  return (g.TW == 32 && g.TH == 2) || (g.TW == 16 && g.TH == 4 && g.NI == 1) ||
         (g.TW == 8 && g.TH == 8 && g.NI == 1);
}

}  // namespace ev

using namespace ev;

extern "C" int ebsdvae_conv3x3_wgrad_split_slices(int B, int H, int W, int cin, int cout, int pieces) {
  WgGeom g;
  if (pieces != 2 && pieces != 3 && pieces != NP_F16) return -1;
  if (B <= 0 || H <= 0 || W <= 0 || cin <= 0 || cout <= 0) return -1;
  if (cin % 32 || !(cout == 32 || cout % 64 == 0)) return -1;
  if (pieces != 3 && wg_pipe()) return wg_pipe_geom(B, H, W, cin, cout, &g) ? g.slices : -1;
  const int pt = 64;
  if (!wg_geom(B, H, W, cin, cout, &g, pt) || !wgs_geom_ok(g, pt)) return -1;
  return g.slices;
}

extern "C" int ebsdvae_conv3x3_wgrad_split(const float* src, const float* src_stats, int src_mode,
                                           const float* gy, float* wpart, float* bpart, int B,
                                           int H, int W, int cin, int cout, int pieces,
                                           ebsdvae_stream_t stream) {
  WgGeom g;
  EV_REQUIRE(src && gy && wpart && bpart && B > 0, "conv3x3_wgrad_split: null pointer");
  EV_REQUIRE(pieces == 2 || pieces == 3, "conv3x3_wgrad_split: pieces=%d (2 or 3)", pieces);
  EV_REQUIRE(src_mode >= 0 && src_mode <= 4 && src_mode != ACT_NORM_POOL,
             "conv3x3_wgrad_split: bad src_mode %d (pool-fed layers pass the pooled activation RAW)",
             src_mode);
  EV_REQUIRE(src_mode == ACT_RAW || src_mode == ACT_UP || src_stats, "conv3x3_wgrad_split: NORM needs stats");
  EV_REQUIRE(cin % 32 == 0 && (cout == 32 || cout % 64 == 0), "conv3x3_wgrad_split: cin=%d cout=%d unsupported",
             cin, cout);
  hipStream_t s = (hipStream_t)stream;
  if (pieces == 2 && wg_pipe()) {
    EV_REQUIRE(wg_pipe_geom(B, H, W, cin, cout, &g), "conv3x3_wgrad_split: unsupported shape H=%d W=%d", H, W);
    const bool narrow = cout == 32;
    dispatch_wgp<2>(src_mode, narrow, wg_pipe_grid(g, cin, cout), s, src, src_stats, gy, wpart, bpart, B,
                    H, W, cin, cout, g, nullptr, 0);
    return evh::check_launch("wgrad_split");
  }
  const int pt = 64;   // 64-pixel tiles: the per-piece LDS images and prefetch registers fit
  EV_REQUIRE(wg_geom(B, H, W, cin, cout, &g, pt) && wgs_geom_ok(g, pt),
             "conv3x3_wgrad_split: unsupported shape H=%d W=%d", H, W);
  // 32-wide co tiles where the 64-wide variant would exceed 256 VGPRs
  const bool narrow = cout == 32 || g.TW == 8 || (pieces == 3 && g.TW == 16);
  const dim3 grid(g.slices, narrow ? cout / 32 : cout / 64, cin / 32);
  if (pieces == 3)
    dispatch_wgs<3>(src_mode, narrow, grid, s, src, src_stats, gy, wpart, bpart, B, H, W, cin, cout, g,
                    nullptr, 0);
  else
    dispatch_wgs<2>(src_mode, narrow, grid, s, src, src_stats, gy, wpart, bpart, B, H, W, cin, cout, g,
                    nullptr, 0);
  return evh::check_launch("wgrad_split");
}

extern "C" int ebsdvae_conv3x3_wgrad_f16(const float* src, const float* src_stats, int src_mode,
                                         const float* gy, const float* gmax, int gm_tiles,
                                         float* wpart, float* bpart, int B, int H, int W, int cin,
                                         int cout, ebsdvae_stream_t stream) {
  WgGeom g;
  EV_REQUIRE(src && gy && gmax && gm_tiles > 0 && wpart && bpart && B > 0,
             "conv3x3_wgrad_f16: null pointer or no gradient maxima");
  EV_REQUIRE(src_mode >= 0 && src_mode <= 4 && src_mode != ACT_NORM_POOL,
             "conv3x3_wgrad_f16: bad src_mode %d (pool-fed layers pass the pooled activation RAW)",
             src_mode);
  EV_REQUIRE(src_mode == ACT_RAW || src_mode == ACT_UP || src_stats, "conv3x3_wgrad_f16: NORM needs stats");
  EV_REQUIRE(cin % 32 == 0 && (cout == 32 || cout % 64 == 0), "conv3x3_wgrad_f16: cin=%d cout=%d unsupported",
             cin, cout);
  if (wg_pipe()) {
    EV_REQUIRE(wg_pipe_geom(B, H, W, cin, cout, &g), "conv3x3_wgrad_f16: unsupported shape H=%d W=%d", H, W);
    const bool narrow = cout == 32;
    dispatch_wgp<NP_F16>(src_mode, narrow, wg_pipe_grid(g, cin, cout), (hipStream_t)stream, src, src_stats,
                         gy, wpart, bpart, B, H, W, cin, cout, g, gmax, gm_tiles);
    return evh::check_launch("wgrad_f16");
  }
  const int pt = 64;
  EV_REQUIRE(wg_geom(B, H, W, cin, cout, &g, pt) && wgs_geom_ok(g, pt),
             "conv3x3_wgrad_f16: unsupported shape H=%d W=%d", H, W);
  const bool narrow = cout == 32 || g.TW == 8;   // the 2-piece VGPR budget (as pieces = 2)
  const dim3 grid(g.slices, narrow ? cout / 32 : cout / 64, cin / 32);
  dispatch_wgs<NP_F16>(src_mode, narrow, grid, (hipStream_t)stream, src, src_stats, gy, wpart, bpart,
                       B, H, W, cin, cout, g, gmax, gm_tiles);
  return evh::check_launch("wgrad_f16");
}

extern "C" int ebsdvae_conv3x3_wgrad_slices(int B, int H, int W, int cin, int cout) {
  WgGeom g;
  if (!wg_geom(B, H, W, cin, cout, &g)) return -1;
  return g.slices;
}

extern "C" int ebsdvae_conv3x3_wgrad(const float* src, const float* src_stats, int src_mode,
                                     const float* gy, float* wpart, float* bpart, int B, int H,
                                     int W, int cin, int cout, ebsdvae_stream_t stream) {
  WgGeom g;
  EV_REQUIRE(src && gy && wpart && bpart && B > 0, "conv3x3_wgrad: null pointer");
  EV_REQUIRE(src_mode >= 0 && src_mode <= 4, "conv3x3_wgrad: bad src_mode");
  EV_REQUIRE(src_mode == ACT_RAW || src_mode == ACT_UP || src_stats, "conv3x3_wgrad: NORM needs stats");
  EV_REQUIRE(wg_geom(B, H, W, cin, cout, &g), "conv3x3_wgrad: unsupported shape H=%d W=%d", H, W);
  hipStream_t s = (hipStream_t)stream;
  if (cin == 1) {
    EV_REQUIRE(cout == 32, "conv3x3_wgrad: cin=1 needs cout=32");
    hipLaunchKernelGGL(wgrad_cin1_kernel, dim3(g.slices), dim3(128), wg_lds(1, g, 32), s, src,
                       (const float2*)src_stats, src_mode, gy, wpart, bpart, B, H, W, cout, g);
    return evh::check_launch("wgrad_cin1");
  }
  if (cout == 1) {
    EV_REQUIRE(cin == 32, "conv3x3_wgrad: cout=1 needs cin=32");
    hipLaunchKernelGGL(wgrad_cout1_kernel, dim3(g.slices), dim3(128), wg_lds(2, g, 0), s, src,
                       (const float2*)src_stats, src_mode, gy, wpart, bpart, B, H, W, cin, g);
    return evh::check_launch("wgrad_cout1");
  }
  EV_REQUIRE(cin % 32 == 0 && (cout == 32 || cout % 64 == 0), "conv3x3_wgrad: cin=%d cout=%d unsupported",
             cin, cout);
  EV_REQUIRE((g.TW == 32 && g.TH == 4) || (g.TW == 16 && g.TH == 8 && g.NI == 1) ||
                 (g.TW == 8 && g.TH == 8 && g.NI == 2),
             "conv3x3_wgrad: unsupported tile geometry H=%d W=%d", H, W);
  EV_REQUIRE(src_mode != ACT_NORM_POOL,
             "conv3x3_wgrad: pass the pooled activation materialised by the forward (RAW)");
  if (cout == 32 || g.TW == 8) {
    const size_t lds = wg_lds(0, g, 32);
    const dim3 grid(g.slices, cout / 32, cin / 32);
    switch (src_mode) {
      case ACT_RAW: launch_wg<1, 2, ACT_RAW>(grid, lds, s, src, src_stats, gy, wpart, bpart, B, H, W, cin, cout, g); break;
      case ACT_NORM: launch_wg<1, 2, ACT_NORM>(grid, lds, s, src, src_stats, gy, wpart, bpart, B, H, W, cin, cout, g); break;
      case ACT_UP: launch_wg<1, 2, ACT_UP>(grid, lds, s, src, src_stats, gy, wpart, bpart, B, H, W, cin, cout, g); break;
      default: launch_wg<1, 2, ACT_NORM_UP>(grid, lds, s, src, src_stats, gy, wpart, bpart, B, H, W, cin, cout, g); break;
    }
  } else {
    const size_t lds = wg_lds(0, g, 64);
    const dim3 grid(g.slices, cout / 64, cin / 32);
    switch (src_mode) {
      case ACT_RAW: launch_wg<2, 1, ACT_RAW>(grid, lds, s, src, src_stats, gy, wpart, bpart, B, H, W, cin, cout, g); break;
      case ACT_NORM: launch_wg<2, 1, ACT_NORM>(grid, lds, s, src, src_stats, gy, wpart, bpart, B, H, W, cin, cout, g); break;
      case ACT_UP: launch_wg<2, 1, ACT_UP>(grid, lds, s, src, src_stats, gy, wpart, bpart, B, H, W, cin, cout, g); break;
      default: launch_wg<2, 1, ACT_NORM_UP>(grid, lds, s, src, src_stats, gy, wpart, bpart, B, H, W, cin, cout, g); break;
    }
  }
  return evh::check_launch("wgrad");
}

extern "C" size_t ebsdvae_wgrad_reduce_work(int slices, int cin, int cout) {
  return (size_t)reduce_groups(slices, cin, cout) * (9 * (size_t)cin * cout + cout) * sizeof(double);
}

extern "C" int ebsdvae_wgrad_reduce(const float* wpart, const float* bpart, int slices, float* dw,
                                    float* db, int cin, int cout, int kind, void* work,
                                    ebsdvae_stream_t stream) {
  EV_REQUIRE(wpart && bpart && dw && work && slices > 0, "wgrad_reduce: bad args");
  const int E = 9 * cin * cout + cout;
  const int G = reduce_groups(slices, cin, cout);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(wgrad_reduce1_kernel, dim3((E + 255) / 256, G), dim3(256), 0, st, wpart, bpart,
                     slices, G, (double*)work, 9 * cin * cout, cout);
  hipLaunchKernelGGL(wgrad_reduce2_kernel, dim3((E + 255) / 256), dim3(256), 0, st,
                     (const double*)work, G, dw, db, cin, cout, kind);
  return evh::check_launch("wgrad_reduce");
}

// host-side layout of the batched work buffer (shared by the size query and the launch)
static bool wg_batch_layout(const ebsdvae_wgrad_reduce_desc* descs, int n, WgReduceBatch* rb,
                            size_t* total, int* maxE, int* maxG) {
  size_t off = 0;
  int blk = 0, blk1 = 0;
  *maxE = 0;
  *maxG = 0;
  for (int i = 0; i < n; ++i) {
    const ebsdvae_wgrad_reduce_desc& q = descs[i];
    if (!q.wpart || !q.bpart || !q.dw || q.slices <= 0 || q.cin <= 0 || q.cout <= 0 ||
        (q.kind != 0 && q.kind != 1))
      return false;
    const int E = 9 * q.cin * q.cout + q.cout;
    const int G = reduce_groups(q.slices, q.cin, q.cout);
    if (rb) {  // (G may differ per layer; level 1 of layer i uses G[i] groups)
      rb->d[i] = q;
      rb->work_off[i] = off;
      rb->G[i] = G;
      rb->blk0[i] = blk;
      rb->r1blk0[i] = blk1;
    }
    blk += (E + 255) / 256;
    blk1 += G * ((E + 255) / 256);
    off += (size_t)G * E;
  }
  if (rb) {
    rb->blk0[n] = blk;
    rb->r1blk0[n] = blk1;
    rb->n = n;
  }
  *maxE = blk;    // total level-2 blocks
  *maxG = blk1;   // total level-1 blocks
  *total = off * sizeof(double);
  return true;
}

extern "C" size_t ebsdvae_wgrad_reduce_batch_work(const ebsdvae_wgrad_reduce_desc* descs, int n) {
  size_t total = 0;
  int maxE, maxG;
  if (!descs || n <= 0 || n > EBSDVAE_MAX_WGRAD_BATCH || !wg_batch_layout(descs, n, nullptr, &total, &maxE, &maxG))
    return 0;
  return total;
}

extern "C" int ebsdvae_wgrad_reduce_batch(const ebsdvae_wgrad_reduce_desc* descs, int n, void* work,
                                          ebsdvae_stream_t stream) {
  EV_REQUIRE(descs && work && n > 0 && n <= EBSDVAE_MAX_WGRAD_BATCH, "wgrad_reduce_batch: n=%d out of range", n);
  WgReduceBatch rb;
  size_t total = 0;
  int maxE = 0, maxG = 0;   // total level-2 / level-1 blocks
  EV_REQUIRE(wg_batch_layout(descs, n, &rb, &total, &maxE, &maxG), "wgrad_reduce_batch: bad descriptor");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(wgrad_reduce1_batch_kernel, dim3(maxG), dim3(256), 0, st, rb, (double*)work);
  hipLaunchKernelGGL(wgrad_reduce2_batch_kernel, dim3(maxE), dim3(256), 0, st, rb, (const double*)work);
  return evh::check_launch("wgrad_reduce_batch");
}
