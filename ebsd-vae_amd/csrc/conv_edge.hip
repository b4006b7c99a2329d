// The two channel-degenerate convs of the network, on the VALU (they are HBM-bound:
// ~4.4 FLOP/B):
//   * the final nn.Conv2d(32, 1, 3, 1, 1) producing the logits x_hat (latice/model.py:148)
//     and its input gradient;
//   * (with flip=1 and a RAW source) the input gradient of the first nn.Conv2d(1, 32)
//     (latice/model.py:110), only needed when the caller asks for d loss / d x.
// The forward stages the producer's activation halo (InstanceNorm + LeakyReLU applied
// on the fly) in LDS with an odd channel stride; weights are wave-uniform (scalar loads).
#include "common.h"
#include "../../include/ebsdvae.h"

namespace ev {

struct EdgeGeom {
  int TH, TW, NI;
};

static bool edge_geom(int H, int W, EdgeGeom* g) {
  g->TW = W < 64 ? W : 64;
  if (H * g->TW >= 256) {
    g->TH = 256 / g->TW;
    g->NI = 1;
  } else {
    g->TH = H;
    g->NI = 256 / (H * W);
    if (g->NI * H * W != 256) return false;
  }
  return (W % g->TW) == 0 && (H % g->TH) == 0;
}

template <int CIN>
__global__ __launch_bounds__(256) void conv_cout1_fwd_kernel(
    const float* __restrict__ src, const float2* __restrict__ sstats, int smode,
    const float* __restrict__ w, const float* __restrict__ bias, float* __restrict__ out,
    int flip, int B, int H, int W, EdgeGeom g) {
  constexpr int CS = CIN + 1;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x;
  const int HP = g.TH + 2, WP = g.TW + 2;
  const int halo = g.NI * HP * WP;
  const int ntx = W / g.TW, nty = H / g.TH;
  const int per_img = ntx * nty;
  const int t = blockIdx.x;
  const int b0 = (t / per_img) * g.NI, r0 = t % per_img;
  const int y0 = (r0 / ntx) * g.TH, x0 = (r0 % ntx) * g.TW;
  for (int i = tid; i < halo * (CIN / 4); i += 256) {
    const int pix = i / (CIN / 4), q = i - pix * (CIN / 4);
    const int img = pix / (HP * WP), rem = pix - img * (HP * WP);
    const int hh = rem / WP, ww = rem - hh * WP;
    const int gh = y0 + hh - 1, gw = x0 + ww - 1, gb = b0 + img;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (gb < B && gh >= 0 && gh < H && gw >= 0 && gw < W)
      v = load_act4(src, sstats, smode, gb, gh, gw, q * 4, H, W, CIN);
    float* d = smem + pix * CS + q * 4;
    d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
  }
  __syncthreads();
  const int tpx = g.TH * g.TW;
  const int img = tid / tpx, rem = tid - img * tpx;
  const int r = rem / g.TW, c = rem - r * g.TW;
  const int gb = b0 + img;
  float acc = bias ? bias[0] : 0.f;
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int kh = tap / 3, kw = tap % 3;
    const int tw = flip ? 8 - tap : tap;
    const float* xr = smem + ((img * HP + r + kh) * WP + c + kw) * CS;
#pragma unroll
    for (int ci = 0; ci < CIN; ++ci) acc = fmaf(xr[ci], w[ci * 9 + tw], acc);
  }
  if (gb < B) out[((size_t)gb * H + y0 + r) * W + x0 + c] = acc;
}

// Streaming row kernel (64 <= W <= 256, W % 64 == 0; RAW or NORM source): one thread per
// image column walks down a TH-row band.  Each input row (W pixels x 32 channels) is read
// ONCE with coalesced float4 loads (next row prefetched into registers), transformed, and
// staged in LDS (pixel stride 36 floats); each thread then dots its pixel's 32 channels
// with all 9 taps.  The 9 per-tap partial sums go through an LDS row so every column can
// gather its three horizontal neighbours; output rows complete one input row later
// (rolling accumulators).  HBM traffic ~ (TH+2)/TH x the input.
#ifndef EV_ROWS_TH
#define EV_ROWS_TH 16
#endif
constexpr int ROWS_TH = EV_ROWS_TH;   // rows per band (a multiple of 3 minus 2)
constexpr int ROWS_PS = 36;   // LDS pixel stride (floats) of the staged row

template <bool NORM, bool FLIP>
__global__ __launch_bounds__(256) void conv_cout1_rows_kernel(
    const float* __restrict__ src, const float2* __restrict__ sstats, const float* __restrict__ w,
    const float* __restrict__ bias, float* __restrict__ out, int H, int W) {
  constexpr int C = 32;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int x = threadIdx.x;
  const int WP = W + 2;
  // single-buffered: each row's two barriers already separate its writes from the
  // previous row's reads of P and A
  float* P = smem;                    // [9][W + 2] per-tap partial sums
  float* A = smem + 9 * WP;           // [W][ROWS_PS] staged activation row

  const int nb = H / ROWS_TH;
  const int b = blockIdx.x / nb, h0 = (blockIdx.x - b * nb) * ROWS_TH;
  if (x < 18) P[(x / 2) * WP + (x & 1) * (W + 1)] = 0.f;
  // float4 item k of this thread: row element x + k*W -> pixel (x + k*W) / 8, channels
  // 4 * (x % 8) .. +3 (W % 8 == 0, so the channel group is the same for every k)
  const int cq = x & 7;
  float2 fs[4];
  if (NORM) {
#pragma unroll
    for (int i = 0; i < 4; ++i) fs[i] = norm_fs(sstats[(size_t)b * C + cq * 4 + i]);
  }
  const float* sb = src + (size_t)b * H * W * C;
  // three row buffers in rotation (the loop is unrolled by 3, so no register copies): while
  // row r is computed, rows r+1 and r+2 are loading.  Loads are unconditional (row index
  // clamped into the image; rows outside it are zeroed when staged), so the compiler's
  // waits stay counted instead of draining every load at each row.
  float4 bA[C / 4], bB[C / 4], bC[C / 4];
  auto load_row = [&](int r, float4 (&d)[C / 4]) EV_LAMBDA_INLINE {
    const int rc = min(max(r, 0), H - 1);
#pragma unroll
    for (int k = 0; k < C / 4; ++k) d[k] = ld4(sb + (size_t)rc * W * C + (size_t)(x + k * W) * 4);
  };
  const float bb = bias ? bias[0] : 0.f;
  float acc_m = 0.f, acc_0 = 0.f;   // output rows r-1 and r (row r+1 starts from zero)
  auto step = [&](int r, float4 (&cur)[C / 4], float4 (&nxt)[C / 4]) EV_LAMBDA_INLINE {
    load_row(r + 2, nxt);
    float* ab = A;
    const bool inside = r >= 0 && r < H;
#pragma unroll
    for (int k = 0; k < C / 4; ++k) {
      float4 v = cur[k];
      if (NORM)
        v = make_float4(normact_fs(v.x, fs[0]), normact_fs(v.y, fs[1]), normact_fs(v.z, fs[2]),
                        normact_fs(v.w, fs[3]));
      if (!inside) v = make_float4(0.f, 0.f, 0.f, 0.f);
      const int e = x + k * W;
      st4(ab + (e >> 3) * ROWS_PS + cq * 4, v);
    }
    __syncthreads();
    float* pb = P;
    // channel-major so each channel's 9 weights are adjacent (merged wide scalar loads); in
    // chunks of 8 channels (72 weights) so a chunk's weights stay in SGPRs -- all 288 at once
    // overflow them and every FMA then pays a v_readlane
    float p[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) p[t] = 0.f;
#pragma unroll 1
    for (int c0 = 0; c0 < C; c0 += 8) {
      const float4 u0 = ld4(ab + x * ROWS_PS + c0), u1 = ld4(ab + x * ROWS_PS + c0 + 4);
      const float a[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
      const float* wc = w + c0 * 9;
#pragma unroll
      for (int c = 0; c < 8; ++c)
#pragma unroll
        for (int t = 0; t < 9; ++t) p[FLIP ? 8 - t : t] = fmaf(a[c], wc[c * 9 + t], p[FLIP ? 8 - t : t]);
    }
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) pb[tap * WP + x + 1] = p[tap];
    __syncthreads();
    // input row r feeds output row r+1 with kh = 0, row r with kh = 1, row r-1 with kh = 2
    float cpart[3];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const float* row = pb + kh * 3 * WP + x;
      cpart[kh] = row[0] + row[WP + 1] + row[2 * WP + 2];
    }
    const float fin = acc_m + cpart[2];   // output row r-1 is complete
    if (r - 1 >= h0 && r - 1 < h0 + ROWS_TH) out[((size_t)b * H + r - 1) * W + x] = fin + bb;
    acc_m = acc_0 + cpart[1];
    acc_0 = cpart[0];
  };
  load_row(h0 - 1, bA);
  load_row(h0, bB);
  static_assert((ROWS_TH + 2) % 3 == 0, "rows per band + halo: whole groups of three");
  for (int r = h0 - 1; r <= h0 + ROWS_TH; r += 3) {
    step(r, bA, bC);
    step(r + 1, bB, bA);
    step(r + 2, bC, bB);
  }
}

// gin[b,h,w,ci] = sum_tap g[b, h-kh+1, w-kw+1] * w[ci][tap]
template <int CIN>
__global__ __launch_bounds__(256) void conv_cout1_dgrad_kernel(
    const float* __restrict__ gsrc, const float* __restrict__ w, float* __restrict__ gin, int B,
    int H, int W, EdgeGeom g) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x;
  const int HP = g.TH + 2, WP = g.TW + 2;
  const int halo = g.NI * HP * WP;
  const int ntx = W / g.TW, nty = H / g.TH;
  const int per_img = ntx * nty;
  const int t = blockIdx.x;
  const int b0 = (t / per_img) * g.NI, r0 = t % per_img;
  const int y0 = (r0 / ntx) * g.TH, x0 = (r0 % ntx) * g.TW;
  for (int i = tid; i < halo; i += 256) {
    const int img = i / (HP * WP), rem = i - img * (HP * WP);
    const int hh = rem / WP, ww = rem - hh * WP;
    const int gh = y0 + hh - 1, gw = x0 + ww - 1, gb = b0 + img;
    float v = 0.f;
    if (gb < B && gh >= 0 && gh < H && gw >= 0 && gw < W) v = gsrc[((size_t)gb * H + gh) * W + gw];
    smem[i] = v;
  }
  __syncthreads();
  constexpr int CG = CIN / 4;
  const int cg = tid % CG;
  float wr[4][9];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) wr[k][tap] = w[(cg * 4 + k) * 9 + tap];
  const int tpx = g.TH * g.TW;
  for (int item = tid; item < 256 * CG; item += 256) {
    const int px = item / CG;
    const int img = px / tpx, rem = px - img * tpx;
    const int r = rem / g.TW, c = rem - r * g.TW;
    float a[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int kh = tap / 3, kw = tap % 3;
      // g at (r - (kh-1), c - (kw-1)) -> halo (r + 2 - kh, c + 2 - kw)
      const float gv = smem[(img * HP + r + 2 - kh) * WP + c + 2 - kw];
#pragma unroll
      for (int k = 0; k < 4; ++k) a[k] = fmaf(gv, wr[k][tap], a[k]);
    }
    const int gb = b0 + img;
    if (gb < B) st4(gin + (((size_t)gb * H + y0 + r) * W + x0 + c) * CIN + cg * 4,
                    make_float4(a[0], a[1], a[2], a[3]));
  }
}

// ------------------------------------------------------------------ first conv (cin == 1)
// y0 = conv3x3(x, w0) + b0 for C == 32 output channels on the VALU (first_conv_px, the fma
// chain the first block's backward recomputes y0 with), plus its InstanceNorm partials
// {mean, M2} per row band of FIRST_PX pixels.  It is a write-bound kernel (1 input channel,
// 32 output channels: 128 B written per 4 B read); block = one row band of one image, x band
// + halo staged in LDS, 8 threads per pixel (4 channels each: one 16-B store, a pixel's 128 B
// contiguous), the band's values kept in registers for the two-pass statistics.
constexpr int FIRST_C = 32, FIRST_PX = 512, FIRST_NPT = FIRST_PX / 32;

static int first_rows(int W) { return (W > 0 && W < FIRST_PX && FIRST_PX % W == 0) ? FIRST_PX / W : 0; }

__global__ __launch_bounds__(256) void conv_first_fwd_kernel(
    const float* __restrict__ x, const float* __restrict__ w0, const float* __restrict__ b0,
    float* __restrict__ y, float2* __restrict__ part, int H, int W, int TH) {
  extern __shared__ float xs[];   // (TH + 2) x (W + 2)
  __shared__ float red[8][8][4];   // [wave (mean) | 4 + wave (M2)][channel group][k]
  const int tile = blockIdx.x, b = blockIdx.y, T = gridDim.x;
  const int tid = threadIdx.x, cg = tid & 7, pr = tid >> 3;
  const int c = cg * 4, r0 = tile * TH, WP = W + 2;
  const float* xb = x + (size_t)b * H * W;
  for (int i = tid; i < (TH + 2) * WP; i += 256) {
    const int r = i / WP, cc = i - r * WP;
    const int gh = r0 - 1 + r, gw = cc - 1;
    xs[i] = (gh >= 0 && gh < H && gw >= 0 && gw < W) ? xb[gh * W + gw] : 0.f;
  }
  pkf2 wt2[2][9], bb2[2];   // channel pairs (2k, 2k+1) for v_pk_fma_f32
#pragma unroll
  for (int k = 0; k < 2; ++k) {
#pragma unroll
    for (int t = 0; t < 9; ++t) wt2[k][t] = pk2(w0[(c + 2 * k) * 9 + t], w0[(c + 2 * k + 1) * 9 + t]);
    bb2[k] = b0 ? pk2(b0[c + 2 * k], b0[c + 2 * k + 1]) : pk2(0.f, 0.f);
  }
  __syncthreads();
  float v[FIRST_NPT][4];
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  float* yb = y ? y + ((size_t)b * H * W + (size_t)r0 * W) * FIRST_C + c : nullptr;
#pragma unroll
  for (int j = 0; j < FIRST_NPT; ++j) {
    const int p = pr + 32 * j, h = p / W, w = p - h * W;
    float nb[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) nb[t] = xs[(h + t / 3) * WP + w + t % 3];
    // two channels per v_pk_fma_f32 (bit-identical to first_conv_px per channel)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const pkf2 y2 = first_conv_px2(nb, wt2[k], bb2[k]);
      v[j][2 * k] = y2.x;
      v[j][2 * k + 1] = y2.y;
      s[2 * k] += y2.x;
      s[2 * k + 1] += y2.y;
    }
    // non-temporal: y0 is read once, by the next conv (first conv 119 -> 113 us, step -0.03 ms).
    // y == NULL: statistics only -- the next conv recomputes y0 from x (ACT_FIRST staging)
    if (y) st4_nt(yb + (size_t)p * FIRST_C, make_float4(v[j][0], v[j][1], v[j][2], v[j][3]));
  }
  // band statistics per channel, fixed order: the 8 pixel lanes of a wave by a shuffle tree
  // (lanes cg, cg + 8, ..., cg + 56), then the 4 waves through LDS (a serial walk over 32
  // LDS partials per channel cost ~8 us per block)
  const int lane = tid & 63, wave = tid >> 6;
  float mean[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float a = s[k];
    a += __shfl_xor(a, 8, 64);
    a += __shfl_xor(a, 16, 64);
    a += __shfl_xor(a, 32, 64);
    if (lane < 8) red[wave][lane][k] = a;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k)
    mean[k] = (red[0][cg][k] + red[1][cg][k] + red[2][cg][k] + red[3][cg][k]) * (1.0f / FIRST_PX);
  float q[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < FIRST_NPT; ++j)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float d = v[j][k] - mean[k];
      q[k] = fmaf(d, d, q[k]);
    }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float a = q[k];
    a += __shfl_xor(a, 8, 64);
    a += __shfl_xor(a, 16, 64);
    a += __shfl_xor(a, 32, 64);
    if (lane < 8) red[4 + wave][lane][k] = a;
  }
  __syncthreads();
  if (tid < FIRST_C) {   // channel tid: group tid / 4, element tid % 4
    const int g = tid >> 2, k = tid & 3;
    const float m = (red[0][g][k] + red[1][g][k] + red[2][g][k] + red[3][g][k]) * (1.0f / FIRST_PX);
    part[((size_t)b * T + tile) * FIRST_C + tid] =
        make_float2(m, red[4][g][k] + red[5][g][k] + red[6][g][k] + red[7][g][k]);
  }
}


// ------------------------------------------------------------------ first-conv statistics (inference)
// The InstanceNorm statistics of y0 = conv(x, w0) + b0 without y0 (ebsdvae_conv_first_stats):
// every channel is a linear map of the 9 shifted copies of x, so with, per image,
//   m_t  = (1/N) sum_p xs_t[p]          and   Q_tt' = (1/N) sum_p xs_t[p] xs_t'[p]
// (xs_t[p] = x[p + d_t], zero outside the image; 9 sums and 45 products per pixel, for all 32
// channels at once instead of 288 MACs per pixel, in double: FP64 FMAs run at half the fp32 rate)
//   mean_c = b_c + sum_t w_ct m_t,   var_c = sum_{t,t'} w_ct w_ct' (Q_tt' - m_t m_t')
// in double (no cancellation to speak of).  Every thread accumulates its column's pixels in
// double; the block's 256 threads fold in a fixed order.  The inference path's first conv then reads x once and writes 256 bytes per image
// (encoder.1 recomputes y0 from x, ebsdvae_conv3x3_fwd_split_first).
constexpr int FG_CH = 32;            // rows per chunk (LDS tile FG_CH + 2 rows)
constexpr int FG_NS = 9 + 45;        // sums per image
__global__ __launch_bounds__(256) void first_gram_kernel(const float* __restrict__ x,
                                                         const float* __restrict__ w0,
                                                         const float* __restrict__ b0,
                                                         float2* __restrict__ st, int C, int H, int W) {
  extern __shared__ float fg_sm[];   // x tile [FG_CH + 2][W + 2], then the fold scratch
  const int b = blockIdx.x, tid = threadIdx.x;
  const int WP = W + 2;
  const float* xb = x + (size_t)b * H * W;
  const int rpc = 256 / W;            // rows of a chunk a column's threads split (W <= 256)
  const int col = tid % W, r_off = tid / W;
  double acc[FG_NS];
#pragma unroll
  for (int e = 0; e < FG_NS; ++e) acc[e] = 0.0;
  for (int h0 = 0; h0 < H; h0 += FG_CH) {
    __syncthreads();
    for (int i = tid; i < (FG_CH + 2) * WP; i += 256) {
      const int r = i / WP, cc = i - r * WP;
      const int gh = h0 - 1 + r, gw = cc - 1;
      fg_sm[i] = (gh >= 0 && gh < H && gw >= 0 && gw < W) ? xb[gh * W + gw] : 0.f;
    }
    __syncthreads();
    if (r_off < rpc) {
      for (int r = r_off; r < FG_CH; r += rpc) {
        double nb[9];
#pragma unroll
        for (int t = 0; t < 9; ++t) nb[t] = (double)fg_sm[(r + t / 3) * WP + col + t % 3];
#pragma unroll
        for (int t = 0; t < 9; ++t) acc[t] += nb[t];
#pragma unroll
        for (int t = 0, e = 9; t < 9; ++t)
#pragma unroll
          for (int u = t; u < 9; ++u, ++e) acc[e] = fma(nb[t], nb[u], acc[e]);
      }
    }
  }
  __syncthreads();
  // fixed-order fold: lanes by a shuffle tree, then the 4 waves
  double* red = reinterpret_cast<double*>(fg_sm);   // [4][FG_NS]
  const int lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int e = 0; e < FG_NS; ++e) {
    double v = acc[e];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) red[wave * FG_NS + e] = v;
  }
  __syncthreads();
  double* tot = red + 4 * FG_NS;                     // [FG_NS]
  if (tid < FG_NS) tot[tid] = ((red[tid] + red[FG_NS + tid]) + red[2 * FG_NS + tid]) + red[3 * FG_NS + tid];
  __syncthreads();
  if (tid < C) {
    const int c = tid;
    const double inv_n = 1.0 / ((double)H * W);
    double m[9], w[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) { m[t] = tot[t] * inv_n; w[t] = (double)w0[c * 9 + t]; }
    double mean = b0 ? (double)b0[c] : 0.0, var = 0.0;
#pragma unroll
    for (int t = 0; t < 9; ++t) mean += w[t] * m[t];
    int e = 9;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int u = t; u < 9; ++u, ++e) {
        const double cov = tot[e] * inv_n - m[t] * m[u];
        var += (t == u ? 1.0 : 2.0) * w[t] * w[u] * cov;
      }
    var = var > 0.0 ? var : 0.0;
    st[(size_t)b * C + c] = make_float2((float)mean, (float)(1.0 / sqrt(var + (double)kInEps)));
  }
}
}  // namespace ev

using namespace ev;

extern "C" int ebsdvae_conv_first_stat_tiles(int H, int W) {
  const int th = first_rows(W);
  return (th > 0 && ev_dim_ok(H) && H % th == 0) ? H / th : -1;
}

extern "C" int ebsdvae_conv_first_fwd(const float* x, const float* w0, const float* b0, float* y,
                                      float* part, int B, int H, int W, int C,
                                      ebsdvae_stream_t stream) {
  EV_REQUIRE(x && w0 && part && B > 0 && C == FIRST_C,
             "conv_first_fwd: bad args (C must be %d)", FIRST_C);
  const int th = first_rows(W);
  EV_REQUIRE(th > 0 && FIRST_PX % W == 0 && H % th == 0,
             "conv_first_fwd: %dx%d unsupported (W must divide %d)", H, W, FIRST_PX);
  hipLaunchKernelGGL(conv_first_fwd_kernel, dim3(H / th, B), dim3(256),
                     (size_t)(th + 2) * (W + 2) * sizeof(float), (hipStream_t)stream, x, w0, b0, y,
                     (float2*)part, H, W, th);
  return evh::check_launch("conv_first_fwd");
}

extern "C" int ebsdvae_conv3x3_cout1_fwd(const float* src, const float* src_stats, int src_mode,
                                         const float* w, const float* bias, float* out, int flip,
                                         int B, int H, int W, int cin, ebsdvae_stream_t stream) {
  EdgeGeom g;
  EV_REQUIRE(src && w && out && B > 0, "conv3x3_cout1_fwd: null pointer");
  EV_REQUIRE(cin == 32, "conv3x3_cout1_fwd: cin=%d unsupported (32)", cin);
  EV_REQUIRE(src_mode == ACT_RAW || src_mode == ACT_UP || src_stats, "conv3x3_cout1_fwd: NORM needs stats");
  if ((src_mode == ACT_RAW || src_mode == ACT_NORM) && W >= 64 && W <= 256 && W % 64 == 0 &&
      H % ROWS_TH == 0) {
    const size_t lds = ((size_t)9 * (W + 2) + (size_t)W * ROWS_PS) * sizeof(float);
    auto k = src_mode == ACT_NORM ? (flip ? conv_cout1_rows_kernel<true, true> : conv_cout1_rows_kernel<true, false>)
                                  : (flip ? conv_cout1_rows_kernel<false, true> : conv_cout1_rows_kernel<false, false>);
    hipLaunchKernelGGL(k, dim3(B * (H / ROWS_TH)), dim3(W), lds, (hipStream_t)stream, src,
                       (const float2*)src_stats, w, bias, out, H, W);
    return evh::check_launch("conv3x3_cout1_fwd");
  }
  EV_REQUIRE(edge_geom(H, W, &g), "conv3x3_cout1_fwd: unsupported shape %dx%d", H, W);
  const int tiles = ((B + g.NI - 1) / g.NI) * (H / g.TH) * (W / g.TW);
  const size_t lds = (size_t)g.NI * (g.TH + 2) * (g.TW + 2) * 33 * sizeof(float);
  hipLaunchKernelGGL(conv_cout1_fwd_kernel<32>, dim3(tiles), dim3(256), lds, (hipStream_t)stream,
                     src, (const float2*)src_stats, src_mode, w, bias, out, flip, B, H, W, g);
  return evh::check_launch("conv3x3_cout1_fwd");
}

extern "C" int ebsdvae_conv3x3_cout1_dgrad(const float* g1, const float* w, float* gin, int B,
                                           int H, int W, int cin, ebsdvae_stream_t stream) {
  EdgeGeom g;
  EV_REQUIRE(g1 && w && gin && B > 0, "conv3x3_cout1_dgrad: null pointer");
  EV_REQUIRE(cin == 32, "conv3x3_cout1_dgrad: cin=%d unsupported (32)", cin);
  EV_REQUIRE(edge_geom(H, W, &g), "conv3x3_cout1_dgrad: unsupported shape %dx%d", H, W);
  const int tiles = ((B + g.NI - 1) / g.NI) * (H / g.TH) * (W / g.TW);
  const size_t lds = (size_t)g.NI * (g.TH + 2) * (g.TW + 2) * sizeof(float);
  hipLaunchKernelGGL(conv_cout1_dgrad_kernel<32>, dim3(tiles), dim3(256), lds, (hipStream_t)stream,
                     g1, w, gin, B, H, W, g);
  return evh::check_launch("conv3x3_cout1_dgrad");
}

extern "C" int ebsdvae_conv_first_stats(const float* x, const float* w0, const float* b0, float* st,
                                        int B, int H, int W, int C, ebsdvae_stream_t stream) {
  EV_REQUIRE(x && w0 && st && B > 0 && C == FIRST_C, "conv_first_stats: bad args (C must be %d)", FIRST_C);
  EV_REQUIRE(W >= 8 && W <= 256 && 256 % W == 0 && H % FG_CH == 0 && ev_dim_ok(H),
             "conv_first_stats: %dx%d unsupported (W must divide 256, H a multiple of %d)", H, W, FG_CH);
  const size_t lds = (size_t)(FG_CH + 2) * (W + 2) * sizeof(float);
  const size_t lds_fold = (size_t)5 * FG_NS * sizeof(double);
  hipLaunchKernelGGL(first_gram_kernel, dim3(B), dim3(256), lds > lds_fold ? lds : lds_fold,
                     (hipStream_t)stream, x, w0, b0, (float2*)st, C, H, W);
  return evh::check_launch("conv_first_stats");
}
