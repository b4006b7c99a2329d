// InstanceNorm2d (affine=False, eps 1e-5, biased variance) + LeakyReLU(0.02) + the 2x2
// max-pool / nearest x2 upsample adjoints, for every block of latice/model.py:93-147.
//
// Forward: the conv epilogue already produced per-tile {mean, M2}; in_stats_finalize
// merges them (Chan's parallel formula) into {mean, rstd} per (b, c).  Nothing else runs
// in the forward: consumers apply the normalisation while staging their input.
//
// Backward of one block (a = lrelu(xhat), xhat = (y - mean) * rstd, out = P(a)):
//   g_a    = P^T(g_next)                       (pool: to the first argmax; up: 2x2 sum)
//   g_xhat = g_a * (xhat > 0 ? 1 : 0.02)
//   g_y    = rstd * (g_xhat - mean(g_xhat) - xhat * mean(g_xhat * xhat))
// two HBM-bound passes (reduce, apply) over NHWC planes with float4 channel vectors; the
// plane sums use fixed-order two-level reductions (deterministic).
#include <hip/hip_ext.h>

#include "common.h"
#include "instnorm_fin.h"
#include "../../include/ebsdvae.h"

namespace ev {

// One workgroup per pattern b (in_stats_finalize_image, instnorm_fin.h).
__global__ __launch_bounds__(256) void in_stats_finalize_kernel(const float2* __restrict__ part,
                                                                float2* __restrict__ st, int C,
                                                                int T, float n) {
  __shared__ float sm[3 * 256];
  in_stats_finalize_image(part, st, C, T, n, blockIdx.x, threadIdx.x, sm);
}

__global__ void act_apply_kernel(const float* __restrict__ src, const float2* __restrict__ st,
                                 int mode, float* __restrict__ out, int B, int H, int W, int C) {
  const size_t n4 = (size_t)B * H * W * (C / 4);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4;
       i += (size_t)gridDim.x * blockDim.x) {
    const int cg = (int)(i % (C / 4));
    size_t p = i / (C / 4);
    const int w = (int)(p % W);
    p /= W;
    const int h = (int)(p % H);
    const int b = (int)(p / H);
    st4(out + i * 4, load_act4(src, st, mode, b, h, w, cg * 4, H, W, C));
  }
}

__global__ void upsample2_bwd_kernel(const float* __restrict__ g, float* __restrict__ out, int B,
                                     int H, int W, int C) {
  const size_t n4 = (size_t)B * H * W * (C / 4);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4;
       i += (size_t)gridDim.x * blockDim.x) {
    const int cg = (int)(i % (C / 4));
    size_t p = i / (C / 4);
    const int w = (int)(p % W);
    p /= W;
    const int h = (int)(p % H);
    const int b = (int)(p / H);
    const float* s = g + (((size_t)b * 2 * H + 2 * h) * 2 * W + 2 * w) * C + cg * 4;
    const size_t rs = (size_t)2 * W * C;
    float4 a = ld4(s), bb = ld4(s + C), c = ld4(s + rs), d = ld4(s + rs + C);
    st4(out + i * 4, make_float4(a.x + bb.x + c.x + d.x, a.y + bb.y + c.y + d.y,
                                 a.z + bb.z + c.z + d.z, a.w + bb.w + c.w + d.w));
  }
}

// per-tile geometry of the backward passes: T tiles per image, each a band of rows
static int in_bwd_tiles_host(int H, int W) {
  int T = (H * W) / 1024;
  if (T < 1) T = 1;
  while (T > 1 && (H % T || ((H / T) & 1))) T >>= 1;   // row bands with an even row count
  return T;
}

// HIN (apply only): gnext is h = g * lrelu'(xhat) at the routed pixel -- the output of a fused
// input-gradient conv (conv_common.h) -- so the LeakyReLU factor is already in it
template <bool APPLY, bool HIN = false>
__global__ __launch_bounds__(256) void in_bwd_kernel(
    const float* __restrict__ gnext, int pmode, const float* __restrict__ y,
    const float2* __restrict__ st, const float2* __restrict__ bst, double2* __restrict__ part,
    float* __restrict__ gy, int H, int W, int C, int T, float* __restrict__ gmax) {
  __shared__ double red[2][4][256];
  float amax = 0.f;   // APPLY: max |gy| of this thread (gmax: per-tile maxima for the f16 dgrad)
  const int tile = blockIdx.x, b = blockIdx.y;
  const int CG = C >> 2;
  const int tid = threadIdx.x;
  const int cg = tid % CG, pr = tid / CG, NPR = 256 / CG;
  const int c = cg * 4;
  const int rows = H / T;
  const float2* sp = st + (size_t)b * C + c;
  const float2 s0 = sp[0], s1 = sp[1], s2 = sp[2], s3 = sp[3];
  const float mean[4] = {s0.x, s1.x, s2.x, s3.x};
  const float rstd[4] = {s0.y, s1.y, s2.y, s3.y};
  float m1[4] = {0.f, 0.f, 0.f, 0.f}, m2[4] = {0.f, 0.f, 0.f, 0.f};
  if (APPLY) {
    const float2* bp = bst + (size_t)b * C + c;
#pragma unroll
    for (int k = 0; k < 4; ++k) { m1[k] = bp[k].x; m2[k] = bp[k].y; }
  }
  double a1[4] = {0.0, 0.0, 0.0, 0.0}, a2[4] = {0.0, 0.0, 0.0, 0.0};
  const float* yb = y + (size_t)b * H * W * C;
  float* gyb = APPLY ? gy + (size_t)b * H * W * C : nullptr;

  if (pmode == P_POOL) {
    const int W2 = W >> 1, H2 = H >> 1;
    const int q0 = tile * (rows >> 1) * W2, q1 = q0 + (rows >> 1) * W2;
    const float* gnb = gnext + (size_t)b * H2 * W2 * C;
#pragma unroll 2
    for (int q = q0 + pr; q < q1; q += NPR) {
      const int h2 = q / W2, w2 = q - h2 * W2;
      const float4 g4 = APPLY ? ld4_nt(gnb + (size_t)q * C + c) : ld4(gnb + (size_t)q * C + c);
      const float gv[4] = {g4.x, g4.y, g4.z, g4.w};
      const size_t p00 = ((size_t)(2 * h2) * W + 2 * w2) * C + c;
      const size_t poff[4] = {p00, p00 + C, p00 + (size_t)W * C, p00 + (size_t)W * C + C};
      float4 yv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) yv[k] = APPLY ? ld4_nt(yb + poff[k]) : ld4(yb + poff[k]);
      float xh[4][4];  // [window slot][channel]
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        xh[k][0] = (yv[k].x - mean[0]) * rstd[0];
        xh[k][1] = (yv[k].y - mean[1]) * rstd[1];
        xh[k][2] = (yv[k].z - mean[2]) * rstd[2];
        xh[k][3] = (yv[k].w - mean[3]) * rstd[3];
      }
      int arg[4];
#pragma unroll
      for (int ch = 0; ch < 4; ++ch) {
        // first maximum of lrelu(xhat) in window order (0,0),(0,1),(1,0),(1,1)
        float best = lrelu(xh[0][ch]);
        int a = 0;
#pragma unroll
        for (int k = 1; k < 4; ++k) {
          const float f = lrelu(xh[k][ch]);
          if (f > best) { best = f; a = k; }
        }
        arg[ch] = a;
      }
      if (!APPLY) {
#pragma unroll
        for (int ch = 0; ch < 4; ++ch) {
          const float x = xh[arg[ch]][ch];
          const float gx = gv[ch] * slope(x);
          a1[ch] += (double)gx;
          a2[ch] = fma((double)gx, (double)x, a2[ch]);
        }
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float o[4];
#pragma unroll
          for (int ch = 0; ch < 4; ++ch) {
            const float x = xh[k][ch];
            const float gx = (arg[ch] == k) ? (HIN ? gv[ch] : gv[ch] * slope(x)) : 0.f;
            o[ch] = rstd[ch] * (gx - m1[ch] - x * m2[ch]);
            amax = fmaxf(amax, fabsf(o[ch]));
          }
          st4(gyb + poff[k], make_float4(o[0], o[1], o[2], o[3]));
        }
      }
    }
  } else {
    const int p0 = tile * rows * W, p1 = p0 + rows * W;
    constexpr int UNR = APPLY ? 8 : 4;   // loads in flight per thread (the apply streams 3 tensors)
#pragma unroll UNR
    for (int p = p0 + pr; p < p1; p += NPR) {
      float4 g4;
      if (pmode == P_ID) {
        g4 = APPLY ? ld4_nt(gnext + ((size_t)b * H * W + p) * C + c) : ld4(gnext + ((size_t)b * H * W + p) * C + c);
      } else {  // P_UP: gnext at (2H, 2W)
        const int h = p / W, w = p - h * W;
        const float* s = gnext + (((size_t)b * 2 * H + 2 * h) * 2 * W + 2 * w) * C + c;
        const size_t rs = (size_t)2 * W * C;
        const float4 u0 = ld4(s), u1 = ld4(s + C), u2 = ld4(s + rs), u3 = ld4(s + rs + C);
        g4 = make_float4(u0.x + u1.x + u2.x + u3.x, u0.y + u1.y + u2.y + u3.y,
                         u0.z + u1.z + u2.z + u3.z, u0.w + u1.w + u2.w + u3.w);
      }
      const float4 y4 = APPLY ? ld4_nt(yb + (size_t)p * C + c) : ld4(yb + (size_t)p * C + c);
      const float gv[4] = {g4.x, g4.y, g4.z, g4.w};
      const float yy[4] = {y4.x, y4.y, y4.z, y4.w};
      float o[4];
#pragma unroll
      for (int ch = 0; ch < 4; ++ch) {
        const float x = (yy[ch] - mean[ch]) * rstd[ch];
        const float gx = HIN ? gv[ch] : gv[ch] * slope(x);
        if (!APPLY) {
          a1[ch] += (double)gx;
          a2[ch] = fma((double)gx, (double)x, a2[ch]);
        } else {
          o[ch] = rstd[ch] * (gx - m1[ch] - x * m2[ch]);
          amax = fmaxf(amax, fabsf(o[ch]));
        }
      }
      if (APPLY) st4(gyb + (size_t)p * C + c, make_float4(o[0], o[1], o[2], o[3]));
    }
  }
  if (APPLY && gmax) {   // block-uniform: one maximum per (image, tile)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) amax = fmaxf(amax, __shfl_xor(amax, off));
    __shared__ float wmax[4];
    if ((tid & 63) == 0) wmax[tid >> 6] = amax;
    __syncthreads();
    if (tid == 0) gmax[(size_t)b * T + tile] = fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]));
  }
  if (!APPLY) {
#pragma unroll
    for (int k = 0; k < 4; ++k) { red[0][k][tid] = a1[k]; red[1][k][tid] = a2[k]; }
    __syncthreads();
    if (tid < CG) {
      double u[4], v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) { u[k] = red[0][k][tid]; v[k] = red[1][k][tid]; }
      for (int r = 1; r < NPR; ++r) {
#pragma unroll
        for (int k = 0; k < 4; ++k) { u[k] += red[0][k][r * CG + tid]; v[k] += red[1][k][r * CG + tid]; }
      }
      double2* o = part + ((size_t)b * T + tile) * C + c;
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = make_double2(u[k], v[k]);
    }
  }
}

// One workgroup per pattern b (in_bwd_finalize_image, instnorm_fin.h).
__global__ __launch_bounds__(256) void in_bwd_finalize_kernel(const double2* __restrict__ part,
                                                              float2* __restrict__ bst, int C,
                                                              int T, double inv_hw) {
  __shared__ double sm[2 * 256];
  in_bwd_finalize_image(part, bst, C, T, inv_hw, blockIdx.x, threadIdx.x, sm);
}

// ------------------------------------------------------------------ network-end fusions
// (C == 32 planes, row-band tiles as in_bwd_kernel; thread = (channel group cg, pixel row pr))
//
// FINAL: the block feeding the last conv nn.Conv2d(32,1) (latice/model.py:147-148).  Its
// output gradient g_a[q][c] = sum_tap g1[q - d(tap)] * w14[c][tap] is recomputed from the
// 1-channel logit gradient g1 (never materialised), and the reduce pass also accumulates
// that conv's weight/bias gradient dW14[c][tap] = sum_q g1[q - d(tap)] * a[q][c].
// FIRST: the block of the first conv nn.Conv2d(1,32) (latice/model.py:110).  Its apply pass
// accumulates dW0[c][tap] = sum_p gy[p][c] * x[p + d(tap)] and db0 directly, so gy is never
// written (the input x needs no gradient).
// Partials are per (b, tile) "slice" in the [slice][tap][co][ci] layout of
// ebsdvae_wgrad_reduce.
// FUSE_FIRST_RC: FUSE_FIRST with y0 recomputed from the staged x band (first_conv_px, the
// forward's fma chain: conv_first_fwd_kernel) instead of read -- 512 MB less per step at B=256
enum EdgeFuse : int { FUSE_FINAL = 1, FUSE_FIRST = 2, FUSE_FIRST_RC = 3 };
constexpr int EDGE_NB_ITEMS = 8;   // staged neighbour-source items per thread (<= 2048 per band)

EV_DEVINL void wave_fold8(float& v) {  // sum over the 8 pixel rows of a wave (lanes l, l^8, ...)
  v += __shfl_xor(v, 8, 64);
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
}

// HIN (FIRST apply only): gsrc is h (the fused input gradient's output), not g
template <int FUSE, bool APPLY, bool HIN = false>
__global__ __launch_bounds__(256) void in_bwd_edge_kernel(
    const float* __restrict__ gsrc, const float* __restrict__ w14, const float* __restrict__ y,
    const float2* __restrict__ st, const float2* __restrict__ bst, const float* __restrict__ x,
    double2* __restrict__ part, float* __restrict__ wpart, float* __restrict__ bpart,
    float* __restrict__ gy, int H, int W, int T, float* __restrict__ gmax,
    const float* __restrict__ b0 = nullptr) {
  constexpr int C = 32, CG = 8, NPR = 32;
  constexpr bool RC = FUSE == FUSE_FIRST_RC;
  constexpr int FUSE_ = RC ? FUSE_FIRST : FUSE;   // RC is FIRST with y recomputed
  float amax = 0.f;   // FINAL apply: max |gy| of this thread (gmax: per-tile maxima, f16 convs)
  __shared__ double red[2][4][256];
  __shared__ float wred[4][CG][37];
  const int tile = blockIdx.x, b = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cg = tid % CG, pr = tid / CG;
  const int c = cg * 4;
  const int rows = H / T;
  const float2* sp = st + (size_t)b * C + c;
  float mean[4], rstd[4], m1[4] = {0.f, 0.f, 0.f, 0.f}, m2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 4; ++k) { const float2 v = sp[k]; mean[k] = v.x; rstd[k] = v.y; }
  if (APPLY) {
    const float2* bp = bst + (size_t)b * C + c;
#pragma unroll
    for (int k = 0; k < 4; ++k) { m1[k] = bp[k].x; m2[k] = bp[k].y; }
  }
  // FINAL: w14 (1, 32, 3, 3); RC: w0 (32, 1, 3, 3) and b0 -- as channel pairs (2k, 2k+1) of
  // this thread's 4 channels, for v_pk_fma_f32
  pkf2 wv2[2][9], bb2[2];
  if (FUSE_ == FUSE_FINAL || RC) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
#pragma unroll
      for (int t = 0; t < 9; ++t) wv2[k][t] = pk2(w14[(c + 2 * k) * 9 + t], w14[(c + 2 * k + 1) * 9 + t]);
      bb2[k] = (RC && b0) ? pk2(b0[c + 2 * k], b0[c + 2 * k + 1]) : pk2(0.f, 0.f);
    }
  }
  double a1[4] = {0.0, 0.0, 0.0, 0.0}, a2[4] = {0.0, 0.0, 0.0, 0.0};
  pkf2 wacc2[2][9];   // weight-gradient partials of the channel pairs
  float bacc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int t = 0; t < 9; ++t) wacc2[k][t] = pk2(0.f, 0.f);
  const float* yb = y + (size_t)b * H * W * C;
  // the 1-channel neighbour source (FINAL: g1, FIRST: x) of this row band plus its 1-pixel
  // halo, staged once in LDS with coalesced loads (zero padding at the image border)
  const float* src1 = ((FUSE_ == FUSE_FINAL) ? gsrc : x) + (size_t)b * H * W;
  extern __shared__ float nbs[];   // (rows + 2) x (W + 2)
  const int r0 = tile * rows, WP = W + 2;
  {
    // all of this thread's loads in flight at once, then the LDS writes (host: <= 8 each)
    const int nbn = (rows + 2) * WP;
    float nv[EDGE_NB_ITEMS];
#pragma unroll
    for (int k = 0; k < EDGE_NB_ITEMS; ++k) {
      const int i = tid + 256 * k;
      const int r = i / WP, cc = i - r * WP;
      const int gh = r0 - 1 + r, gw = cc - 1;
      nv[k] = (i < nbn && gh >= 0 && gh < H && gw >= 0 && gw < W) ? src1[gh * W + gw] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < EDGE_NB_ITEMS; ++k)
      if (tid + 256 * k < nbn) nbs[tid + 256 * k] = nv[k];
  }
  __syncthreads();
  const int p0 = tile * rows * W, p1 = p0 + rows * W;
  // software-pipelined over groups of U pixels per thread: the next group's y (and, FIRST,
  // gnext) loads are issued before this group is processed
  // the FINAL reduce is VALU-heavy (9-tap recompute + 36 weight-gradient FMAs per pixel)
  // and register-bound: 2 pixels per group, loaded at the group's start, no prefetch
  constexpr bool PF = !(FUSE_ == FUSE_FINAL && !APPLY);
  constexpr int U = PF ? 4 : 2;
  constexpr bool LG = FUSE_ == FUSE_FIRST;
  // single-use stream reads: non-temporal (the reduce-only FINAL pass keeps the default)
  auto ldy = [&](int p) {
    return (!RC && p < p1) ? (APPLY ? ld4_nt(yb + (size_t)p * C + c) : ld4(yb + (size_t)p * C + c))
                           : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  auto ldg = [&](int p) {
    return (LG && p < p1) ? ld4_nt(gsrc + ((size_t)b * H * W + p) * C + c)
                          : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  // two register sets, swapped by a two-group loop (no copies between groups)
  float4 yA[U], gA[U], yB[U], gB[U];
  if (PF) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (!RC) yA[u] = ldy(p0 + pr + u * NPR);
      gA[u] = ldg(p0 + pr + u * NPR);
    }
  }
  // the pixel's (row, column), advanced by NPR per pixel (W is a multiple of NPR = 32, so a
  // step wraps at most once): no per-pixel division
  int ph = (p0 + pr) / W, pw = (p0 + pr) - ph * W;
  auto group = [&](int pg, float4 (&ycur)[U], float4 (&gcur)[U], float4 (&ynxt)[U],
                   float4 (&gnxt)[U]) EV_LAMBDA_INLINE {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (PF) {
        if constexpr (!RC) ynxt[u] = ldy(pg + (U + u) * NPR);
        gnxt[u] = ldg(pg + (U + u) * NPR);
      } else {
        if constexpr (!RC) ycur[u] = ldy(pg + u * NPR);
        gcur[u] = ldg(pg + u * NPR);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
    const int p = pg + u * NPR;
    const int h = ph, w = pw;
    pw += NPR;
    if (pw >= W) { pw -= W; ++ph; }
    if (p >= p1) break;
    float nb[9];   // FINAL: g1[q - d(tap)] ; FIRST: x[p + d(tap)]
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int kh = t / 3, kw = t % 3;
      const int lr = (FUSE_ == FUSE_FINAL) ? h - r0 + 2 - kh : h - r0 + kh;
      const int lc = (FUSE_ == FUSE_FINAL) ? w + 2 - kw : w + kw;
      nb[t] = nbs[lr * WP + lc];
    }
    float ga[4];
    if (FUSE_ == FUSE_FINAL) {
      // two channels per v_pk_fma_f32 (per channel the same fma chain)
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        pkf2 s = pk2(0.f, 0.f);
#pragma unroll
        for (int t = 0; t < 9; ++t) s = pkfma(pk2(nb[t], nb[t]), wv2[k][t], s);
        ga[2 * k] = s.x;
        ga[2 * k + 1] = s.y;
      }
      if (!APPLY && cg == 0) bacc[0] += nb[4];   // g1[p] itself (centre tap): db14
    } else {
      const float4 g4 = gcur[u];
      ga[0] = g4.x; ga[1] = g4.y; ga[2] = g4.z; ga[3] = g4.w;
    }
    float yy[4];
    if constexpr (!RC) {
      const float4 y4 = ycur[u];
      yy[0] = y4.x; yy[1] = y4.y; yy[2] = y4.z; yy[3] = y4.w;
    } else {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const pkf2 y2 = first_conv_px2(nb, wv2[k], bb2[k]);
        yy[2 * k] = y2.x;
        yy[2 * k + 1] = y2.y;
      }
    }
    float o[4], av[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float xh = (yy[k] - mean[k]) * rstd[k];
      const float gx = (HIN && FUSE_ == FUSE_FIRST) ? ga[k] : ga[k] * slope(xh);
      if (!APPLY) {
        a1[k] += (double)gx;
        a2[k] = fma((double)gx, (double)xh, a2[k]);
        av[k] = lrelu(xh);
      } else {
        o[k] = rstd[k] * (gx - m1[k] - xh * m2[k]);
        if (FUSE_ == FUSE_FIRST) bacc[k] += o[k];
      }
    }
    // weight-gradient partials, two channels per v_pk_fma_f32 (per channel the same chain)
    if ((FUSE_ == FUSE_FINAL && !APPLY) || (FUSE_ == FUSE_FIRST && APPLY)) {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const pkf2 f = (FUSE_ == FUSE_FINAL) ? pk2(av[2 * k], av[2 * k + 1]) : pk2(o[2 * k], o[2 * k + 1]);
#pragma unroll
        for (int t = 0; t < 9; ++t) wacc2[k][t] = pkfma(pk2(nb[t], nb[t]), f, wacc2[k][t]);
      }
    }
    if (APPLY && FUSE_ == FUSE_FINAL) {
      st4(gy + ((size_t)b * H * W + p) * C + c, make_float4(o[0], o[1], o[2], o[3]));
      amax = fmaxf(fmaxf(amax, fmaxf(fabsf(o[0]), fabsf(o[1]))), fmaxf(fabsf(o[2]), fabsf(o[3])));
    }
    }
  };
  for (int pg = p0 + pr; pg < p1; pg += 2 * U * NPR) {
    group(pg, yA, gA, yB, gB);
    if (pg + U * NPR >= p1) break;
    group(pg + U * NPR, yB, gB, yA, gA);
  }
  const int slice = b * T + tile;
  if (FUSE_ == FUSE_FINAL && APPLY && gmax) {   // block-uniform: one maximum per (image, tile)
    __shared__ float wmax[4];
    for (int off = 32; off > 0; off >>= 1) amax = fmaxf(amax, __shfl_xor(amax, off));
    if (lane == 0) wmax[wave] = amax;
    __syncthreads();
    if (tid == 0) gmax[slice] = fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]));
  }
  if (!APPLY) {   // InstanceNorm-backward plane partials (double, fixed order): the pixel
                  // lanes of a wave by a shuffle tree, then the 4 waves through LDS
    double* rd = &red[0][0][0];   // [4 waves][C][2]
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      double u = a1[k], v = a2[k];
#pragma unroll
      for (int o = CG; o < 64; o <<= 1) { u += __shfl_xor(u, o, 64); v += __shfl_xor(v, o, 64); }
      if (lane < CG) { rd[(wave * C + lane * 4 + k) * 2] = u; rd[(wave * C + lane * 4 + k) * 2 + 1] = v; }
    }
    __syncthreads();
    if (tid < C) {
      double u = 0.0, v = 0.0;
#pragma unroll
      for (int wv = 0; wv < 4; ++wv) { u += rd[(wv * C + tid) * 2]; v += rd[(wv * C + tid) * 2 + 1]; }
      part[(size_t)slice * C + tid] = make_double2(u, v);
    }
  }
  if ((FUSE_ == FUSE_FINAL && !APPLY) || (FUSE_ == FUSE_FIRST && APPLY)) {
    // fold the 36 weight partials (+ bias) of the block: in-wave over its 8 pixel rows,
    // then across the 4 waves in order
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        float v = (k & 1) ? wacc2[k >> 1][t].y : wacc2[k >> 1][t].x;
        wave_fold8(v);
        if (lane < CG) wred[wave][lane][k * 9 + t] = v;
      }
      float v = bacc[k];
      wave_fold8(v);
      // bias: FINAL keeps one scalar (k == 0, cg == 0 lane); FIRST keeps 4 per channel group
      if (lane < CG) {
        if (FUSE_ == FUSE_FINAL && k == 0) wred[wave][lane][36] = v;
        if (FUSE_ == FUSE_FIRST) bacc[k] = v;
      }
    }
    __syncthreads();
    // FINAL: Cout = 1, Cin = 32 -> [slice][tap][0][ci];  FIRST: Cout = 32, Cin = 1 ->
    // [slice][tap][co][0]; both are offset t * 32 + channel
    for (int i = tid; i < CG * 36; i += 256) {
      const int g = i / 36, e = i % 36;   // channel group, (k, tap)
      const float s = wred[0][g][e] + wred[1][g][e] + wred[2][g][e] + wred[3][g][e];
      const int k = e / 9, t = e % 9;
      wpart[((size_t)slice * 9 + t) * 32 + g * 4 + k] = s;
    }
    if (FUSE_ == FUSE_FINAL && tid == 0)
      bpart[slice] = wred[0][0][36] + wred[1][0][36] + wred[2][0][36] + wred[3][0][36];
    if (FUSE_ == FUSE_FIRST) {
      __syncthreads();
      if (lane < CG) {
#pragma unroll
        for (int k = 0; k < 4; ++k) wred[wave][lane][k] = bacc[k];
      }
      __syncthreads();
      if (tid < C) {
        const int g = tid / 4, k = tid % 4;
        bpart[(size_t)slice * 32 + tid] = wred[0][g][k] + wred[1][g][k] + wred[2][g][k] + wred[3][g][k];
      }
    }
  }
}

// dynamic LDS of in_bwd_edge_kernel: the 1-channel source of one row band + halo
static size_t edge_lds(int H, int W, int T) { return (size_t)(H / T + 2) * (W + 2) * sizeof(float); }
// (W a multiple of the 32 pixel rows of a block: the kernel steps its pixel coordinates by 32)
static bool edge_ok(int H, int W, int T) { return W % 32 == 0 && (H / T + 2) * (W + 2) <= 256 * EDGE_NB_ITEMS; }

static int grid_for(size_t n4) {
  size_t g = (n4 + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace ev

using namespace ev;

extern "C" int ebsdvae_in_stats_finalize(const float* part, float* stats, int B, int C, int tiles,
                                         int n_per_tile, ebsdvae_stream_t stream) {
  EV_REQUIRE(part && stats && B > 0 && C > 0 && tiles > 0 && C <= 256 && (256 % C) == 0,
             "in_stats_finalize: bad args (C=%d)", C);
  hipLaunchKernelGGL(in_stats_finalize_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream,
                     (const float2*)part, (float2*)stats, C, tiles, (float)n_per_tile);
  return evh::check_launch("in_stats_finalize");
}

extern "C" int ebsdvae_act_apply(const float* src, const float* src_stats, int src_mode,
                                 float* out, int B, int H, int W, int C,
                                 ebsdvae_stream_t stream) {
  EV_REQUIRE(src && out && C % 4 == 0, "act_apply: bad args (C=%d)", C);
  EV_REQUIRE(src_mode == ACT_RAW || src_mode == ACT_UP || src_stats, "act_apply: NORM needs stats");
  const size_t n4 = (size_t)B * H * W * (C / 4);
  hipLaunchKernelGGL(act_apply_kernel, dim3(grid_for(n4)), dim3(256), 0, (hipStream_t)stream, src,
                     (const float2*)src_stats, src_mode, out, B, H, W, C);
  return evh::check_launch("act_apply");
}

extern "C" int ebsdvae_upsample2_bwd(const float* g, float* out, int B, int H, int W, int C,
                                     ebsdvae_stream_t stream) {
  EV_REQUIRE(g && out && C % 4 == 0, "upsample2_bwd: bad args");
  const size_t n4 = (size_t)B * H * W * (C / 4);
  hipLaunchKernelGGL(upsample2_bwd_kernel, dim3(grid_for(n4)), dim3(256), 0, (hipStream_t)stream,
                     g, out, B, H, W, C);
  return evh::check_launch("upsample2_bwd");
}

extern "C" int ebsdvae_in_bwd_tiles(int H, int W, int C) {
  (void)C;
  if (!ev_dim_ok(H) || !ev_dim_ok(W)) return -1;
  return in_bwd_tiles_host(H, W);
}

extern "C" int ebsdvae_in_bwd_reduce(const float* gnext, int pmode, const float* y,
                                     const float* stats, double* part, int B, int H, int W, int C,
                                     ebsdvae_stream_t stream) {
  EV_REQUIRE(gnext && y && stats && part, "in_bwd_reduce: null pointer");
  EV_REQUIRE(pmode >= 0 && pmode <= 2 && C % 4 == 0 && C <= 1024 && (256 % (C / 4)) == 0,
             "in_bwd_reduce: bad pmode/C");
  EV_REQUIRE(pmode != P_POOL || ((H | W) & 1) == 0, "in_bwd_reduce: pool needs even H, W");
  const int T = in_bwd_tiles_host(H, W);
  hipLaunchKernelGGL(in_bwd_kernel<false>, dim3(T, B), dim3(256), 0, (hipStream_t)stream, gnext,
                     pmode, y, (const float2*)stats, (const float2*)nullptr, (double2*)part,
                     (float*)nullptr, H, W, C, T, (float*)nullptr);
  return evh::check_launch("in_bwd_reduce");
}

extern "C" int ebsdvae_in_bwd_finalize(const double* part, float* bstats, int B, int C, int tiles,
                                       int HW, ebsdvae_stream_t stream) {
  EV_REQUIRE(part && bstats, "in_bwd_finalize: null pointer");
  EV_REQUIRE(C > 0 && C <= 256 && 256 % C == 0 && tiles > 0, "in_bwd_finalize: C=%d unsupported", C);
  hipLaunchKernelGGL(in_bwd_finalize_kernel, dim3(B), dim3(256), 0, (hipStream_t)stream,
                     (const double2*)part, (float2*)bstats, C, tiles, 1.0 / (double)HW);
  return evh::check_launch("in_bwd_finalize");
}

// the apply pass keeps no per-tile partials: split the planes finer than the reduce so
// small maps still put >= 2048 workgroups (8 per CU) in flight
static int in_bwd_apply_tiles_host(int B, int H, int W) {
  int T = in_bwd_tiles_host(H, W);
  if (H <= 0) return T;
  while (B * T < 2048 && H % (2 * T) == 0 && ((H / (2 * T)) & 1) == 0) T *= 2;
  return T;
}

extern "C" int ebsdvae_in_bwd_apply_tiles(int B, int H, int W, int C) {
  (void)C;
  if (B <= 0 || !ev_dim_ok(H) || !ev_dim_ok(W)) return -1;
  return in_bwd_apply_tiles_host(B, H, W);
}

extern "C" int ebsdvae_in_bwd_apply_max(const float* gnext, int pmode, const float* y,
                                        const float* stats, const float* bstats, float* gy,
                                        float* gmax, int B, int H, int W, int C,
                                        ebsdvae_stream_t stream) {
  EV_REQUIRE(gnext && y && stats && bstats && gy, "in_bwd_apply: null pointer");
  EV_REQUIRE(pmode >= 0 && pmode <= 2 && C % 4 == 0 && (256 % (C / 4)) == 0, "in_bwd_apply: bad pmode/C");
  const int T = in_bwd_apply_tiles_host(B, H, W);
  // an armed side-stream fork (ebsdvae_fork_arm) rides on this launch's completion signal
  if (hipEvent_t fe = evh::take_fork_event()) {
    hipExtLaunchKernelGGL(in_bwd_kernel<true>, dim3(T, B), dim3(256), 0, (hipStream_t)stream, nullptr,
                          fe, 0, gnext, pmode, y, (const float2*)stats, (const float2*)bstats,
                          (double2*)nullptr, gy, H, W, C, T, gmax);
  } else {
    hipLaunchKernelGGL(in_bwd_kernel<true>, dim3(T, B), dim3(256), 0, (hipStream_t)stream, gnext,
                       pmode, y, (const float2*)stats, (const float2*)bstats, (double2*)nullptr, gy,
                       H, W, C, T, gmax);
  }
  return evh::check_launch("in_bwd_apply");
}

// the apply of a block whose output gradient came from a fused input-gradient conv, which
// writes h = g * lrelu'(xhat) (conv_common.h): the same pass without the LeakyReLU factor
extern "C" int ebsdvae_in_bwd_happly(const float* h, int pmode, const float* y, const float* stats,
                                     const float* bstats, float* gy, float* gmax, int B, int H,
                                     int W, int C, ebsdvae_stream_t stream) {
  EV_REQUIRE(h && y && stats && bstats && gy, "in_bwd_happly: null pointer");
  EV_REQUIRE(pmode >= 0 && pmode <= 2 && C % 4 == 0 && (256 % (C / 4)) == 0, "in_bwd_happly: bad pmode/C");
  const int T = in_bwd_apply_tiles_host(B, H, W);
  if (hipEvent_t fe = evh::take_fork_event()) {
    hipExtLaunchKernelGGL((in_bwd_kernel<true, true>), dim3(T, B), dim3(256), 0, (hipStream_t)stream,
                          nullptr, fe, 0, h, pmode, y, (const float2*)stats, (const float2*)bstats,
                          (double2*)nullptr, gy, H, W, C, T, gmax);
  } else {
    hipLaunchKernelGGL((in_bwd_kernel<true, true>), dim3(T, B), dim3(256), 0, (hipStream_t)stream, h,
                       pmode, y, (const float2*)stats, (const float2*)bstats, (double2*)nullptr, gy,
                       H, W, C, T, gmax);
  }
  return evh::check_launch("in_bwd_happly");
}

extern "C" int ebsdvae_in_bwd_apply(const float* gnext, int pmode, const float* y,
                                    const float* stats, const float* bstats, float* gy, int B,
                                    int H, int W, int C, ebsdvae_stream_t stream) {
  return ebsdvae_in_bwd_apply_max(gnext, pmode, y, stats, bstats, gy, nullptr, B, H, W, C, stream);
}

// ------------------------------------------------------------------ network-end fusions (ABI)
extern "C" int ebsdvae_in_bwd_final_reduce(const float* g1, const float* w14, const float* y,
                                           const float* stats, double* part, float* wpart,
                                           float* bpart, int B, int H, int W, int C,
                                           ebsdvae_stream_t stream) {
  EV_REQUIRE(g1 && w14 && y && stats && part && wpart && bpart && C == 32,
             "in_bwd_final_reduce: bad args (C must be 32)");
  const int T = in_bwd_tiles_host(H, W);
  EV_REQUIRE(edge_ok(H, W, T), "in_bwd edge: %dx%d unsupported (W a multiple of 32, row band too large)", H, W);
  hipLaunchKernelGGL((in_bwd_edge_kernel<FUSE_FINAL, false>), dim3(T, B), dim3(256), edge_lds(H, W, T),
                     (hipStream_t)stream, g1, w14, y, (const float2*)stats, (const float2*)nullptr,
                     (const float*)nullptr, (double2*)part, wpart, bpart, (float*)nullptr, H, W, T,
                     (float*)nullptr);
  return evh::check_launch("in_bwd_final_reduce");
}

extern "C" int ebsdvae_in_bwd_final_apply(const float* g1, const float* w14, const float* y,
                                          const float* stats, const float* bstats, float* gy,
                                          int B, int H, int W, int C, ebsdvae_stream_t stream) {
  EV_REQUIRE(g1 && w14 && y && stats && bstats && gy && C == 32,
             "in_bwd_final_apply: bad args (C must be 32)");
  const int T = in_bwd_tiles_host(H, W);
  EV_REQUIRE(edge_ok(H, W, T), "in_bwd edge: %dx%d unsupported (W a multiple of 32, row band too large)", H, W);
  hipLaunchKernelGGL((in_bwd_edge_kernel<FUSE_FINAL, true>), dim3(T, B), dim3(256), edge_lds(H, W, T),
                     (hipStream_t)stream, g1, w14, y, (const float2*)stats, (const float2*)bstats,
                     (const float*)nullptr, (double2*)nullptr, (float*)nullptr, (float*)nullptr, gy,
                     H, W, T, (float*)nullptr);
  return evh::check_launch("in_bwd_final_apply");
}

extern "C" int ebsdvae_in_bwd_final_tiles(int H, int W) {
  return (ev_dim_ok(H) && ev_dim_ok(W)) ? in_bwd_tiles_host(H, W) : -1;
}

extern "C" int ebsdvae_in_bwd_final_apply_max(const float* g1, const float* w14, const float* y,
                                              const float* stats, const float* bstats, float* gy,
                                              float* gmax, int B, int H, int W, int C,
                                              ebsdvae_stream_t stream) {
  EV_REQUIRE(g1 && w14 && y && stats && bstats && gy && gmax && C == 32,
             "in_bwd_final_apply_max: bad args (C must be 32)");
  const int T = in_bwd_tiles_host(H, W);
  EV_REQUIRE(edge_ok(H, W, T), "in_bwd edge: %dx%d unsupported (W a multiple of 32, row band too large)", H, W);
  hipLaunchKernelGGL((in_bwd_edge_kernel<FUSE_FINAL, true>), dim3(T, B), dim3(256), edge_lds(H, W, T),
                     (hipStream_t)stream, g1, w14, y, (const float2*)stats, (const float2*)bstats,
                     (const float*)nullptr, (double2*)nullptr, (float*)nullptr, (float*)nullptr, gy,
                     H, W, T, gmax);
  return evh::check_launch("in_bwd_final_apply_max");
}

extern "C" int ebsdvae_in_bwd_first_apply_wgrad_rc(const float* gnext, const float* w0,
                                                   const float* b0, const float* stats,
                                                   const float* bstats, const float* x, float* wpart,
                                                   float* bpart, int B, int H, int W, int C,
                                                   ebsdvae_stream_t stream) {
  EV_REQUIRE(gnext && w0 && stats && bstats && x && wpart && bpart && C == 32,
             "in_bwd_first_apply_wgrad_rc: bad args (C must be 32)");
  const int T = in_bwd_tiles_host(H, W);
  EV_REQUIRE(edge_ok(H, W, T), "in_bwd edge: %dx%d unsupported (W a multiple of 32, row band too large)", H, W);
  hipLaunchKernelGGL((in_bwd_edge_kernel<FUSE_FIRST_RC, true>), dim3(T, B), dim3(256),
                     edge_lds(H, W, T), (hipStream_t)stream, gnext, w0, (const float*)nullptr,
                     (const float2*)stats, (const float2*)bstats, x, (double2*)nullptr, wpart, bpart,
                     (float*)nullptr, H, W, T, (float*)nullptr, b0);
  return evh::check_launch("in_bwd_first_apply_wgrad_rc");
}

// the first block's pass with h (a fused input gradient's output) instead of g
extern "C" int ebsdvae_in_bwd_first_happly_wgrad_rc(const float* h, const float* w0, const float* b0,
                                                    const float* stats, const float* bstats,
                                                    const float* x, float* wpart, float* bpart,
                                                    int B, int H, int W, int C,
                                                    ebsdvae_stream_t stream) {
  EV_REQUIRE(h && w0 && stats && bstats && x && wpart && bpart && C == 32,
             "in_bwd_first_happly_wgrad_rc: bad args (C must be 32)");
  const int T = in_bwd_tiles_host(H, W);
  EV_REQUIRE(edge_ok(H, W, T), "in_bwd edge: %dx%d unsupported (W a multiple of 32, row band too large)", H, W);
  hipLaunchKernelGGL((in_bwd_edge_kernel<FUSE_FIRST_RC, true, true>), dim3(T, B), dim3(256),
                     edge_lds(H, W, T), (hipStream_t)stream, h, w0, (const float*)nullptr,
                     (const float2*)stats, (const float2*)bstats, x, (double2*)nullptr, wpart, bpart,
                     (float*)nullptr, H, W, T, (float*)nullptr, b0);
  return evh::check_launch("in_bwd_first_happly_wgrad_rc");
}

extern "C" int ebsdvae_in_bwd_first_happly_wgrad(const float* h, const float* y, const float* stats,
                                                 const float* bstats, const float* x, float* wpart,
                                                 float* bpart, int B, int H, int W, int C,
                                                 ebsdvae_stream_t stream) {
  EV_REQUIRE(h && y && stats && bstats && x && wpart && bpart && C == 32,
             "in_bwd_first_happly_wgrad: bad args (C must be 32)");
  const int T = in_bwd_tiles_host(H, W);
  EV_REQUIRE(edge_ok(H, W, T), "in_bwd edge: %dx%d unsupported (W a multiple of 32, row band too large)", H, W);
  hipLaunchKernelGGL((in_bwd_edge_kernel<FUSE_FIRST, true, true>), dim3(T, B), dim3(256), edge_lds(H, W, T),
                     (hipStream_t)stream, h, (const float*)nullptr, y, (const float2*)stats,
                     (const float2*)bstats, x, (double2*)nullptr, wpart, bpart, (float*)nullptr, H, W,
                     T, (float*)nullptr);
  return evh::check_launch("in_bwd_first_happly_wgrad");
}

extern "C" int ebsdvae_in_bwd_first_apply_wgrad(const float* gnext, const float* y,
                                                const float* stats, const float* bstats,
                                                const float* x, float* wpart, float* bpart, int B,
                                                int H, int W, int C, ebsdvae_stream_t stream) {
  EV_REQUIRE(gnext && y && stats && bstats && x && wpart && bpart && C == 32,
             "in_bwd_first_apply_wgrad: bad args (C must be 32)");
  const int T = in_bwd_tiles_host(H, W);
  EV_REQUIRE(edge_ok(H, W, T), "in_bwd edge: %dx%d unsupported (W a multiple of 32, row band too large)", H, W);
  hipLaunchKernelGGL((in_bwd_edge_kernel<FUSE_FIRST, true>), dim3(T, B), dim3(256), edge_lds(H, W, T),
                     (hipStream_t)stream, gnext, (const float*)nullptr, y, (const float2*)stats,
                     (const float2*)bstats, x, (double2*)nullptr, wpart, bpart, (float*)nullptr, H, W,
                     T, (float*)nullptr);
  return evh::check_launch("in_bwd_first_apply_wgrad");
}
