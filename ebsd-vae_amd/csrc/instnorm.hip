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
#include "common.h"
#include "../../include/ebsdvae.h"

namespace ev {

enum PMode : int { P_ID = 0, P_POOL = 1, P_UP = 2 };

EV_DEVINL float slope(float xh) { return xh > 0.f ? 1.f : kSlope; }

__global__ void in_stats_finalize_kernel(const float2* __restrict__ part, float2* __restrict__ st,
                                         int B, int C, int T, float n) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B * C) return;
  const int b = e / C, c = e - b * C;
  const float2* p = part + (size_t)b * T * C + c;
  float m = 0.f;
  for (int t = 0; t < T; ++t) m += p[(size_t)t * C].x;
  m /= (float)T;
  float m2 = 0.f, dm = 0.f;
  for (int t = 0; t < T; ++t) {
    const float2 v = p[(size_t)t * C];
    m2 += v.y;
    const float d = v.x - m;
    dm = fmaf(d, d, dm);
  }
  const float var = (m2 + n * dm) / (n * (float)T);
  st[e] = make_float2(m, 1.0f / sqrtf(var + kInEps));
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

template <bool APPLY>
__global__ __launch_bounds__(256) void in_bwd_kernel(
    const float* __restrict__ gnext, int pmode, const float* __restrict__ y,
    const float2* __restrict__ st, const float2* __restrict__ bst, double2* __restrict__ part,
    float* __restrict__ gy, int H, int W, int C, int T) {
  __shared__ double red[2][4][256];
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
    for (int q = q0 + pr; q < q1; q += NPR) {
      const int h2 = q / W2, w2 = q - h2 * W2;
      const float4 g4 = ld4(gnb + (size_t)q * C + c);
      const float gv[4] = {g4.x, g4.y, g4.z, g4.w};
      const size_t p00 = ((size_t)(2 * h2) * W + 2 * w2) * C + c;
      const size_t poff[4] = {p00, p00 + C, p00 + (size_t)W * C, p00 + (size_t)W * C + C};
      float4 yv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) yv[k] = ld4(yb + poff[k]);
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
            const float gx = (arg[ch] == k) ? gv[ch] * slope(x) : 0.f;
            o[ch] = rstd[ch] * (gx - m1[ch] - x * m2[ch]);
          }
          st4(gyb + poff[k], make_float4(o[0], o[1], o[2], o[3]));
        }
      }
    }
  } else {
    const int p0 = tile * rows * W, p1 = p0 + rows * W;
    for (int p = p0 + pr; p < p1; p += NPR) {
      float4 g4;
      if (pmode == P_ID) {
        g4 = ld4(gnext + ((size_t)b * H * W + p) * C + c);
      } else {  // P_UP: gnext at (2H, 2W)
        const int h = p / W, w = p - h * W;
        const float* s = gnext + (((size_t)b * 2 * H + 2 * h) * 2 * W + 2 * w) * C + c;
        const size_t rs = (size_t)2 * W * C;
        const float4 u0 = ld4(s), u1 = ld4(s + C), u2 = ld4(s + rs), u3 = ld4(s + rs + C);
        g4 = make_float4(u0.x + u1.x + u2.x + u3.x, u0.y + u1.y + u2.y + u3.y,
                         u0.z + u1.z + u2.z + u3.z, u0.w + u1.w + u2.w + u3.w);
      }
      const float4 y4 = ld4(yb + (size_t)p * C + c);
      const float gv[4] = {g4.x, g4.y, g4.z, g4.w};
      const float yy[4] = {y4.x, y4.y, y4.z, y4.w};
      float o[4];
#pragma unroll
      for (int ch = 0; ch < 4; ++ch) {
        const float x = (yy[ch] - mean[ch]) * rstd[ch];
        const float gx = gv[ch] * slope(x);
        if (!APPLY) {
          a1[ch] += (double)gx;
          a2[ch] = fma((double)gx, (double)x, a2[ch]);
        } else {
          o[ch] = rstd[ch] * (gx - m1[ch] - x * m2[ch]);
        }
      }
      if (APPLY) st4(gyb + (size_t)p * C + c, make_float4(o[0], o[1], o[2], o[3]));
    }
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

__global__ void in_bwd_finalize_kernel(const double2* __restrict__ part, float2* __restrict__ bst,
                                       int B, int C, int T, double inv_hw) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B * C) return;
  const int b = e / C, c = e - b * C;
  double s1 = 0.0, s2 = 0.0;
  for (int t = 0; t < T; ++t) {
    const double2 v = part[((size_t)b * T + t) * C + c];
    s1 += v.x;
    s2 += v.y;
  }
  bst[e] = make_float2((float)(s1 * inv_hw), (float)(s2 * inv_hw));
}

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
  EV_REQUIRE(part && stats && B > 0 && C > 0 && tiles > 0, "in_stats_finalize: bad args");
  const int n = B * C;
  hipLaunchKernelGGL(in_stats_finalize_kernel, dim3((n + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, (const float2*)part, (float2*)stats, B, C, tiles,
                     (float)n_per_tile);
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
                     (float*)nullptr, H, W, C, T);
  return evh::check_launch("in_bwd_reduce");
}

extern "C" int ebsdvae_in_bwd_finalize(const double* part, float* bstats, int B, int C, int tiles,
                                       int HW, ebsdvae_stream_t stream) {
  EV_REQUIRE(part && bstats, "in_bwd_finalize: null pointer");
  const int n = B * C;
  hipLaunchKernelGGL(in_bwd_finalize_kernel, dim3((n + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, (const double2*)part, (float2*)bstats, B, C, tiles,
                     1.0 / (double)HW);
  return evh::check_launch("in_bwd_finalize");
}

extern "C" int ebsdvae_in_bwd_apply(const float* gnext, int pmode, const float* y,
                                    const float* stats, const float* bstats, float* gy, int B,
                                    int H, int W, int C, ebsdvae_stream_t stream) {
  EV_REQUIRE(gnext && y && stats && bstats && gy, "in_bwd_apply: null pointer");
  EV_REQUIRE(pmode >= 0 && pmode <= 2 && C % 4 == 0 && (256 % (C / 4)) == 0, "in_bwd_apply: bad pmode/C");
  const int T = in_bwd_tiles_host(H, W);
  hipLaunchKernelGGL(in_bwd_kernel<true>, dim3(T, B), dim3(256), 0, (hipStream_t)stream, gnext,
                     pmode, y, (const float2*)stats, (const float2*)bstats, (double2*)nullptr, gy, H,
                     W, C, T);
  return evh::check_launch("in_bwd_apply");
}
