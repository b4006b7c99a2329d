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

}  // namespace ev

using namespace ev;

extern "C" int ebsdvae_conv3x3_cout1_fwd(const float* src, const float* src_stats, int src_mode,
                                         const float* w, const float* bias, float* out, int flip,
                                         int B, int H, int W, int cin, ebsdvae_stream_t stream) {
  EdgeGeom g;
  EV_REQUIRE(src && w && out && B > 0, "conv3x3_cout1_fwd: null pointer");
  EV_REQUIRE(cin == 32, "conv3x3_cout1_fwd: cin=%d unsupported (32)", cin);
  EV_REQUIRE(src_mode == ACT_RAW || src_mode == ACT_UP || src_stats, "conv3x3_cout1_fwd: NORM needs stats");
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
