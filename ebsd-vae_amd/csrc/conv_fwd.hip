// 3x3 stride-1 pad-1 convolution as an implicit GEMM on the fp32 MFMA
// (v_mfma_f32_32x32x2_f32, exact f32 at the 157 TF vector rate; gfx950 has no xf32).
//
// Replaces, for every block of the reference VAE:
//   nn.Conv2d(...)           latice/model.py:95 (encoder), :148 is the cout=1 kernel
//   nn.ConvTranspose2d(...)  latice/model.py:102-104 (== conv with the weight transposed and
//                            spatially flipped; done by ebsdvae_pack_conv_weight)
// and, with a for_dgrad weight pack and a RAW source, their input gradients.
//
// Layout / tiling (MI355X-first):
//   * NHWC activations; a block owns M output pixels (full-width row bands TH x W of one
//     image, or NI whole images when H*W < M) x all Cout channels;
//   * K loop over Cin in chunks of 8 channels x 9 taps.  Per chunk the block stages
//       - the weight slab [9][8][Cout] (contiguous copy, 16-B LDS writes) and
//       - the input halo [(TH+2)][(W+2)][8] with an ODD pixel stride (9 floats) so that the
//         32 consecutive pixels of an MFMA A-fragment hit 32 different LDS banks,
//     applying the producer's InstanceNorm + LeakyReLU (+ 2x2 max-pool or nearest x2
//     upsample) on the fly: the normalised activation never touches HBM;
//   * 4 waves, each a 64x64 (or 128x32) register tile = 4 accumulators of 32x32 (64 AGPR/
//     VGPR); per k-step 2 A + 2 B ds_read_b32 feed 4 MFMAs (256 MFMA cycles per SIMD);
//   * epilogue: + bias, coalesced 128-B row stores of y, and per-wave InstanceNorm partials
//     {mean, M2} (Chan-combinable, no E[x^2]-E[x]^2 cancellation).
#include "common.h"
#include "../../include/ebsdvae.h"

namespace ev {

constexpr int CK = 8;        // input channels per K chunk
constexpr int CKP = CK + 1;  // LDS pixel stride of the input halo

template <int WM, int MF, int NF, bool CIN1>
__global__ __launch_bounds__(256) void conv3x3_fwd_kernel(
    const float* __restrict__ src, const float2* __restrict__ sstats, int smode,
    const float* __restrict__ wp, const float* __restrict__ bias, float* __restrict__ y,
    float2* __restrict__ spart, int B, int H, int W, int Cin, int TH, int NI) {
  constexpr int WN = 4 / WM;
  constexpr int N = WN * NF * 32;  // == Cout
  constexpr int MW = MF * 32;      // pixels per wave
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int HP = TH + 2, WP = W + 2;
  const int pixP = NI * HP * WP;
  float* lw = smem;
  float* lx = smem + (CIN1 ? 9 * N : 9 * CK * N);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int l32 = lane & 31, hk = lane >> 5;
  int b0, h0;
  if (NI > 1) {
    b0 = blockIdx.x * NI;
    h0 = 0;
  } else {
    const int tpi = H / TH;
    b0 = blockIdx.x / tpi;
    h0 = (blockIdx.x % tpi) * TH;
  }
  const int tpx = TH * W;  // pixels per image region of the tile

  int abase[MF];
#pragma unroll
  for (int mf = 0; mf < MF; ++mf) {
    const int p = wm * MW + mf * 32 + l32;
    const int img = p / tpx, rem = p - img * tpx;
    const int r = rem / W, c = rem - r * W;
    abase[mf] = CIN1 ? ((img * HP + r) * WP + c) : (((img * HP + r) * WP + c) * CKP + hk);
  }

  f32x16 acc[MF][NF];
#pragma unroll
  for (int mf = 0; mf < MF; ++mf)
#pragma unroll
    for (int nf = 0; nf < NF; ++nf)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mf][nf][r] = 0.f;

  const int nchunks = CIN1 ? 1 : Cin / CK;
  const int ncol = wn * NF * 32 + l32;
  for (int ch = 0; ch < nchunks; ++ch) {
    __syncthreads();
    if (CIN1) {
      for (int i = tid; i < 9 * N; i += 256) lw[i] = wp[i];
      for (int i = tid; i < pixP; i += 256) {
        const int img = i / (HP * WP), rem = i - img * (HP * WP);
        const int hh = rem / WP, ww = rem - hh * WP;
        const int gh = h0 + hh - 1, gw = ww - 1, gb = b0 + img;
        float v = 0.f;
        if (gb < B && gh >= 0 && gh < H && gw >= 0 && gw < W)
          v = load_act1(src, sstats, smode, gb, gh, gw, 0, H, W, 1);
        lx[i] = v;
      }
    } else {
      for (int i = tid; i < 9 * CK * N / 4; i += 256) {
        const int e = i * 4;
        const int t = e / (CK * N), rem = e - t * (CK * N);
        st4(lw + e, ld4(wp + ((size_t)t * Cin + ch * CK) * N + rem));
      }
      for (int i = tid; i < pixP * (CK / 4); i += 256) {
        const int pix = i >> 1, q = i & 1;
        const int img = pix / (HP * WP), rem = pix - img * (HP * WP);
        const int hh = rem / WP, ww = rem - hh * WP;
        const int gh = h0 + hh - 1, gw = ww - 1, gb = b0 + img;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (gb < B && gh >= 0 && gh < H && gw >= 0 && gw < W)
          v = load_act4(src, sstats, smode, gb, gh, gw, ch * CK + q * 4, H, W, Cin);
        float* d = lx + pix * CKP + q * 4;
        d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
      }
    }
    __syncthreads();

    if (CIN1) {
      // K = the 9 taps (padded to 10): k-step s covers taps 2s (lanes 0-31), 2s+1 (32-63)
#pragma unroll
      for (int s = 0; s < 5; ++s) {
        const int t = 2 * s + hk;
        const bool ok = t < 9;
        const int kh = t / 3, kw = t - kh * 3;
        float a[MF], bv[NF];
#pragma unroll
        for (int mf = 0; mf < MF; ++mf) a[mf] = ok ? lx[abase[mf] + kh * WP + kw] : 0.f;
#pragma unroll
        for (int nf = 0; nf < NF; ++nf) bv[nf] = ok ? lw[t * N + ncol + nf * 32] : 0.f;
#pragma unroll
        for (int mf = 0; mf < MF; ++mf)
#pragma unroll
          for (int nf = 0; nf < NF; ++nf)
            acc[mf][nf] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[mf], bv[nf], acc[mf][nf], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int kh = tap / 3, kw = tap % 3;
        const int toff = (kh * WP + kw) * CKP;
#pragma unroll
        for (int kp = 0; kp < CK / 2; ++kp) {
          float a[MF], bv[NF];
#pragma unroll
          for (int mf = 0; mf < MF; ++mf) a[mf] = lx[abase[mf] + toff + 2 * kp];
          const float* wrow = lw + (tap * CK + 2 * kp + hk) * N + ncol;
#pragma unroll
          for (int nf = 0; nf < NF; ++nf) bv[nf] = wrow[nf * 32];
#pragma unroll
          for (int mf = 0; mf < MF; ++mf)
#pragma unroll
            for (int nf = 0; nf < NF; ++nf)
              acc[mf][nf] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[mf], bv[nf], acc[mf][nf], 0, 0, 0);
        }
      }
    }
  }

  // ---------------------------------------------------------------- epilogue
  const int wpx0 = wm * MW;                 // first tile pixel of this wave
  const int wimg = wpx0 / tpx;              // the wave's pixels lie in ONE image
  const int gb = b0 + wimg;
  const bool bvalid = gb < B;
#pragma unroll
  for (int nf = 0; nf < NF; ++nf) {
    const int co = ncol + nf * 32;
    const float bb = bias ? bias[co] : 0.f;
    float s = 0.f;
#pragma unroll
    for (int mf = 0; mf < MF; ++mf)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = wpx0 + mf * 32 + (r & 3) + 8 * (r >> 2) + 4 * hk;
        const int rem = m - wimg * tpx;
        const float v = acc[mf][nf][r] + bb;
        acc[mf][nf][r] = v;
        s += v;
        if (bvalid) y[(((size_t)gb * H + h0) * W + rem) * N + co] = v;
      }
    if (spart) {
      s += __shfl_xor(s, 32, 64);
      const float mean = s * (1.0f / MW);
      float q = 0.f;
#pragma unroll
      for (int mf = 0; mf < MF; ++mf)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float d = acc[mf][nf][r] - mean;
          q = fmaf(d, d, q);
        }
      q += __shfl_xor(q, 32, 64);
      if (hk == 0 && bvalid) {
        const int T = (H * W) / MW;
        const int slot = (h0 * W + (wpx0 - wimg * tpx)) / MW;
        spart[((size_t)gb * T + slot) * N + co] = make_float2(mean, q);
      }
    }
  }
}

// Weight packing into [tap][Cin'][Cout'] (see ebsdvae.h).
__global__ void pack_conv_weight_kernel(const float* __restrict__ s, float* __restrict__ d,
                                        int cin, int cout, int kind, int dgrad) {
  const int ci_ = dgrad ? cout : cin;   // packed input-channel count
  const int co_ = dgrad ? cin : cout;
  const int n = 9 * ci_ * co_;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const int t = e / (ci_ * co_);
    const int rem = e - t * (ci_ * co_);
    const int i = rem / co_, o = rem - i * co_;
    // logical conv-equivalent (co, ci) of the layer
    const int co = dgrad ? i : o;
    const int ci = dgrad ? o : i;
    int tt;
    size_t idx;
    if (kind == 0) {  // Conv2d weight (cout, cin, 3, 3); Wc[co][ci][t] = s[co][ci][t]
      tt = dgrad ? 8 - t : t;
      idx = ((size_t)co * cin + ci) * 9 + tt;
    } else {          // ConvTranspose2d weight (cin, cout, 3, 3); Wc[co][ci][t] = s[ci][co][8-t]
      tt = dgrad ? t : 8 - t;
      idx = ((size_t)ci * cout + co) * 9 + tt;
    }
    d[e] = s[idx];
  }
}

struct FwdCfg {
  int M, TH, NI;
  size_t lds;
};

static bool fwd_cfg(int H, int W, int cin, int cout, FwdCfg* c) {
  int M;
  if (cout == 128) M = 128;
  else if (cout == 64) M = 256;
  else if (cout == 32) M = 512;
  else return false;
  if (W > M || (M % W) != 0) return false;
  c->M = M;
  if (H * W >= M) {
    c->TH = M / W;
    c->NI = 1;
    if (H % c->TH) return false;
  } else {
    c->TH = H;
    c->NI = M / (H * W);
    if (M % (H * W)) return false;
  }
  const int MW = (cout == 32) ? 128 : 64;
  if ((H * W) % MW) return false;
  const bool cin1 = (cin == 1);
  const size_t wfl = cin1 ? 9 * cout : 9 * CK * cout;
  const size_t xfl = (size_t)c->NI * (c->TH + 2) * (W + 2) * (cin1 ? 1 : CKP);
  c->lds = (wfl + xfl) * sizeof(float);
  return c->lds <= 160 * 1024;
}

}  // namespace ev

using namespace ev;

extern "C" int ebsdvae_conv3x3_stat_tiles(int H, int W, int cout) {
  const int MW = (cout == 32) ? 128 : 64;
  return (H * W) / MW;
}

extern "C" int ebsdvae_pack_conv_weight(const float* src, float* dst, int cin, int cout,
                                        int kind, int for_dgrad, ebsdvae_stream_t stream) {
  EV_REQUIRE(src && dst && cin > 0 && cout > 0 && (kind == 0 || kind == 1),
             "pack_conv_weight: bad arguments");
  const int n = 9 * cin * cout;
  const int blocks = (n + 255) / 256;
  hipLaunchKernelGGL(pack_conv_weight_kernel, dim3(blocks < 1024 ? blocks : 1024), dim3(256), 0,
                     (hipStream_t)stream, src, dst, cin, cout, kind, for_dgrad);
  return evh::check_launch("pack_conv_weight");
}

template <int WM, int MF, int NF, bool CIN1>
static int launch_fwd(const FwdCfg& c, const float* src, const float* st, int mode,
                      const float* wp, const float* bias, float* y, float* part, int B, int H,
                      int W, int cin, hipStream_t s) {
  auto k = conv3x3_fwd_kernel<WM, MF, NF, CIN1>;
  static bool attr_done = false;   // once per instantiation (keeps graph capture clean)
  if (!attr_done) {
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_done = true;
  }
  const int blocks = (c.NI > 1) ? (B + c.NI - 1) / c.NI : B * (H / c.TH);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), c.lds, s, src, (const float2*)st, mode, wp, bias,
                     y, (float2*)part, B, H, W, cin, c.TH, c.NI);
  return evh::check_launch("conv3x3_fwd");
}

extern "C" int ebsdvae_conv3x3_fwd(const float* src, const float* src_stats, int src_mode,
                                   const float* wpack, const float* bias, float* y,
                                   float* stat_part, int B, int H, int W, int cin, int cout,
                                   ebsdvae_stream_t stream) {
  FwdCfg c;
  EV_REQUIRE(src && wpack && y && B > 0, "conv3x3_fwd: null pointer or empty batch");
  EV_REQUIRE(src_mode >= 0 && src_mode <= 4, "conv3x3_fwd: bad src_mode %d", src_mode);
  EV_REQUIRE(src_mode == ACT_RAW || src_mode == ACT_UP || src_stats,
             "conv3x3_fwd: NORM modes need src_stats");
  EV_REQUIRE(cin == 1 || (cin % CK) == 0, "conv3x3_fwd: cin=%d must be 1 or a multiple of %d", cin, CK);
  EV_REQUIRE(cin != 1 || cout == 32, "conv3x3_fwd: cin=1 supports cout=32 only");
  EV_REQUIRE(fwd_cfg(H, W, cin, cout, &c), "conv3x3_fwd: unsupported shape H=%d W=%d cin=%d cout=%d",
             H, W, cin, cout);
  hipStream_t s = (hipStream_t)stream;
  if (cin == 1) return launch_fwd<4, 4, 1, true>(c, src, src_stats, src_mode, wpack, bias, y, stat_part, B, H, W, cin, s);
  if (cout == 128) return launch_fwd<2, 2, 2, false>(c, src, src_stats, src_mode, wpack, bias, y, stat_part, B, H, W, cin, s);
  if (cout == 64) return launch_fwd<4, 2, 2, false>(c, src, src_stats, src_mode, wpack, bias, y, stat_part, B, H, W, cin, s);
  return launch_fwd<4, 4, 1, false>(c, src, src_stats, src_mode, wpack, bias, y, stat_part, B, H, W, cin, s);
}
