// 3x3 stride-1 pad-1 convolution as an implicit GEMM on the fp32 MFMA
// (v_mfma_f32_32x32x2_f32, exact f32 at the 157 TF vector rate; gfx950 has no xf32).
//
// Replaces, for every block of the reference VAE:
//   nn.Conv2d(...)           latice/model.py:95 (encoder), :148 is the cout=1 kernel
//   nn.ConvTranspose2d(...)  latice/model.py:102-104 (== conv with the weight transposed and
//                            spatially flipped; done by ebsdvae_pack_conv_weight)
// and, with a for_dgrad weight pack and a RAW source, their input gradients.
//
// GEMM view: M = output pixels (NHWC), N = Cout, K = 9 taps x Cin, swept in chunks of 8
// input channels x 9 taps.  Packed weights are laid out [chunk][tap][ci8][Cout] so each
// chunk's slab is ONE contiguous run.
//
// Main kernel (conv3x3_big_kernel, H*W >= 256): 512 threads = 8 waves (2 per SIMD), each a
// 64x64 (or 128x32) register tile of four 32x32 accumulators.  Software pipeline with one
// barrier per chunk:
//     issue  global_load_lds (DMA) of the NEXT weight slab -> LDS buffer (c+1)&1
//     issue  raw global loads of the NEXT input halo       -> registers
//     MFMA   the current chunk from LDS buffers c&1
//     apply  the producer's InstanceNorm + LeakyReLU (+ 2x2 max-pool / nearest x2
//            upsample) to the halo registers, write LDS buffer (c+1)&1 (odd pixel stride
//            9 floats -> the 32 pixels of an A fragment hit 32 different banks)
//     barrier (drains the DMA)
// so HBM/L2 latency hides under ~18k MFMA cycles per chunk and the normalised activation
// never touches HBM.
// Small-image kernel (conv3x3_small_kernel, 8x8 and the cin=1 first conv): 256 threads,
// whole images per block, Cout split over blockIdx.y to fill the 256 CUs.
// Epilogue (both): + bias, coalesced 128-B row stores of y, and per-wave InstanceNorm
// partials {mean, M2} (Chan-combinable, no E[x^2]-E[x]^2 cancellation).
#include "conv_common.h"

namespace ev {

constexpr int CK = 8;        // input channels per K chunk
constexpr int CKP = CK + 1;  // LDS pixel stride of the input halo

// 9 taps x 4 k-pairs of one 8-channel chunk: A from the halo, B from the weight slab
template <int MF, int NF>
EV_DEVINL void mma_chunk(f32x16 (&acc)[MF][NF], const float* __restrict__ lx,
                         const float* __restrict__ lw, const int (&abase)[MF], int WP, int NT,
                         int ncol, int hk) {
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int kh = tap / 3, kw = tap % 3;
    const int toff = (kh * WP + kw) * CKP;
#pragma unroll
    for (int kp = 0; kp < CK / 2; ++kp) {
      float a[MF], bv[NF];
#pragma unroll
      for (int mf = 0; mf < MF; ++mf) a[mf] = lx[abase[mf] + toff + 2 * kp];
      const float* wrow = lw + (tap * CK + 2 * kp + hk) * NT + ncol;
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

// ------------------------------------------------------------------ main pipelined kernel
// 8 waves as WM (pixels) x WN (channels); KX = halo float4 items per thread (compile-time
// upper bound); MODE = act source mode.
template <int NWV, int WM, int MF, int NF, int KX, int MODE, int FP>
__global__ __launch_bounds__(NWV * 64, 2) void conv3x3_big_kernel(
    const float* __restrict__ src, const float2* __restrict__ sstats, const float* __restrict__ wp,
    const float* __restrict__ bias, float* __restrict__ y, float2* __restrict__ spart,
    float* __restrict__ act_out, int B, int H, int W, int Cin, int TH,
    const float* __restrict__ yprev, const float2* __restrict__ stprev, double2* __restrict__ ipart) {
  constexpr int WN = NWV / WM;
  constexpr int NT = WN * NF * 32;   // == Cout
  constexpr int MW = MF * 32;
  constexpr int NTHR = NWV * 64;
  constexpr int WSLAB = 9 * CK * NT;  // floats per weight chunk
  constexpr bool POOL = (MODE == ACT_NORM_POOL);
  constexpr bool NORM = (MODE == ACT_NORM || MODE == ACT_NORM_POOL || MODE == ACT_NORM_UP);
  constexpr bool UPS = (MODE == ACT_UP || MODE == ACT_NORM_UP);
  constexpr int NR = POOL ? 4 : 1;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int HP = TH + 2, WP = W + 2;
  const int pixP = HP * WP;
  const int xslab = (pixP + 1) * CKP;   // + one dummy pixel slot for out-of-halo items
  float* lw0 = smem;
  float* lx0 = smem + 2 * WSLAB;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int l32 = lane & 31, hk = lane >> 5;
  const int tpi = H / TH;
  const int b0 = blockIdx.x / tpi;
  const int h0 = (blockIdx.x % tpi) * TH;
  const int tpx = TH * W;

  int abase[MF];
#pragma unroll
  for (int mf = 0; mf < MF; ++mf) {
    const int p = wm * MW + mf * 32 + l32;
    const int r = p / W, c = p - r * W;
    abase[mf] = ((r * WP) + c) * CKP + hk;
  }

  // source geometry
  const int Hs = POOL ? 2 * H : (UPS ? H / 2 : H);
  const int Ws = POOL ? 2 * W : (UPS ? W / 2 : W);
  const float* sb = src + (size_t)b0 * Hs * Ws * Cin;
  const int q = tid & 1;  // this thread's 4-channel half of every 8-channel chunk

  // halo item k of this thread: pixel (tid + NTHR*k) >> 1, channels q*4..q*4+3.  Its
  // source coordinates are chunk-invariant: packed once as (gh << 16) | gw, -1 = zero pad.
  int hw[KX];
#pragma unroll
  for (int k = 0; k < KX; ++k) {
    const int pix = (tid + NTHR * k) >> 1;
    const int hh = pix / WP, ww = pix - hh * WP;
    const int gh = h0 + hh - 1, gw = ww - 1;
    hw[k] = (pix < pixP && gh >= 0 && gh < H && gw >= 0 && gw < W) ? ((gh << 16) | gw) : -1;
  }
  float4 raw[KX][NR];
  float2 st[4];
  int cur_ch = 0;   // chunk whose halo is held in raw[]
  // Branch-free staging: padding items load from a safe in-range address and are zeroed by
  // select; items past the halo write a dummy LDS pixel slot (pixP).  Per-item divergent
  // branches cost ~25 SALU + exec juggling per item inside the MFMA loop.
  auto issue_halo = [&](int ch) {
    cur_ch = ch;
    const int c = ch * CK + q * 4;
#pragma unroll
    for (int k = 0; k < KX; ++k) {
      const int hv = hw[k] < 0 ? 0 : hw[k];
      const int gh = hv >> 16, gw = hv & 0xffff;
#ifdef EV_TIMING_PROBE_NOHALO   // timing experiment only: no halo traffic (wrong results)
      raw[k][0] = make_float4(gh, gw, 1.f, 1.f);
      continue;
#endif
      if (POOL) {
        const float* p = sb + ((size_t)(2 * gh) * Ws + 2 * gw) * Cin + c;
        const size_t rs = (size_t)Ws * Cin;
        raw[k][0] = ld4(p);
        raw[k][NR > 1 ? 1 : 0] = ld4(p + Cin);
        raw[k][NR > 2 ? 2 : 0] = ld4(p + rs);
        raw[k][NR > 3 ? 3 : 0] = ld4(p + rs + Cin);
      } else if (UPS) {
        raw[k][0] = ld4(sb + ((size_t)(gh >> 1) * Ws + (gw >> 1)) * Cin + c);
      } else {
        raw[k][0] = ld4(sb + ((size_t)gh * Ws + gw) * Cin + c);
      }
    }
    if (NORM) {
      const float2* s = sstats + (size_t)b0 * Cin + c;
      st[0] = s[0]; st[1] = s[1]; st[2] = s[2]; st[3] = s[3];
    }
  };
  auto store_halo = [&](float* lx) {
    float2 fs[4];
    if (NORM) {
#pragma unroll
      for (int i = 0; i < 4; ++i) fs[i] = norm_fs(st[i]);
    }
#pragma unroll
    for (int k = 0; k < KX; ++k) {
      const int pix = (tid + NTHR * k) >> 1;
      float4 v = raw[k][0];
      if (POOL)
        v = max4(max4(raw[k][0], raw[k][NR > 1 ? 1 : 0]),
                 max4(raw[k][NR > 2 ? 2 : 0], raw[k][NR > 3 ? 3 : 0]));
      if (NORM)
        v = make_float4(normact_fs(v.x, fs[0]), normact_fs(v.y, fs[1]), normact_fs(v.z, fs[2]),
                        normact_fs(v.w, fs[3]));
      const bool ok = hw[k] >= 0;
      v = make_float4(ok ? v.x : 0.f, ok ? v.y : 0.f, ok ? v.z : 0.f, ok ? v.w : 0.f);
      // interior pixels: optionally materialise the (pooled) activation for the wgrad
      if (act_out) {   // uniform (kernel argument)
        const int gh = hw[k] >> 16, gw = hw[k] & 0xffff;
        if (ok && gh >= h0 && gh < h0 + TH)
          st4(act_out + (((size_t)b0 * H + gh) * W + gw) * Cin + cur_ch * CK + q * 4, v);
      }
      float* d = lx + (pix < pixP ? pix : pixP) * CKP + q * 4;
      d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
    }
  };
  auto issue_weights = [&](int ch, float* lw) {
    const float* g = wp + (size_t)ch * WSLAB;
    for (int pc = wave; pc < WSLAB / 256; pc += NWV) glds16(g + pc * 256 + lane * 4, lw + pc * 256);
  };

  f32x16 acc[MF][NF];
#pragma unroll
  for (int mf = 0; mf < MF; ++mf)
#pragma unroll
    for (int nf = 0; nf < NF; ++nf)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mf][nf][r] = 0.f;

  const int nchunks = Cin / CK;
  issue_weights(0, lw0);
  issue_halo(0);
  store_halo(lx0);
  __syncthreads();
  const int ncol = wn * NF * 32 + l32;
  for (int ch = 0; ch < nchunks; ++ch) {
    const int cur = ch & 1, nxt = cur ^ 1;
    const bool more = ch + 1 < nchunks;
    if (more) {
      issue_weights(ch + 1, lw0 + nxt * WSLAB);
      issue_halo(ch + 1);
    }
    mma_chunk<MF, NF>(acc, lx0 + cur * xslab, lw0 + cur * WSLAB, abase, WP, NT, ncol, hk);
    if (more) store_halo(lx0 + nxt * xslab);
    __syncthreads();
  }
  conv_epilogue<MF, NF, FP>(acc, bias, y, spart, B, H, W, NT, b0, h0, tpx, wm * MW, wn * NF * 32, hk,
                            l32, yprev, stprev, ipart);
}

// ------------------------------------------------------------------ small-image kernel
// 256 threads; TH-row bands (whole 8x8 images) per block; Cout split into NT-wide column
// blocks over blockIdx.y.  CIN1: K = the 9 taps (first conv), NI images per block.
template <int WM, int MF, int NF, bool CIN1, int FP>
__global__ __launch_bounds__(256) void conv3x3_small_kernel(
    const float* __restrict__ src, const float2* __restrict__ sstats, int smode,
    const float* __restrict__ wp, const float* __restrict__ bias, float* __restrict__ y,
    float2* __restrict__ spart, float* __restrict__ act_out, int B, int H, int W, int Cin, int Cout,
    int TH, int NI, const float* __restrict__ yprev, const float2* __restrict__ stprev,
    double2* __restrict__ ipart) {
  constexpr int WN = 4 / WM;
  constexpr int NT = WN * NF * 32;
  constexpr int MW = MF * 32;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int HP = TH + 2, WP = W + 2;
  const int pixP = NI * HP * WP;
  float* lw = smem;
  float* lx = smem + (CIN1 ? 9 * NT : 9 * CK * NT);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int l32 = lane & 31, hk = lane >> 5;
  const int n0 = blockIdx.y * NT;
  int b0, h0;
  if (NI > 1) {
    b0 = blockIdx.x * NI;
    h0 = 0;
  } else {
    const int tpi = H / TH;
    b0 = blockIdx.x / tpi;
    h0 = (blockIdx.x % tpi) * TH;
  }
  const int tpx = TH * W;
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
      for (int i = tid; i < 9 * NT; i += 256) lw[i] = wp[(i / NT) * Cout + n0 + (i % NT)];
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
      const float* g = wp + (size_t)ch * 9 * CK * Cout + n0;
      for (int i = tid; i < 9 * CK * NT / 4; i += 256) {
        const int e = i * 4;
        const int row = e / NT, col = e - row * NT;
        st4(lw + e, ld4(g + (size_t)row * Cout + col));
      }
      for (int i = tid; i < pixP * (CK / 4); i += 256) {
        const int pix = i >> 1, q = i & 1;
        const int img = pix / (HP * WP), rem = pix - img * (HP * WP);
        const int hh = rem / WP, ww = rem - hh * WP;
        const int gh = h0 + hh - 1, gw = ww - 1, gb = b0 + img;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        const bool ok = gb < B && gh >= 0 && gh < H && gw >= 0 && gw < W;
        if (ok) v = load_act4(src, sstats, smode, gb, gh, gw, ch * CK + q * 4, H, W, Cin);
        float* d = lx + pix * CKP + q * 4;
        d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
        if (act_out && ok && blockIdx.y == 0 && hh >= 1 && hh <= TH)
          st4(act_out + (((size_t)gb * H + gh) * W + gw) * Cin + ch * CK + q * 4, v);
      }
    }
    __syncthreads();
    if (CIN1) {
#pragma unroll
      for (int s = 0; s < 5; ++s) {
        const int t = 2 * s + hk;
        const bool ok = t < 9;
        const int kh = t / 3, kw = t - kh * 3;
        float a[MF], bv[NF];
#pragma unroll
        for (int mf = 0; mf < MF; ++mf) a[mf] = ok ? lx[abase[mf] + kh * WP + kw] : 0.f;
#pragma unroll
        for (int nf = 0; nf < NF; ++nf) bv[nf] = ok ? lw[t * NT + ncol + nf * 32] : 0.f;
#pragma unroll
        for (int mf = 0; mf < MF; ++mf)
#pragma unroll
          for (int nf = 0; nf < NF; ++nf)
            acc[mf][nf] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[mf], bv[nf], acc[mf][nf], 0, 0, 0);
      }
    } else {
      mma_chunk<MF, NF>(acc, lx, lw, abase, WP, NT, ncol, hk);
    }
  }
  conv_epilogue<MF, NF, FP>(acc, bias, y, spart, B, H, W, Cout, b0, h0, tpx, wm * MW,
                            n0 + wn * NF * 32, hk, l32, yprev, stprev, ipart);
}

// Weight packing into [chunk][tap][ci8][Cout'] (CK = 8; CK = 1 when Cin' == 1).
__global__ void pack_conv_weight_kernel(const float* __restrict__ s, float* __restrict__ d,
                                        int cin, int cout, int kind, int dgrad) {
  const int ci_ = dgrad ? cout : cin;   // packed input-channel count
  const int co_ = dgrad ? cin : cout;
  const int ck = ci_ < CK ? ci_ : CK;
  const int n = 9 * ci_ * co_;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const int o = e % co_;
    const int r = e / co_;            // (chunk, tap, ci8)
    const int c8 = r % ck;
    const int r2 = r / ck;
    const int t = r2 % 9, chunk = r2 / 9;
    const int i = chunk * ck + c8;
    // logical conv-equivalent (co, ci) of the layer
    const int co = dgrad ? i : o;
    const int ci = dgrad ? o : i;
    size_t idx;
    if (kind == 0) {  // Conv2d weight (cout, cin, 3, 3); Wc[co][ci][t] = s[co][ci][t]
      idx = ((size_t)co * cin + ci) * 9 + (dgrad ? 8 - t : t);
    } else {          // ConvTranspose2d weight (cin, cout, 3, 3); Wc[co][ci][t] = s[ci][co][8-t]
      idx = ((size_t)ci * cout + co) * 9 + (dgrad ? t : 8 - t);
    }
    d[e] = s[idx];
  }
}

// one launch packs every conv weight of a step: blockIdx.y = descriptor (kernel argument)
__global__ void pack_conv_weights_kernel(const PackBatch pb) {
  const ebsdvae_pack_desc& q = pb.d[blockIdx.y];
  const int ci_ = q.for_dgrad ? q.cout : q.cin;
  const int co_ = q.for_dgrad ? q.cin : q.cout;
  const int ck = ci_ < CK ? ci_ : CK;
  const int n = 9 * ci_ * co_;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const int o = e % co_;
    const int r = e / co_;
    const int c8 = r % ck;
    const int r2 = r / ck;
    const int t = r2 % 9, chunk = r2 / 9;
    const int i = chunk * ck + c8;
    const int co = q.for_dgrad ? i : o;
    const int ci = q.for_dgrad ? o : i;
    size_t idx;
    if (q.kind == 0) idx = ((size_t)co * q.cin + ci) * 9 + (q.for_dgrad ? 8 - t : t);
    else idx = ((size_t)ci * q.cout + co) * 9 + (q.for_dgrad ? t : 8 - t);
    q.dst[e] = q.src[idx];
  }
}

// ------------------------------------------------------------------ host-side planning
struct Cfg {
  int kind;   // 0 big, 1 small, 2 cin1
  int M, TH, NI, NT, KX;
  size_t lds;
};

static bool plan_conv(int H, int W, int cin, int cout, Cfg* c) {
  if (cin == 1) {
    if (cout != 32) return false;
    c->kind = 2;
    c->M = 512;
    c->NT = 32;
    if (W > c->M || c->M % W) return false;
    if (H * W >= c->M) { c->TH = c->M / W; c->NI = 1; } else { c->TH = H; c->NI = c->M / (H * W); }
    if (H % c->TH) return false;
    c->lds = (9 * 32 + (size_t)c->NI * (c->TH + 2) * (W + 2)) * sizeof(float);
    return true;
  }
  if (cin % CK) return false;
  if (H * W >= 256) {
    if (!(cout == 128 || cout == 64 || cout == 32)) return false;
    c->kind = 0;
    // 8 waves (1 block/CU) for cout 128 (16 K chunks amortise the prologue/epilogue);
    // 4 waves (2 blocks/CU overlap each other's prologue/epilogue) for cout 64 / 32
    c->M = cout == 128 ? 256 : (cout == 64 ? 256 : 512);
    const int nthr = cout == 128 ? 512 : 256;
    c->NT = cout;
    if (W > c->M || c->M % W || H * W < c->M) return false;
    c->TH = c->M / W;
    c->NI = 1;
    if (H % c->TH) return false;
    const int pix = (c->TH + 2) * (W + 2);
    c->KX = (pix * 2 + nthr - 1) / nthr;
    const int kxmax = cout == 128 ? 2 : (cout == 64 ? 5 : 9);
    if (c->KX > kxmax) return false;
    c->lds = (2 * (size_t)9 * CK * cout + 2 * (size_t)(pix + 1) * CKP) * sizeof(float);
    return c->lds <= 160 * 1024;
  }
  // small images (8x8): one 64-pixel band per block, 64-wide Cout column blocks
  if (cout % 64 || (H * W) % 64 || W > 64) return false;
  c->kind = 1;
  c->NT = 64;
  c->M = 64;
  c->TH = 64 / W;
  c->NI = 1;
  if (H % c->TH) return false;
  c->lds = ((size_t)9 * CK * c->NT + (size_t)(c->TH + 2) * (W + 2) * CKP) * sizeof(float);
  return true;
}

template <typename K>
static void allow_big_lds(K k) {
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

template <int NWV, int WM, int MF, int NF, int KX, int MODE, int FP>
static void launch_big1(const Cfg& c, const float* src, const float* st, const float* wp,
                        const float* bias, float* y, float* part, float* aout, int B, int H, int W,
                        int cin, hipStream_t s, const InBwdFuse& f) {
  auto k = conv3x3_big_kernel<NWV, WM, MF, NF, KX, MODE, FP>;
  static bool once = false;
  if (!once) { allow_big_lds(k); once = true; }
  hipLaunchKernelGGL(k, dim3(B * (H / c.TH)), dim3(NWV * 64), c.lds, s, src, (const float2*)st, wp, bias,
                     y, (float2*)part, aout, B, H, W, cin, c.TH, f.yprev, f.stprev, f.part);
}

template <int NWV, int WM, int MF, int NF, int KX>
static void launch_big(const Cfg& c, const float* src, const float* st, int mode, const float* wp,
                       const float* bias, float* y, float* part, float* aout, int B, int H, int W,
                       int cin, hipStream_t s) {
  const InBwdFuse f;
  switch (mode) {
    case ACT_RAW: launch_big1<NWV, WM, MF, NF, KX, ACT_RAW, FP_NONE>(c, src, st, wp, bias, y, part, aout, B, H, W, cin, s, f); break;
    case ACT_NORM: launch_big1<NWV, WM, MF, NF, KX, ACT_NORM, FP_NONE>(c, src, st, wp, bias, y, part, aout, B, H, W, cin, s, f); break;
    case ACT_NORM_POOL: launch_big1<NWV, WM, MF, NF, KX, ACT_NORM_POOL, FP_NONE>(c, src, st, wp, bias, y, part, aout, B, H, W, cin, s, f); break;
    case ACT_UP: launch_big1<NWV, WM, MF, NF, KX, ACT_UP, FP_NONE>(c, src, st, wp, bias, y, part, aout, B, H, W, cin, s, f); break;
    default: launch_big1<NWV, WM, MF, NF, KX, ACT_NORM_UP, FP_NONE>(c, src, st, wp, bias, y, part, aout, B, H, W, cin, s, f); break;
  }
}

template <int NWV, int WM, int MF, int NF, int KX>
static void launch_big_fused(const Cfg& c, const float* src, const float* wp, float* y, int B, int H,
                             int W, int cin, hipStream_t s, int pmode, const InBwdFuse& f) {
  switch (pmode) {
    case P_ID: launch_big1<NWV, WM, MF, NF, KX, ACT_RAW, P_ID>(c, src, nullptr, wp, nullptr, y, nullptr, nullptr, B, H, W, cin, s, f); break;
    case P_POOL: launch_big1<NWV, WM, MF, NF, KX, ACT_RAW, P_POOL>(c, src, nullptr, wp, nullptr, y, nullptr, nullptr, B, H, W, cin, s, f); break;
    default: launch_big1<NWV, WM, MF, NF, KX, ACT_RAW, P_UP>(c, src, nullptr, wp, nullptr, y, nullptr, nullptr, B, H, W, cin, s, f); break;
  }
}

template <int WM, int MF, int NF, bool CIN1, int FP>
static void launch_small(const Cfg& c, const float* src, const float* st, int mode, const float* wp,
                         const float* bias, float* y, float* part, float* aout, int B, int H, int W,
                         int cin, int cout, hipStream_t s, const InBwdFuse& f = InBwdFuse()) {
  auto k = conv3x3_small_kernel<WM, MF, NF, CIN1, FP>;
  static bool once = false;
  if (!once) { allow_big_lds(k); once = true; }
  const int bx = (c.NI > 1) ? (B + c.NI - 1) / c.NI : B * (H / c.TH);
  hipLaunchKernelGGL(k, dim3(bx, cout / c.NT), dim3(256), c.lds, s, src, (const float2*)st, mode, wp,
                     bias, y, (float2*)part, aout, B, H, W, cin, cout, c.TH, c.NI, f.yprev, f.stprev,
                     f.part);
}

}  // namespace ev

using namespace ev;

// pixels per wave of the producing configuration -> InstanceNorm partial tiles per image
extern "C" int ebsdvae_conv3x3_stat_tiles(int H, int W, int cout) {
  if (!ev_dim_ok(H) || !ev_dim_ok(W)) return -1;
  const int MW = (H * W >= 256) ? (cout == 32 ? 128 : 64) : 32;
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

extern "C" int ebsdvae_pack_conv_weights(const ebsdvae_pack_desc* descs, int n,
                                         ebsdvae_stream_t stream) {
  EV_REQUIRE(descs && n > 0 && n <= EBSDVAE_MAX_PACK, "pack_conv_weights: n=%d out of range", n);
  PackBatch pb;
  int maxn = 0;
  for (int i = 0; i < n; ++i) {
    const ebsdvae_pack_desc& q = descs[i];
    EV_REQUIRE(q.src && q.dst && q.cin > 0 && q.cout > 0 && (q.kind == 0 || q.kind == 1),
               "pack_conv_weights: bad descriptor %d", i);
    pb.d[i] = q;
    const int e = 9 * q.cin * q.cout;
    if (e > maxn) maxn = e;
  }
  int bx = (maxn + 255) / 256;
  if (bx > 64) bx = 64;
  hipLaunchKernelGGL(pack_conv_weights_kernel, dim3(bx, n), dim3(256), 0, (hipStream_t)stream, pb);
  return evh::check_launch("pack_conv_weights");
}

extern "C" int ebsdvae_conv3x3_fwd(const float* src, const float* src_stats, int src_mode,
                                   const float* wpack, const float* bias, float* y,
                                   float* stat_part, float* act_out, int B, int H, int W, int cin,
                                   int cout, ebsdvae_stream_t stream) {
  Cfg c;
  EV_REQUIRE(src && wpack && y && B > 0, "conv3x3_fwd: null pointer or empty batch");
  EV_REQUIRE(src_mode >= 0 && src_mode <= 4, "conv3x3_fwd: bad src_mode %d", src_mode);
  EV_REQUIRE(src_mode == ACT_RAW || src_mode == ACT_UP || src_stats,
             "conv3x3_fwd: NORM modes need src_stats");
  EV_REQUIRE(cin == 1 || (cin % CK) == 0, "conv3x3_fwd: cin=%d must be 1 or a multiple of %d", cin, CK);
  EV_REQUIRE(cin != 1 || cout == 32, "conv3x3_fwd: cin=1 supports cout=32 only");
  EV_REQUIRE(!act_out || cin != 1, "conv3x3_fwd: act_out needs cin > 1");
  EV_REQUIRE(plan_conv(H, W, cin, cout, &c), "conv3x3_fwd: unsupported shape H=%d W=%d cin=%d cout=%d",
             H, W, cin, cout);
  hipStream_t s = (hipStream_t)stream;
  if (c.kind == 2) {
    launch_small<4, 4, 1, true, FP_NONE>(c, src, src_stats, src_mode, wpack, bias, y, stat_part, act_out, B, H, W, cin, cout, s);
  } else if (c.kind == 1) {
    launch_small<2, 1, 1, false, FP_NONE>(c, src, src_stats, src_mode, wpack, bias, y, stat_part, act_out, B, H, W, cin, cout, s);
  } else if (cout == 128) {
    launch_big<8, 4, 2, 2, 2>(c, src, src_stats, src_mode, wpack, bias, y, stat_part, act_out, B, H, W, cin, s);
  } else if (cout == 64) {
    launch_big<4, 4, 2, 2, 5>(c, src, src_stats, src_mode, wpack, bias, y, stat_part, act_out, B, H, W, cin, s);
  } else {
    launch_big<4, 4, 4, 1, 9>(c, src, src_stats, src_mode, wpack, bias, y, stat_part, act_out, B, H, W, cin, s);
  }
  return evh::check_launch("conv3x3_fwd");
}

extern "C" int ebsdvae_conv3x3_dgrad_inbwd(const float* g, const float* wpack, float* gin,
                                           const float* y_prev, const float* st_prev, int pmode,
                                           double* part, int B, int H, int W, int cin, int cout,
                                           ebsdvae_stream_t stream) {
  Cfg c;
  EV_REQUIRE(g && wpack && gin && y_prev && st_prev && part && B > 0,
             "conv3x3_dgrad_inbwd: null pointer or empty batch");
  EV_REQUIRE(pmode == P_ID || pmode == P_POOL || pmode == P_UP, "conv3x3_dgrad_inbwd: bad pmode %d", pmode);
  EV_REQUIRE(cin % CK == 0 && (W & (W - 1)) == 0 && (pmode != P_UP || (H % 2 == 0 && W % 2 == 0)),
             "conv3x3_dgrad_inbwd: cin=%d W=%d unsupported", cin, W);
  EV_REQUIRE(plan_conv(H, W, cin, cout, &c) && c.kind != 2,
             "conv3x3_dgrad_inbwd: unsupported shape H=%d W=%d cin=%d cout=%d", H, W, cin, cout);
  hipStream_t s = (hipStream_t)stream;
  InBwdFuse f;
  f.yprev = y_prev;
  f.stprev = (const float2*)st_prev;
  f.part = (double2*)part;
  if (c.kind == 1) {
    switch (pmode) {
      case P_ID: launch_small<2, 1, 1, false, P_ID>(c, g, nullptr, ACT_RAW, wpack, nullptr, gin, nullptr, nullptr, B, H, W, cin, cout, s, f); break;
      case P_POOL: launch_small<2, 1, 1, false, P_POOL>(c, g, nullptr, ACT_RAW, wpack, nullptr, gin, nullptr, nullptr, B, H, W, cin, cout, s, f); break;
      default: launch_small<2, 1, 1, false, P_UP>(c, g, nullptr, ACT_RAW, wpack, nullptr, gin, nullptr, nullptr, B, H, W, cin, cout, s, f); break;
    }
  } else if (cout == 128) {
    launch_big_fused<8, 4, 2, 2, 2>(c, g, wpack, gin, B, H, W, cin, s, pmode, f);
  } else if (cout == 64) {
    launch_big_fused<4, 4, 2, 2, 5>(c, g, wpack, gin, B, H, W, cin, s, pmode, f);
  } else {
    launch_big_fused<4, 4, 4, 1, 9>(c, g, wpack, gin, B, H, W, cin, s, pmode, f);
  }
  return evh::check_launch("conv3x3_dgrad_inbwd");
}
