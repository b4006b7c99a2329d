// 3x3 stride-1 pad-1 convolution (forward and input gradient) on the bf16 MFMA with split
// operands: every fp32 operand x is carried as NP bf16 pieces
//     x0 = bf16(x), x1 = bf16(x - x0) [, x2 = bf16(x - x0 - x1)]
// (8 mantissa bits each; |x - sum| <= 2^-18 |x| for NP = 2, 2^-27 |x| for NP = 3), and each
// product keeps the terms of total order < NP (bf16 x bf16 products are exact in fp32,
// accumulation is fp32):
//   NP = 2 ("bf16x3"): a0b0 + a0b1 + a1b0                    3 MFMAs, ~2^-16.5 rel. error
//   NP = 3 ("bf16x6"): + a0b2 + a2b0 + a1b1                  6 MFMAs, ~2^-25 (fp32 grade)
// at 16x the fp32-MFMA rate per v_mfma_f32_32x32x16_bf16: 5.3x / 2.7x the fp32 MFMA peak
// (split-precision MFMA path, gated by the parity tests).  Replaces the same reference ops as conv_fwd.hip:
// nn.Conv2d / nn.ConvTranspose2d forward (latice/model.py:95,102-104) and their input
// gradients, with the same fused prologue (InstanceNorm + LeakyReLU [+ pool / upsample] of
// the producer's saved output) and epilogue (bias, InstanceNorm partials, optional fused
// InstanceNorm-backward reduce).
//
// GEMM view as in conv_fwd.hip: M = output pixels, N = Cout, K = 9 taps x Cin swept in
// 8-channel chunks.  One 32x32x16 k-step covers two taps: lane half h = lane >> 5 takes tap
// 2s + h (s = 0..4; a zero tenth tap pads the odd tap count).
//   LDS halo record per pixel (48 B): piece 0 [8 ch] | piece 1 [8 ch] | piece 2 or pad ->
//     one ds_read_b128 per piece, conflict-free over 16 consecutive pixels (3 x 16 B granules
//     apart);
//   LDS weight slab per chunk: [tap 0..9][piece][Cout][8 ch] bf16, DMA'd by global_load_lds
//     from the split pack (ebsdvae_pack_conv_weights_split).
#include "conv_common.h"

namespace ev {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

constexpr int XCK = 8;      // input channels per chunk
constexpr int XTAPS = 10;   // 9 taps + one zero tap
constexpr int XPS = 48;     // halo pixel record (bytes)

// x -> NP bf16 pieces (the remainder is re-split exactly in fp32 at every step)
template <int NP>
EV_DEVINL void split_bf16(float x, __bf16 (&p)[NP]) {
  float r = x;
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    p[i] = (__bf16)r;
    r -= (float)p[i];
  }
}

template <int NP>
EV_DEVINL void split4(float4 v, bf16x4 (&out)[NP]) {
  const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    __bf16 p[NP];
    split_bf16<NP>(e[c], p);
#pragma unroll
    for (int i = 0; i < NP; ++i) out[i][c] = p[i];
  }
}

EV_DEVINL bf16x8 lds_frag(const char* p) { return *reinterpret_cast<const bf16x8*>(p); }

template <int NP, int NWV, int WM, int MF, int NF, int KX, int MODE, int FP>
__global__ __launch_bounds__(NWV * 64, 2) void conv3x3_split_kernel(
    const float* __restrict__ src, const float2* __restrict__ sstats, const char* __restrict__ wp,
    const float* __restrict__ bias, float* __restrict__ y, float2* __restrict__ spart,
    float* __restrict__ act_out, int B, int H, int W, int Cin, int TH,
    const float* __restrict__ yprev, const float2* __restrict__ stprev, double2* __restrict__ ipart) {
  constexpr int WN = NWV / WM;
  constexpr int NT = WN * NF * 32;               // == Cout
  constexpr int MW = MF * 32;
  constexpr int NTHR = NWV * 64;
  constexpr int WSLAB = XTAPS * NP * NT * 16;    // bytes per weight chunk
  constexpr bool POOL = (MODE == ACT_NORM_POOL);
  constexpr bool NORM = (MODE == ACT_NORM || MODE == ACT_NORM_POOL || MODE == ACT_NORM_UP);
  constexpr bool UPS = (MODE == ACT_UP || MODE == ACT_NORM_UP);
  constexpr int NR = POOL ? 4 : 1;
  extern __shared__ __attribute__((aligned(16))) char xsm[];
  const int HP = TH + 2, WP = W + 2;
  const int pixP = HP * WP;
  const int xslab = (pixP + 1) * XPS;   // + one dummy record for out-of-halo items
  char* lw0 = xsm;
  char* lx0 = xsm + 2 * WSLAB;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int l32 = lane & 31, hk = lane >> 5;
  const int tpi = H / TH;
  const int b0 = blockIdx.x / tpi;
  const int h0 = (blockIdx.x % tpi) * TH;
  const int tpx = TH * W;

  // A rows: halo pixel of this lane's output pixel for each m-fragment
  int abase[MF];
#pragma unroll
  for (int mf = 0; mf < MF; ++mf) {
    const int p = wm * MW + mf * 32 + l32;
    const int r = p / W, c = p - r * W;
    abase[mf] = r * WP + c;
  }
  // this lane half's tap of k-step s (tap 9 reads tap 8's pixels; its weights are zero)
  int toff[5];
#pragma unroll
  for (int s = 0; s < 5; ++s) {
    const int t = min(2 * s + hk, 8);
    toff[s] = (t / 3) * WP + t % 3;
  }

  const int Hs = POOL ? 2 * H : (UPS ? H / 2 : H);
  const int Ws = POOL ? 2 * W : (UPS ? W / 2 : W);
  const float* sb = src + (size_t)b0 * Hs * Ws * Cin;
  const int q = tid & 1;   // this thread's 4-channel half of every 8-channel chunk

  // halo item k: pixel (tid + NTHR*k) >> 1, channels q*4..q*4+3; chunk-invariant source
  // coordinates packed as (gh << 16) | gw, -1 = zero padding / past the halo
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
  int cur_ch = 0;
  auto issue_halo = [&](int ch) {   // branch-free: padding items load a safe address
    cur_ch = ch;
    const int c = ch * XCK + q * 4;
#pragma unroll
    for (int k = 0; k < KX; ++k) {
      const int hv = hw[k] < 0 ? 0 : hw[k];
      const int gh = hv >> 16, gw = hv & 0xffff;
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
  auto store_halo = [&](char* lx) {
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
      if (act_out) {   // uniform: materialise the (pooled) activation for the wgrad
        const int gh = hw[k] >> 16, gw = hw[k] & 0xffff;
        if (ok && gh >= h0 && gh < h0 + TH)
          st4(act_out + (((size_t)b0 * H + gh) * W + gw) * Cin + cur_ch * XCK + q * 4, v);
      }
      bf16x4 pc[NP];
      split4<NP>(v, pc);
      char* d = lx + (pix < pixP ? pix : pixP) * XPS + q * 8;
#pragma unroll
      for (int i = 0; i < NP; ++i) *reinterpret_cast<bf16x4*>(d + 16 * i) = pc[i];
    }
  };
  auto issue_weights = [&](int ch, char* lw) {
    const char* g = wp + (size_t)ch * WSLAB;
    for (int pc = wave; pc < WSLAB / 1024; pc += NWV)
      __builtin_amdgcn_global_load_lds((const void*)(g + pc * 1024 + lane * 16),
                                       (lds_void_ptr)(lw + pc * 1024), 16, 0, 0);
  };

  f32x16 acc[MF][NF];
#pragma unroll
  for (int mf = 0; mf < MF; ++mf)
#pragma unroll
    for (int nf = 0; nf < NF; ++nf)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mf][nf][r] = 0.f;

  const int nchunks = Cin / XCK;
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
    const char* lx = lx0 + cur * xslab;
    const char* lw = lw0 + cur * WSLAB;
#pragma unroll
    for (int s = 0; s < 5; ++s) {
      bf16x8 a[NP][MF], b[NP][NF];
#pragma unroll
      for (int mf = 0; mf < MF; ++mf) {
        const char* pa = lx + (abase[mf] + toff[s]) * XPS;
#pragma unroll
        for (int i = 0; i < NP; ++i) a[i][mf] = lds_frag(pa + 16 * i);
      }
      const int t = 2 * s + hk;
#pragma unroll
      for (int nf = 0; nf < NF; ++nf) {
        const char* pb = lw + ((t * NP) * NT + ncol + nf * 32) * 16;
#pragma unroll
        for (int i = 0; i < NP; ++i) b[i][nf] = lds_frag(pb + i * NT * 16);
      }
      // terms of total order < NP, smallest first
#pragma unroll
      for (int mf = 0; mf < MF; ++mf)
#pragma unroll
        for (int nf = 0; nf < NF; ++nf) {
          if (NP == 3) {
            acc[mf][nf] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][mf], b[NP - 2][nf], acc[mf][nf], 0, 0, 0);
            acc[mf][nf] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[NP - 1][mf], b[0][nf], acc[mf][nf], 0, 0, 0);
            acc[mf][nf] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][mf], b[NP - 1][nf], acc[mf][nf], 0, 0, 0);
          }
          acc[mf][nf] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][mf], b[0][nf], acc[mf][nf], 0, 0, 0);
          acc[mf][nf] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][mf], b[1][nf], acc[mf][nf], 0, 0, 0);
          acc[mf][nf] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][mf], b[0][nf], acc[mf][nf], 0, 0, 0);
        }
    }
    if (more) store_halo(lx0 + nxt * xslab);
    __syncthreads();
  }
  conv_epilogue<MF, NF, FP>(acc, bias, y, spart, B, H, W, NT, b0, h0, tpx, wm * MW, wn * NF * 32, hk,
                            l32, yprev, stprev, ipart);
}

// split weight pack: [chunk][tap 0..9][piece][co'][8 ci'] bf16 of the conv-equivalent
// weight (tap 9 = 0); (ci', co') = (cin, cout) of the layer, swapped for the input gradient.
__global__ void pack_split_kernel(const PackBatch pb, int np) {
  const ebsdvae_pack_desc& q = pb.d[blockIdx.y];
  const int ci_ = q.for_dgrad ? q.cout : q.cin;
  const int co_ = q.for_dgrad ? q.cin : q.cout;
  const int nch = ci_ / XCK;
  const int n = nch * XTAPS * co_ * XCK;
  __bf16* d = reinterpret_cast<__bf16*>(q.dst);
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    const int c8 = e % XCK;
    int r = e / XCK;
    const int o = r % co_;
    r /= co_;
    const int t = r % XTAPS, chunk = r / XTAPS;
    float w = 0.f;
    if (t < 9) {
      const int i = chunk * XCK + c8;
      const int co = q.for_dgrad ? i : o;
      const int ci = q.for_dgrad ? o : i;
      size_t idx;
      if (q.kind == 0) idx = ((size_t)co * q.cin + ci) * 9 + (q.for_dgrad ? 8 - t : t);
      else idx = ((size_t)ci * q.cout + co) * 9 + (q.for_dgrad ? t : 8 - t);
      w = q.src[idx];
    }
    const size_t base = ((size_t)(chunk * XTAPS + t) * np) * co_ * XCK + (size_t)o * XCK + c8;
    float rr = w;
    for (int i = 0; i < np; ++i) {
      const __bf16 p = (__bf16)rr;
      rr -= (float)p;
      d[base + (size_t)i * co_ * XCK] = p;
    }
  }
}

struct X3Cfg {
  int M, TH, NT, KX, nwv;
  size_t lds;
};

// NP = 2: Cout 128 -> 8 waves x M 256; Cout 64 / 32 -> 4 waves x M 256 (2 blocks / CU).
// NP = 3: the 3-piece weight slab is 1.5x larger, so every Cout runs 8 waves (M 256 for
// Cout 128, M 512 otherwise) with one block per CU.
static bool plan_split(int H, int W, int cin, int cout, int np, X3Cfg* c) {
  if ((np != 2 && np != 3) || cin % XCK || !(cout == 128 || cout == 64 || cout == 32)) return false;
  c->M = (np == 3 && cout != 128) ? 512 : 256;
  if (H * W < c->M || W > c->M || c->M % W) return false;
  c->TH = c->M / W;
  if (H % c->TH) return false;
  c->NT = cout;
  c->nwv = (cout == 128 || np == 3) ? 8 : 4;
  const int pix = (c->TH + 2) * (W + 2);
  c->KX = (pix * 2 + c->nwv * 64 - 1) / (c->nwv * 64);
  const int kxmax = np == 2 ? (cout == 128 ? 2 : (cout == 64 ? 5 : 7)) : (cout == 128 ? 2 : (cout == 64 ? 4 : 5));
  if (c->KX > kxmax) return false;
  c->lds = 2 * (size_t)XTAPS * np * cout * 16 + 2 * (size_t)(pix + 1) * XPS;
  return c->lds <= 160 * 1024;
}

template <int NP, int NWV, int WM, int MF, int NF, int KX, int MODE, int FP>
static void launch_x3_1(const X3Cfg& c, const float* src, const float* st, const void* wp,
                        const float* bias, float* y, float* part, float* aout, int B, int H, int W,
                        int cin, hipStream_t s, const InBwdFuse& f) {
  auto k = conv3x3_split_kernel<NP, NWV, WM, MF, NF, KX, MODE, FP>;
  static bool once = false;
  if (!once) {
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    once = true;
  }
  hipLaunchKernelGGL(k, dim3(B * (H / c.TH)), dim3(NWV * 64), c.lds, s, src, (const float2*)st,
                     (const char*)wp, bias, y, (float2*)part, aout, B, H, W, cin, c.TH, f.yprev,
                     f.stprev, f.part);
}

template <int NP, int NWV, int WM, int MF, int NF, int KX>
static void launch_x3(const X3Cfg& c, const float* src, const float* st, int mode, const void* wp,
                      const float* bias, float* y, float* part, float* aout, int B, int H, int W,
                      int cin, hipStream_t s, int pmode, const InBwdFuse& f) {
  if (pmode >= 0) {
    switch (pmode) {
      case P_ID: launch_x3_1<NP, NWV, WM, MF, NF, KX, ACT_RAW, P_ID>(c, src, nullptr, wp, nullptr, y, nullptr, nullptr, B, H, W, cin, s, f); break;
      case P_POOL: launch_x3_1<NP, NWV, WM, MF, NF, KX, ACT_RAW, P_POOL>(c, src, nullptr, wp, nullptr, y, nullptr, nullptr, B, H, W, cin, s, f); break;
      default: launch_x3_1<NP, NWV, WM, MF, NF, KX, ACT_RAW, P_UP>(c, src, nullptr, wp, nullptr, y, nullptr, nullptr, B, H, W, cin, s, f); break;
    }
    return;
  }
  switch (mode) {
    case ACT_RAW: launch_x3_1<NP, NWV, WM, MF, NF, KX, ACT_RAW, FP_NONE>(c, src, st, wp, bias, y, part, aout, B, H, W, cin, s, f); break;
    case ACT_NORM: launch_x3_1<NP, NWV, WM, MF, NF, KX, ACT_NORM, FP_NONE>(c, src, st, wp, bias, y, part, aout, B, H, W, cin, s, f); break;
    case ACT_NORM_POOL: launch_x3_1<NP, NWV, WM, MF, NF, KX, ACT_NORM_POOL, FP_NONE>(c, src, st, wp, bias, y, part, aout, B, H, W, cin, s, f); break;
    case ACT_UP: launch_x3_1<NP, NWV, WM, MF, NF, KX, ACT_UP, FP_NONE>(c, src, st, wp, bias, y, part, aout, B, H, W, cin, s, f); break;
    default: launch_x3_1<NP, NWV, WM, MF, NF, KX, ACT_NORM_UP, FP_NONE>(c, src, st, wp, bias, y, part, aout, B, H, W, cin, s, f); break;
  }
}

static void dispatch_split(const X3Cfg& c, int np, const float* src, const float* st, int mode,
                           const void* wp, const float* bias, float* y, float* part, float* aout,
                           int B, int H, int W, int cin, int cout, hipStream_t s, int pmode,
                           const InBwdFuse& f) {
  if (np == 2) {
    if (cout == 128)
      launch_x3<2, 8, 4, 2, 2, 2>(c, src, st, mode, wp, bias, y, part, aout, B, H, W, cin, s, pmode, f);
    else if (cout == 64)
      launch_x3<2, 4, 4, 2, 2, 5>(c, src, st, mode, wp, bias, y, part, aout, B, H, W, cin, s, pmode, f);
    else
      launch_x3<2, 4, 4, 2, 1, 7>(c, src, st, mode, wp, bias, y, part, aout, B, H, W, cin, s, pmode, f);
  } else {
    if (cout == 128)
      launch_x3<3, 8, 4, 2, 2, 2>(c, src, st, mode, wp, bias, y, part, aout, B, H, W, cin, s, pmode, f);
    else if (cout == 64)
      launch_x3<3, 8, 8, 2, 2, 4>(c, src, st, mode, wp, bias, y, part, aout, B, H, W, cin, s, pmode, f);
    else
      launch_x3<3, 8, 8, 2, 1, 5>(c, src, st, mode, wp, bias, y, part, aout, B, H, W, cin, s, pmode, f);
  }
}

}  // namespace ev

using namespace ev;

extern "C" int ebsdvae_conv3x3_split_supported(int H, int W, int cin, int cout, int pieces) {
  X3Cfg c;
  return plan_split(H, W, cin, cout, pieces, &c) ? 1 : 0;
}

extern "C" int ebsdvae_conv3x3_split_stat_tiles(int H, int W, int cout) {
  (void)cout;
  return (H * W) / 64;   // every split configuration has 64-pixel wave tiles
}

extern "C" size_t ebsdvae_pack_split_bytes(int cin, int cout, int pieces) {
  return (size_t)(cin / XCK) * XTAPS * pieces * cout * XCK * 2;
}

extern "C" int ebsdvae_pack_conv_weights_split(const ebsdvae_pack_desc* descs, int n, int pieces,
                                               ebsdvae_stream_t stream) {
  EV_REQUIRE(descs && n > 0 && n <= EBSDVAE_MAX_PACK, "pack_conv_weights_split: n=%d out of range", n);
  EV_REQUIRE(pieces == 2 || pieces == 3, "pack_conv_weights_split: pieces=%d (2 or 3)", pieces);
  PackBatch pb;
  int maxn = 0;
  for (int i = 0; i < n; ++i) {
    const ebsdvae_pack_desc& q = descs[i];
    const int ci_ = q.for_dgrad ? q.cout : q.cin;
    EV_REQUIRE(q.src && q.dst && q.cin > 0 && q.cout > 0 && (q.kind == 0 || q.kind == 1) && ci_ % XCK == 0,
               "pack_conv_weights_split: bad descriptor %d", i);
    pb.d[i] = q;
    const int e = (ci_ / XCK) * XTAPS * (q.for_dgrad ? q.cin : q.cout) * XCK;
    if (e > maxn) maxn = e;
  }
  int bx = (maxn + 255) / 256;
  if (bx > 64) bx = 64;
  hipLaunchKernelGGL(pack_split_kernel, dim3(bx, n), dim3(256), 0, (hipStream_t)stream, pb, pieces);
  return evh::check_launch("pack_conv_weights_split");
}

extern "C" int ebsdvae_conv3x3_fwd_split(const float* src, const float* src_stats, int src_mode,
                                         const void* wpack, const float* bias, float* y,
                                         float* stat_part, float* act_out, int B, int H, int W,
                                         int cin, int cout, int pieces, ebsdvae_stream_t stream) {
  X3Cfg c;
  EV_REQUIRE(src && wpack && y && B > 0, "conv3x3_fwd_split: null pointer or empty batch");
  EV_REQUIRE(src_mode >= 0 && src_mode <= 4, "conv3x3_fwd_split: bad src_mode %d", src_mode);
  EV_REQUIRE(src_mode == ACT_RAW || src_mode == ACT_UP || src_stats,
             "conv3x3_fwd_split: NORM modes need src_stats");
  EV_REQUIRE(plan_split(H, W, cin, cout, pieces, &c),
             "conv3x3_fwd_split: unsupported shape H=%d W=%d cin=%d cout=%d pieces=%d", H, W, cin, cout,
             pieces);
  dispatch_split(c, pieces, src, src_stats, src_mode, wpack, bias, y, stat_part, act_out, B, H, W,
                 cin, cout, (hipStream_t)stream, -1, InBwdFuse());
  return evh::check_launch("conv3x3_fwd_split");
}

extern "C" int ebsdvae_conv3x3_dgrad_inbwd_split(const float* g, const void* wpack, float* gin,
                                                 const float* y_prev, const float* st_prev,
                                                 int pmode, double* part, int B, int H, int W,
                                                 int cin, int cout, int pieces,
                                                 ebsdvae_stream_t stream) {
  X3Cfg c;
  EV_REQUIRE(g && wpack && gin && B > 0, "conv3x3_dgrad_inbwd_split: null pointer or empty batch");
  EV_REQUIRE(pmode >= -1 && pmode <= P_UP, "conv3x3_dgrad_inbwd_split: bad pmode %d", pmode);
  EV_REQUIRE(pmode < 0 || (y_prev && st_prev && part && (W & (W - 1)) == 0),
             "conv3x3_dgrad_inbwd_split: fused reduce needs y_prev, st_prev, part and W = 2^k");
  EV_REQUIRE(plan_split(H, W, cin, cout, pieces, &c),
             "conv3x3_dgrad_inbwd_split: unsupported shape H=%d W=%d cin=%d cout=%d pieces=%d", H, W,
             cin, cout, pieces);
  InBwdFuse f;
  f.yprev = y_prev;
  f.stprev = (const float2*)st_prev;
  f.part = (double2*)part;
  dispatch_split(c, pieces, g, nullptr, ACT_RAW, wpack, nullptr, gin, nullptr, nullptr, B, H, W, cin,
                 cout, (hipStream_t)stream, pmode, f);
  return evh::check_launch("conv3x3_dgrad_inbwd_split");
}
