// Shared device helpers for the ebsd-vae MI355X kernels (gfx950 / CDNA4 only).
//
// Conventions used by every kernel in this library:
//  * activations are NHWC fp32, index ((b*H + h)*W + w)*C + c;
//  * a conv block's saved tensor is its PRE-norm output y (conv + bias); the
//    normalised activation lrelu((y-mean)*rstd) is never written to HBM: consumers
//    recompute it while staging their input tile (the "act source" below);
//  * InstanceNorm statistics are float2 {mean, rstd} per (b, c);
//  * launches never allocate, free or synchronise; every buffer is owned by the caller.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define EV_DEVINL __device__ __forceinline__
// device lambdas that must inline (a call spills the whole register state)
#define EV_LAMBDA_INLINE __attribute__((always_inline))

namespace ev {

constexpr float kSlope = 0.02f;   // LeakyReLU(0.02), latice/model.py:97,106
constexpr float kInEps = 1e-5f;   // InstanceNorm2d default eps, latice/model.py:96,105

// How a conv (or any consumer) reads its logical input at (b, h, w, c) from a source
// tensor.  Matches the block boundaries of latice/model.py:109-148.
enum ActMode : int {
  ACT_RAW = 0,        // src itself, same resolution
  ACT_NORM = 1,       // lrelu((src - mean) * rstd), same resolution (conv -> IN -> LReLU)
  ACT_NORM_POOL = 2,  // max over 2x2 of ACT_NORM of src at 2x resolution (MaxPool2d(2,2))
  ACT_UP = 3,         // src at half resolution, nearest x2 (UpsamplingNearest2d(2))
  ACT_NORM_UP = 4,    // ACT_NORM of src at half resolution, nearest x2
};

// max(v, slope*v) == (v > 0 ? v : slope*v) bit for bit for 0 < slope < 1 (2 VALU ops)
EV_DEVINL float lrelu(float v) { return fmaxf(v, kSlope * v); }

EV_DEVINL float normact(float v, float2 st) { return lrelu((v - st.x) * st.y); }

// how a block's output reaches its consumer (InstanceNorm backward routing)
enum PMode : int { P_ID = 0, P_POOL = 1, P_UP = 2, P_UPSUM = 3 /* dgrad_inbwd_split only */ };
// d lrelu / d xhat
EV_DEVINL float slope(float xh) { return xh > 0.f ? 1.f : kSlope; }

// {mean, rstd} -> {rstd, -mean*rstd}: normact as one FMA + lrelu (staging hot loops)
EV_DEVINL float2 norm_fs(float2 st) { return make_float2(st.y, -st.x * st.y); }
EV_DEVINL float normact_fs(float v, float2 fs) { return lrelu(fmaf(v, fs.x, fs.y)); }

EV_DEVINL float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
// non-temporal (CPol NT) forms for single-use stream traffic, so the L2 keeps what other
// kernels re-read
typedef float f32v4 __attribute__((ext_vector_type(4)));
EV_DEVINL float4 ld4_nt(const float* p) {
  const f32v4 v = __builtin_nontemporal_load(reinterpret_cast<const f32v4*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}
EV_DEVINL void st4_nt(float* p, float4 v) {
  __builtin_nontemporal_store(f32v4{v.x, v.y, v.z, v.w}, reinterpret_cast<f32v4*>(p));
}

// The first conv (1 -> C, latice/model.py:110) at one pixel and one output channel: nb[t] =
// x[h + t/3 - 1][w + t%3 - 1] (0 outside the image), wt = the channel's 9 taps.  One fixed fma
// chain, shared by the forward (conv_first_fwd_kernel) and the first block's backward, which
// recomputes y0 from x with it instead of re-reading y0 (bit-identical by construction).
EV_DEVINL float first_conv_px(const float (&nb)[9], const float (&wt)[9], float bias) {
  float s = nb[0] * wt[0];
#pragma unroll
  for (int t = 1; t < 9; ++t) s = fmaf(nb[t], wt[t], s);
  return s + bias;
}
// Two channels of first_conv_px at once on v_pk_fma_f32 (each lane of the pair runs exactly
// first_conv_px's chain, so the values are bit-identical): w2[t] = the two channels' tap t.
typedef float pkf2 __attribute__((ext_vector_type(2)));
EV_DEVINL pkf2 pk2(float a, float b) { return pkf2{a, b}; }
EV_DEVINL pkf2 pkfma(pkf2 a, pkf2 b, pkf2 c) { return __builtin_elementwise_fma(a, b, c); }
EV_DEVINL pkf2 first_conv_px2(const float (&nb)[9], const pkf2 (&w2)[9], pkf2 b2) {
  pkf2 s = pk2(nb[0], nb[0]) * w2[0];
#pragma unroll
  for (int t = 1; t < 9; ++t) s = pkfma(pk2(nb[t], nb[t]), w2[t], s);
  return s + b2;
}
EV_DEVINL void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }

EV_DEVINL float4 max4(float4 a, float4 b) {
  return make_float4(fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z), fmaxf(a.w, b.w));
}

// 4 consecutive channels (c..c+3) of the logical input at (b,h,w); (h,w) in bounds.
// H, W are the LOGICAL (consumer) dimensions, C the source channel count.
EV_DEVINL float4 load_act4(const float* __restrict__ src, const float2* __restrict__ stats,
                           int mode, int b, int h, int w, int c, int H, int W, int C) {
  float4 v;
  if (mode == ACT_RAW) {
    v = ld4(src + (((size_t)b * H + h) * W + w) * C + c);
    return v;
  }
  if (mode == ACT_UP || mode == ACT_NORM_UP) {
    const int Hs = H >> 1, Ws = W >> 1;
    v = ld4(src + (((size_t)b * Hs + (h >> 1)) * Ws + (w >> 1)) * C + c);
    if (mode == ACT_UP) return v;
  } else if (mode == ACT_NORM_POOL) {
    const int Hs = H << 1, Ws = W << 1;
    const float* p = src + (((size_t)b * Hs + 2 * h) * Ws + 2 * w) * C + c;
    // max before normalising: x -> lrelu((x-m)*r) is monotone non-decreasing in fp32,
    // so max(f(x_i)) == f(max(x_i)) bit for bit.
    v = max4(max4(ld4(p), ld4(p + C)), max4(ld4(p + (size_t)Ws * C), ld4(p + (size_t)Ws * C + C)));
  } else {  // ACT_NORM
    v = ld4(src + (((size_t)b * H + h) * W + w) * C + c);
  }
  const float2* s = stats + (size_t)b * C + c;
  float2 s0 = s[0], s1 = s[1], s2 = s[2], s3 = s[3];
  return make_float4(normact(v.x, s0), normact(v.y, s1), normact(v.z, s2), normact(v.w, s3));
}

// single-channel variant (C == 1 sources, e.g. the input patterns)
EV_DEVINL float load_act1(const float* __restrict__ src, const float2* __restrict__ stats,
                          int mode, int b, int h, int w, int c, int H, int W, int C) {
  float v;
  if (mode == ACT_RAW) return src[(((size_t)b * H + h) * W + w) * C + c];
  if (mode == ACT_UP || mode == ACT_NORM_UP) {
    const int Hs = H >> 1, Ws = W >> 1;
    v = src[(((size_t)b * Hs + (h >> 1)) * Ws + (w >> 1)) * C + c];
    if (mode == ACT_UP) return v;
  } else if (mode == ACT_NORM_POOL) {
    const int Ws = W << 1, Hs = H << 1;
    const float* p = src + (((size_t)b * Hs + 2 * h) * Ws + 2 * w) * C + c;
    v = fmaxf(fmaxf(p[0], p[C]), fmaxf(p[(size_t)Ws * C], p[(size_t)Ws * C + C]));
  } else {
    v = src[(((size_t)b * H + h) * W + w) * C + c];
  }
  return normact(v, stats[(size_t)b * C + c]);
}

// wave64 reductions (DPP/permute via __shfl_xor; width 64)
EV_DEVINL float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// ---- split-fp16 piece format ("f16x3", include/ebsdvae.h EBSDVAE_PIECES_F16): two fp16
// pieces x0 = f16(x), x1 = f16(x - x0) per operand, products a0b0 + a0b1 + a1b0 on the fp16
// MFMA.  Weights are packed as w * 2^k with one power of two per layer from its max |w|
// (f16_wshift, stored in the pack's trailer); gradient operands are scaled by a power of two
// from their maximum (f16_shift) so that both sit inside fp16's range.
constexpr int NP_F16 = 16;   // == EBSDVAE_PIECES_F16
// bytes after the split-fp16 pack: int32 weight shift k (16-byte head), then the
// kF16MaxParts partial maxima of |w| it is computed from (pack_wmax_kernel)
constexpr int kF16MaxParts = 64;
constexpr int kF16PackTrailer = 16 + 4 * kF16MaxParts;
constexpr int npc(int np) { return np == NP_F16 ? 2 : np; }   // pieces per operand

// Two floats -> their split-fp16 pieces, packed: hi = (f16(a), f16(b)) round-to-nearest
// (v_cvt_pk_f16_f32), lo = (f16(a - hi.x), f16(b - hi.y)) by v_fma_mix{lo,hi}_f16, which
// forms the residual in fp32 (exact: hi is a's leading bits) and rounds it once -- the same
// bits as the scalar cvt / cvt-back / subtract / cvt sequence, in 3 instructions instead of 8.
EV_DEVINL void split_f16x2(float a, float b, unsigned& hi, unsigned& lo) {
  typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
  const h2_t h = {(_Float16)a, (_Float16)b};
  hi = __builtin_bit_cast(unsigned, h);
  asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %0, %1, -1.0, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
      : "=&v"(lo) : "v"(hi), "v"(a), "v"(b));
}
// split_f16x2 of (a * s, b * s) for a power of two s (the gradient operands' scale): the
// products are exact in fp32, so hi = f16(a s) by one v_fma_mix (a s + 0) and lo = f16(a s - hi)
// by another (fma_mix forms a s - hi exactly and rounds once) -- the same bits as scaling first
// and splitting, in 4 instructions instead of 5
EV_DEVINL void split_f16x2_scaled(float a, float b, float s, unsigned& hi, unsigned& lo) {
  asm("v_fma_mixlo_f16 %0, %2, %4, 0\n\t"
      "v_fma_mixhi_f16 %0, %3, %4, 0\n\t"
      "v_fma_mixlo_f16 %1, %2, %4, -%0 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %1, %3, %4, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(hi), "=&v"(lo) : "v"(a), "v"(b), "v"(s));
}
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// k such that m * 2^k lies in [2^11, 2^12) (0 for a zero / non-finite maximum)
EV_DEVINL int f16_shift_of(float m) {
  if (!(m > 0.f) || !(m <= 3.4e38f)) return 0;
  int e;
  (void)frexpf(m, &e);   // m = f * 2^e, f in [0.5, 1)
  return min(max(12 - e, -100), 100);
}
// the shift of images [b0, b1] from per-tile maxima gmax (B, gmT) (0 without them)
EV_DEVINL int f16_gshift(const float* __restrict__ gmax, int gmT, int b0, int b1) {
  if (!gmax) return 0;
  float m = 0.f;
  for (size_t i = (size_t)b0 * gmT; i < (size_t)(b1 + 1) * gmT; ++i) m = fmaxf(m, gmax[i]);
  return f16_shift_of(m);
}
EV_DEVINL int f16_gshift(const float* __restrict__ gmax, int gmT, int b) {
  return f16_gshift(gmax, gmT, b, b);
}

}  // namespace ev

// ---------------------------------------------------------------- host-side error plumbing
namespace evh {
void set_error(const char* fmt, ...);
int check_launch(const char* what);
// the event armed by ebsdvae_fork_arm for the next gy-producing launch (nullptr if none); the
// caller attaches it to that launch (hipExtLaunchKernel stopEvent)
hipEvent_t take_fork_event();
// compute units a stream may run on: the count registered by ebsdvae_stream_create_cus for a
// CU-masked stream, else 0 (the device's; the persistent kernels size their grids by it)
int stream_cus(hipStream_t s);
}  // namespace evh

// a spatial extent the shape queries accept (H * W and its multiples stay inside int)
inline bool ev_dim_ok(int n) { return n > 0 && n <= 65536 && (long long)n * n <= (1LL << 30); }
// a per-image byte range the 32-bit buffer descriptors can address (num_records and the
// offsets are 32-bit; out-of-range reads return 0, so an overflow would read zeros silently)
inline bool ev_buf_bytes_ok(long long bytes) { return bytes > 0 && bytes < (1LL << 31); }

#define EV_REQUIRE(cond, ...)        \
  do {                               \
    if (!(cond)) {                   \
      evh::set_error(__VA_ARGS__);   \
      return 1;                      \
    }                                \
  } while (0)
