// Latent heads, reparameterisation and sampler (latice/model.py:25-38, 55-64, 127-131).
//
//   flat   = encoder_out.flatten(1,-1)            NCHW order: k = c*S*S + h*S + w
//   mu     = flat @ Wmu^T + bmu ; logvar = flat @ Wlv^T + blv      (Linear(F, L))
//   std    = exp(logvar / 2) ;  z = mu + eps * std                (Normal(mu,std).rsample)
//   dec_in = (z @ W2^T + b2).view(B, C, S, S)   -> written NHWC for the decoder
//
// Three small launches per direction, each spread over >= 256 blocks so that every weight and
// activation byte is read once from HBM (the heads are a few MFLOP: what costs is bandwidth
// and latency, and a block-per-pattern layout re-reads every weight matrix B times):
//   heads_dot_partial   split-K over feature chunks of CC channels x S*S pixels (about 128
//                       features, a contiguous range of the NCHW flatten, so every weight row is
//                       read in one run): block (chunk, pattern tile) dots its patterns' chunk
//                       with every output row's matching weights, both staged in LDS; partial
//                       sums per (chunk, pattern, output) go to `work`, and the NCHW copy of the
//                       inputs (flat / g_out) is written on the way
//   heads_*_finalize    per (pattern, latent): the chunk partials summed in chunk order, then
//                       bias + reparameterisation (forward) or the reparameterisation adjoint
//   heads_expand        per (pixel hw, pattern tile): the rank-L (2L) product back to the F
//                       features of pixel hw, written NHWC (linear2 / g_enc), coalesced over c
// Every sum has a fixed order: results are deterministic run to run.
#include "common.h"
#include "../../include/ebsdvae.h"

namespace ev {

constexpr int MAXL = 64;
constexpr int HT = 256;          // threads per heads block

// output rows padded to a power of two in 16..128 (2L <= 128)
static int heads_np(int n) {
  int p = 16;
  while (p < n) p *= 2;
  return p;
}

// Partial dots over one chunk of the features: chunk g = CC consecutive channels c0 = g*CC ..
// at every pixel, i.e. the contiguous feature range k = c0*SS .. (c0+CC)*SS - 1 of the NCHW
// flatten (KC = CC*SS features; every weight row read in one contiguous run):
//   part[(g * B + b) * NP + n] = sum_{k in chunk} A[b, k] * Wrow_n[k]
// with A[b, k = c*SS + hw] = the NHWC input at (hw, c) (runs of CC channels).
// MODE 0: rows = [Wmu; Wlv] (N = 2L) or Wmu (N = L), Wrow_n[k] = w[n * F + k];
// MODE 1: rows = W2^T (N = L), Wrow_n[k] = W2[k * L + n].
// R = BT * NP / 256 patterns per thread; copy (if given) receives A in NCHW flatten order at
// copy[b * cstride + coff + k] (contiguous runs of SS).
template <int MODE, int R>
__global__ __launch_bounds__(HT) void heads_dot_partial_kernel(
    const float* __restrict__ A, const float* __restrict__ w0, const float* __restrict__ w1,
    float* __restrict__ part, float* __restrict__ copy, int cstride, int coff, int B, int C,
    int SS, int CC, int L, int N, int NP, int BT) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int KC = CC * SS, NPP = NP + 1;
  float* Wl = sm;                  // [KC][NP + 1]
  float* Al = sm + KC * NPP;       // [BT][KC + 1]
  const int g = blockIdx.x, b0 = blockIdx.y * BT, c0 = g * CC;
  const int tid = threadIdx.x;
  const int F = C * SS;
  const size_t k0 = (size_t)c0 * SS;
  for (int i = tid; i < NP * KC; i += HT) {
    if (MODE == 0) {   // row n, feature kk: contiguous in kk
      const int n = i / KC, kk = i - n * KC;
      float v = 0.f;
      if (n < L) v = w0[(size_t)n * F + k0 + kk];
      else if (n < N) v = w1[(size_t)(n - L) * F + k0 + kk];
      Wl[kk * NPP + n] = v;
    } else {           // W2 row k0 + kk, column n: contiguous in n
      const int kk = i / NP, n = i - kk * NP;
      Wl[kk * NPP + n] = n < N ? w0[(k0 + kk) * L + n] : 0.f;
    }
  }
  for (int i = tid; i < BT * KC; i += HT) {   // NHWC runs of CC channels
    const int bl = i / KC, r = i - bl * KC;
    const int hw = r / CC, ci = r - hw * CC;
    const int b = b0 + bl;
    Al[bl * (KC + 1) + ci * SS + hw] = b < B ? A[((size_t)b * SS + hw) * C + c0 + ci] : 0.f;
  }
  __syncthreads();
  if (copy) {   // NCHW runs of SS pixels
    for (int i = tid; i < BT * KC; i += HT) {
      const int bl = i / KC, kk = i - bl * KC;
      const int b = b0 + bl;
      if (b < B) copy[(size_t)b * cstride + coff + k0 + kk] = Al[bl * (KC + 1) + kk];
    }
  }
  const int n = tid % NP, bq = tid / NP, PB = HT / NP;
  float acc[R];
#pragma unroll
  for (int i = 0; i < R; ++i) acc[i] = 0.f;
  for (int k = 0; k < KC; ++k) {
    const float w = Wl[k * NPP + n];
#pragma unroll
    for (int i = 0; i < R; ++i) acc[i] = fmaf(Al[(bq + i * PB) * (KC + 1) + k], w, acc[i]);
  }
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int b = b0 + bq + i * PB;
    if (b < B && n < N) part[((size_t)g * B + b) * NP + n] = acc[i];
  }
}

// forward finalize: thread (b, j): mu, std, z (MU_ONLY: mu)
template <bool MU_ONLY>
__global__ __launch_bounds__(HT) void heads_fwd_finalize_kernel(
    const float* __restrict__ part, const float* __restrict__ bmu, const float* __restrict__ blv,
    const float* __restrict__ eps, float* __restrict__ mu, float* __restrict__ stdo,
    float* __restrict__ z, int B, int KS, int L, int NP) {
  const int i = blockIdx.x * HT + threadIdx.x;
  if (i >= B * L) return;
  const int b = i / L, j = i - b * L;
  float m = 0.f, lv = 0.f;
  for (int g = 0; g < KS; ++g) {   // the feature chunks in order
    const float* p = part + ((size_t)g * B + b) * NP;
    m += p[j];
    if (!MU_ONLY) lv += p[L + j];
  }
  m += bmu[j];
  mu[i] = m;
  if (MU_ONLY) return;
  lv += blv[j];
  const float sd = expf(lv * 0.5f);
  stdo[i] = sd;
  z[i] = fmaf(eps[i], sd, m);
}

// backward finalize: thread (b, j): g_z total (linear2 adjoint + direct), then the
// reparameterisation adjoint into gs = [g_mu_tot | g_logvar | g_out] (g_out: the partial pass)
__global__ __launch_bounds__(HT) void heads_bwd_finalize_kernel(
    const float* __restrict__ part, const float* __restrict__ gz, const float* __restrict__ gmu,
    const float* __restrict__ gstd, const float* __restrict__ stdv, const float* __restrict__ eps,
    float* __restrict__ gs, int B, int KS, int L, int NP, int G) {
  const int i = blockIdx.x * HT + threadIdx.x;
  if (i >= B * L) return;
  const int b = i / L, j = i - b * L;
  float gzt = 0.f;
  for (int g = 0; g < KS; ++g) gzt += part[((size_t)g * B + b) * NP + j];
  if (gz) gzt += gz[i];
  const float gmt = gzt + (gmu ? gmu[i] : 0.f);
  const float glv = ((gstd ? gstd[i] : 0.f) + gzt * eps[i]) * stdv[i] * 0.5f;
  gs[(size_t)b * G + j] = gmt;
  gs[(size_t)b * G + L + j] = glv;
}

// out[b, hw, c] (NHWC) = bias[c*SS + hw] + sum_j V[b, j] * M[c*SS + hw][j]
// MODE 0 (linear2): V = z (J = L, vstride L), M[k][j] = W2[k * L + j], bias b2
// MODE 1 (g_enc):   V = gs[:, 0:2L] (J = 2L, vstride G), M[k][j] = j < L ? Wmu[j][k] : Wlv[j-L][k]
template <int MODE, int R>
__global__ __launch_bounds__(HT) void heads_expand_kernel(
    const float* __restrict__ V, int vstride, const float* __restrict__ m0,
    const float* __restrict__ m1, const float* __restrict__ bias, float* __restrict__ out, int B,
    int C, int SS, int L, int J, int BT) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* Ml = sm;                  // [J][C]
  float* Vl = sm + J * C;          // [BT][J]
  const int hw = blockIdx.x, b0 = blockIdx.y * BT;
  const int tid = threadIdx.x;
  const int F = C * SS;
  for (int i = tid; i < J * C; i += HT) {
    float v;
    if (MODE == 0) {
      const int c = i / J, j = i - c * J;   // W2 rows: j fastest (contiguous)
      v = m0[(size_t)(c * SS + hw) * L + j];
      Ml[j * C + c] = v;
    } else {
      const int j = i / C, c = i - j * C;
      v = j < L ? m0[(size_t)j * F + c * SS + hw] : m1[(size_t)(j - L) * F + c * SS + hw];
      Ml[i] = v;
    }
  }
  for (int i = tid; i < BT * J; i += HT) {
    const int bl = i / J, j = i - bl * J;
    const int b = b0 + bl;
    Vl[i] = b < B ? V[(size_t)b * vstride + j] : 0.f;
  }
  __syncthreads();
  const int c = tid % C, bq = tid / C, PB = HT / C;
  const float bb = MODE == 0 ? bias[c * SS + hw] : 0.f;
  float acc[R];
#pragma unroll
  for (int i = 0; i < R; ++i) acc[i] = bb;
  for (int j = 0; j < J; ++j) {
    const float m = Ml[j * C + c];
#pragma unroll
    for (int i = 0; i < R; ++i) acc[i] = fmaf(Vl[(bq + i * PB) * J + j], m, acc[i]);
  }
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int b = b0 + bq + i * PB;
    if (b < B) out[((size_t)b * SS + hw) * C + c] = acc[i];
  }
}

// Weight grads of the three Linear layers as a split-batch reduction: blockIdx.y takes a
// chunk of HB patterns; thread (j, e) (e fastest: coalesced flat / g_out rows) writes its
// chunk's partial dWmu[j][e], dWlv[j][e], dW2[e][j] (stored [j][e]) and, for j == 0,
// db2[e]; threads past F*L take dbmu / dblv.  heads_wgrad_reduce sums the chunks in order.
constexpr int HB = 16;   // patterns per chunk

__global__ __launch_bounds__(256) void heads_wgrad_kernel(
    const float* __restrict__ flat, const float* __restrict__ z, const float* __restrict__ gs,
    float* __restrict__ part, int B, int F, int L) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  const int G = 2 * L + F;
  const size_t FL = (size_t)F * L;
  const size_t per = 3 * FL + F + 2 * L;   // one chunk's partial record
  float* pc = part + (size_t)blockIdx.y * per;
  const int b0 = blockIdx.y * HB, b1 = min(b0 + HB, B);
  if (idx < F * L) {
    const int j = idx / F, e = idx - j * F;
    float am = 0.f, al = 0.f, a2 = 0.f, ab = 0.f;
#pragma unroll 4
    for (int b = b0; b < b1; ++b) {
      const float fv = flat[(size_t)b * F + e];
      const float* gb = gs + (size_t)b * G;
      const float go = gb[2 * L + e];
      am = fmaf(gb[j], fv, am);
      al = fmaf(gb[L + j], fv, al);
      a2 = fmaf(go, z[(size_t)b * L + j], a2);
      ab += go;
    }
    pc[idx] = am;
    pc[FL + idx] = al;
    pc[2 * FL + idx] = a2;
    if (j == 0) pc[3 * FL + e] = ab;
  } else if (idx < F * L + L) {
    const int j = idx - F * L;
    float sm = 0.f, sl = 0.f;
    for (int b = b0; b < b1; ++b) {
      sm += gs[(size_t)b * G + j];
      sl += gs[(size_t)b * G + L + j];
    }
    pc[3 * FL + F + j] = sm;
    pc[3 * FL + F + L + j] = sl;
  }
}

__global__ __launch_bounds__(256) void heads_wgrad_reduce_kernel(
    const float* __restrict__ part, int nch, float* __restrict__ gwmu, float* __restrict__ gbmu,
    float* __restrict__ gwlv, float* __restrict__ gblv, float* __restrict__ gw2,
    float* __restrict__ gb2, int F, int L) {
  const size_t FL = (size_t)F * L;
  const size_t per = 3 * FL + F + 2 * L;
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= per) return;
  float s = 0.f;
  for (int c = 0; c < nch; ++c) s += part[(size_t)c * per + i];
  if (i < FL) {
    gwmu[i] = s;
  } else if (i < 2 * FL) {
    gwlv[i - FL] = s;
  } else if (i < 3 * FL) {
    const size_t r = i - 2 * FL;           // [j][e] -> W2 grad layout [e][j]
    const size_t j = r / F, e = r - j * F;
    gw2[e * L + j] = s;
  } else if (i < 3 * FL + F) {
    gb2[i - 3 * FL] = s;
  } else if (i < 3 * FL + F + L) {
    gbmu[i - 3 * FL - F] = s;
  } else {
    gblv[i - 3 * FL - F - L] = s;
  }
}

// ------------------------------------------------------------------ generic Linear
__global__ void linear_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                  const float* __restrict__ b, float* __restrict__ y, int M, int K,
                                  int N) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= M * N) return;
  const int m = e / N, n = e - m * N;
  float s = b ? b[n] : 0.f;
  for (int k = 0; k < K; ++k) s = fmaf(x[(size_t)m * K + k], w[(size_t)n * K + k], s);
  y[e] = s;
}

__global__ void linear_bwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                  const float* __restrict__ gy, float* __restrict__ gx,
                                  float* __restrict__ gw, float* __restrict__ gb, int M, int K,
                                  int N) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int nx = gx ? M * K : 0, nw = gw ? N * K : 0, nb = gb ? N : 0;
  if (e < nx) {
    const int m = e / K, k = e - m * K;
    float s = 0.f;
    for (int n = 0; n < N; ++n) s = fmaf(gy[(size_t)m * N + n], w[(size_t)n * K + k], s);
    gx[e] = s;
  } else if (e < nx + nw) {
    const int i = e - nx, n = i / K, k = i - n * K;
    float s = 0.f;
    for (int m = 0; m < M; ++m) s = fmaf(gy[(size_t)m * N + n], x[(size_t)m * K + k], s);
    gw[i] = s;
  } else if (e < nx + nw + nb) {
    const int n = e - nx - nw;
    float s = 0.f;
    for (int m = 0; m < M; ++m) s += gy[(size_t)m * N + n];
    gb[n] = s;
  }
}

__global__ void reparam_fwd_kernel(const float* __restrict__ mu, const float* __restrict__ lv,
                                   const float* __restrict__ eps, float* __restrict__ z,
                                   float* __restrict__ sd, int64_t n) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float s = expf(lv[i] * 0.5f);
  if (sd) sd[i] = s;
  z[i] = fmaf(eps[i], s, mu[i]);
}

__global__ void reparam_bwd_kernel(const float* __restrict__ gz, const float* __restrict__ gsd,
                                   const float* __restrict__ eps, const float* __restrict__ sd,
                                   float* __restrict__ gmu, float* __restrict__ glv, int64_t n) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float g = gz ? gz[i] : 0.f;
  if (gmu) gmu[i] = g;
  if (glv) glv[i] = ((gsd ? gsd[i] : 0.f) + g * eps[i]) * sd[i] * 0.5f;
}

// ------------------------------------------------------------------ Philox4x32-10 normal
EV_DEVINL void philox_round(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3, uint32_t k0,
                            uint32_t k1) {
  const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
  const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
  const uint32_t h0 = (uint32_t)(p0 >> 32), l0 = (uint32_t)p0;
  const uint32_t h1 = (uint32_t)(p1 >> 32), l1 = (uint32_t)p1;
  const uint32_t n0 = h1 ^ c1 ^ k0, n2 = h0 ^ c3 ^ k1;
  c0 = n0; c1 = l1; c2 = n2; c3 = l0;
}

__global__ void normal_tick_kernel(uint64_t* counter) { *counter += 1; }

__global__ void normal_fill_kernel(float* __restrict__ out, int64_t n, uint64_t seed,
                                   uint64_t offset, const uint64_t* __restrict__ counter) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;  // 4 normals per thread
  if (i * 4 >= n) return;
  const uint64_t base = counter ? offset + *counter * (uint64_t)((n + 3) / 4) : offset;
  const uint64_t ctr = base + (uint64_t)i;
  uint32_t c0 = (uint32_t)ctr, c1 = (uint32_t)(ctr >> 32), c2 = 0, c3 = 0;
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    philox_round(c0, c1, c2, c3, k0, k1);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  const float inv = 2.3283064365386963e-10f;  // 2^-32
  const float u0 = ((float)c0 + 0.5f) * inv, u1 = ((float)c1 + 0.5f) * inv;
  const float u2 = ((float)c2 + 0.5f) * inv, u3 = ((float)c3 + 0.5f) * inv;
  const float r0 = sqrtf(-2.f * logf(u0)), r1 = sqrtf(-2.f * logf(u2));
  const float tp = 6.283185307179586f;
  float v[4];
  v[0] = r0 * cosf(tp * u1);
  v[1] = r0 * sinf(tp * u1);
  v[2] = r1 * cosf(tp * u3);
  v[3] = r1 * sinf(tp * u3);
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (i * 4 + k < n) out[i * 4 + k] = v[k];
}

}  // namespace ev

using namespace ev;

// ------------------------------------------------------------------ host side
namespace {

// pattern tile of a per-pixel launch with n lanes per pattern: R = BT * n / 256 in {1,2,4,8},
// as few blocks as still gives >= 256 of them (SS pixels x ceil(B / BT) tiles)
int heads_tile(int B, int SS, int n) {
  int bt = 2048 / n;
  while (bt > 256 / n && (long)SS * ((B + bt - 1) / bt) < 256) bt /= 2;
  return bt;
}

template <typename K>
void heads_lds_attr(K kernel, size_t lds) {
  if (lds > 64 * 1024)
    (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
}

// feature chunks of the partial pass: CC channels (a power of two dividing C) x all SS pixels,
// about 128 features each; KS = C / CC chunks
int heads_cc(int C, int SS) {
  int cc = 1;
  while (cc * 2 * SS <= 128 && cc * 2 <= C) cc *= 2;
  return cc;
}
int heads_ks(int C, int SS) { return C / heads_cc(C, SS); }

template <int MODE>
int launch_partial(const float* A, const float* w0, const float* w1, float* part, float* copy,
                   int cstride, int coff, int B, int C, int SS, int L, int N, hipStream_t st) {
  const int NP = heads_np(N);
  const int CC = heads_cc(C, SS), KS = C / CC, KC = CC * SS;
  const int bt = heads_tile(B, KS, NP);
  const int R = bt * NP / HT;
  const size_t lds = ((size_t)KC * (NP + 1) + (size_t)bt * (KC + 1)) * sizeof(float);
  EV_REQUIRE(lds <= 160 * 1024, "heads: feature chunk of %d too large", KC);
  const dim3 grid(KS, (B + bt - 1) / bt);
#define EV_HP(RR)                                                                              \
  case RR:                                                                                     \
    heads_lds_attr(heads_dot_partial_kernel<MODE, RR>, lds);                                   \
    hipLaunchKernelGGL((heads_dot_partial_kernel<MODE, RR>), grid, dim3(HT), lds, st, A, w0, w1, \
                       part, copy, cstride, coff, B, C, SS, CC, L, N, NP, bt);                 \
    break;
  switch (R) {
    EV_HP(1) EV_HP(2) EV_HP(4) EV_HP(8)
    default: EV_REQUIRE(false, "heads: tile %d x %d", bt, NP);
  }
#undef EV_HP
  return 0;
}

template <int MODE>
int launch_expand(const float* V, int vstride, const float* m0, const float* m1, const float* bias,
                  float* out, int B, int C, int SS, int L, int J, hipStream_t st) {
  const int bt = heads_tile(B, SS, C);
  const int R = bt * C / HT;
  const size_t lds = ((size_t)J * C + (size_t)bt * J) * sizeof(float);
  EV_REQUIRE(lds <= 160 * 1024, "heads: expand tile too large");
  const dim3 grid(SS, (B + bt - 1) / bt);
#define EV_HE(RR)                                                                              \
  case RR:                                                                                     \
    heads_lds_attr(heads_expand_kernel<MODE, RR>, lds);                                        \
    hipLaunchKernelGGL((heads_expand_kernel<MODE, RR>), grid, dim3(HT), lds, st, V, vstride, m0, \
                       m1, bias, out, B, C, SS, L, J, bt);                                     \
    break;
  switch (R) {
    EV_HE(1) EV_HE(2) EV_HE(4) EV_HE(8)
    default: EV_REQUIRE(false, "heads: expand tile %d x %d", bt, C);
  }
#undef EV_HE
  return 0;
}

bool heads_shape_ok(int B, int C, int S, int L) {
  return B > 0 && L > 0 && L <= MAXL && S > 0 && S <= 1024 && C >= 16 && C <= 256 &&
         (C & (C - 1)) == 0;
}

}  // namespace

extern "C" size_t ebsdvae_heads_work(int B, int C, int S, int L) {
  if (!heads_shape_ok(B, C, S, L)) return 0;
  return (size_t)heads_ks(C, S * S) * B * heads_np(2 * L) * sizeof(float);
}

extern "C" int ebsdvae_heads_fwd(const float* enc, const float* w_mu, const float* b_mu,
                                 const float* w_lv, const float* b_lv, const float* w_l2,
                                 const float* b_l2, const float* eps, float* flat, float* mu,
                                 float* std, float* z, float* dec_in, void* work, int B, int C,
                                 int S, int L, ebsdvae_stream_t stream) {
  EV_REQUIRE(enc && w_mu && b_mu && w_lv && b_lv && w_l2 && b_l2 && eps && flat && mu && std && z &&
                 dec_in && work,
             "heads_fwd: null pointer");
  EV_REQUIRE(heads_shape_ok(B, C, S, L), "heads_fwd: bad shape B=%d C=%d S=%d L=%d", B, C, S, L);
  hipStream_t st = (hipStream_t)stream;
  const int SS = S * S, F = C * SS;
  float* part = (float*)work;
  if (launch_partial<0>(enc, w_mu, w_lv, part, flat, F, 0, B, C, SS, L, 2 * L, st)) return 1;
  hipLaunchKernelGGL(heads_fwd_finalize_kernel<false>, dim3((B * L + HT - 1) / HT), dim3(HT), 0, st,
                     part, b_mu, b_lv, eps, mu, std, z, B, heads_ks(C, SS), L, heads_np(2 * L));
  if (launch_expand<0>(z, L, w_l2, nullptr, b_l2, dec_in, B, C, SS, L, L, st)) return 1;
  return evh::check_launch("heads_fwd");
}

extern "C" int ebsdvae_latent_mu(const float* enc, const float* w_mu, const float* b_mu, float* mu,
                                 void* work, int B, int C, int S, int L, ebsdvae_stream_t stream) {
  EV_REQUIRE(enc && w_mu && b_mu && mu && work, "latent_mu: null pointer");
  EV_REQUIRE(heads_shape_ok(B, C, S, L), "latent_mu: bad shape B=%d C=%d S=%d L=%d", B, C, S, L);
  hipStream_t st = (hipStream_t)stream;
  const int SS = S * S;
  float* part = (float*)work;
  if (launch_partial<0>(enc, w_mu, nullptr, part, nullptr, 0, 0, B, C, SS, L, L, st)) return 1;
  hipLaunchKernelGGL(heads_fwd_finalize_kernel<true>, dim3((B * L + HT - 1) / HT), dim3(HT), 0, st,
                     part, b_mu, nullptr, nullptr, mu, nullptr, nullptr, B, heads_ks(C, SS), L,
                     heads_np(L));
  return evh::check_launch("latent_mu");
}

extern "C" int ebsdvae_heads_bwd(const float* g_dec, const float* g_z, const float* g_mu,
                                 const float* g_std, const float* std, const float* eps,
                                 const float* w_mu, const float* w_lv, const float* w_l2,
                                 float* g_enc, float* gs, void* work, int B, int C, int S, int L,
                                 ebsdvae_stream_t stream) {
  EV_REQUIRE(g_dec && std && eps && w_mu && w_lv && w_l2 && g_enc && gs && work,
             "heads_bwd: null pointer");
  EV_REQUIRE(heads_shape_ok(B, C, S, L), "heads_bwd: bad shape B=%d C=%d S=%d L=%d", B, C, S, L);
  hipStream_t st = (hipStream_t)stream;
  const int SS = S * S, F = C * SS, G = 2 * L + F;
  float* part = (float*)work;
  // g_z partials (linear2 adjoint); g_out copied into gs in NCHW order for heads_wgrad
  if (launch_partial<1>(g_dec, w_l2, nullptr, part, gs, G, 2 * L, B, C, SS, L, L, st)) return 1;
  hipLaunchKernelGGL(heads_bwd_finalize_kernel, dim3((B * L + HT - 1) / HT), dim3(HT), 0, st, part,
                     g_z, g_mu, g_std, std, eps, gs, B, heads_ks(C, SS), L, heads_np(L), G);
  if (launch_expand<1>(gs, G, w_mu, w_lv, nullptr, g_enc, B, C, SS, L, 2 * L, st)) return 1;
  return evh::check_launch("heads_bwd");
}

extern "C" size_t ebsdvae_heads_wgrad_work(int B, int F, int L) {
  const size_t per = 3 * (size_t)F * L + F + 2 * (size_t)L;
  return (size_t)((B + HB - 1) / HB) * per * sizeof(float);
}

extern "C" int ebsdvae_heads_wgrad(const float* flat, const float* z, const float* gs, float* gw_mu,
                                   float* gb_mu, float* gw_lv, float* gb_lv, float* gw_l2,
                                   float* gb_l2, void* work, int B, int F, int L,
                                   ebsdvae_stream_t stream) {
  EV_REQUIRE(flat && z && gs && gw_mu && gb_mu && gw_lv && gb_lv && gw_l2 && gb_l2 && work,
             "heads_wgrad: null pointer");
  EV_REQUIRE(B > 0 && L > 0 && L <= MAXL, "heads_wgrad: bad L");
  const int n = F * L + L;
  const int nch = (B + HB - 1) / HB;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(heads_wgrad_kernel, dim3((n + 255) / 256, nch), dim3(256), 0, s, flat, z, gs,
                     (float*)work, B, F, L);
  const size_t per = 3 * (size_t)F * L + F + 2 * (size_t)L;
  hipLaunchKernelGGL(heads_wgrad_reduce_kernel, dim3((unsigned)((per + 255) / 256)), dim3(256), 0, s,
                     (const float*)work, nch, gw_mu, gb_mu, gw_lv, gb_lv, gw_l2, gb_l2, F, L);
  return evh::check_launch("heads_wgrad");
}

extern "C" int ebsdvae_linear_fwd(const float* x, const float* w, const float* b, float* y, int M,
                                  int K, int N, ebsdvae_stream_t stream) {
  EV_REQUIRE(x && w && y && M > 0 && K > 0 && N > 0, "linear_fwd: bad args");
  const int n = M * N;
  hipLaunchKernelGGL(linear_fwd_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, x, w,
                     b, y, M, K, N);
  return evh::check_launch("linear_fwd");
}

extern "C" int ebsdvae_linear_bwd(const float* x, const float* w, const float* gy, float* gx,
                                  float* gw, float* gb, int M, int K, int N,
                                  ebsdvae_stream_t stream) {
  EV_REQUIRE(x && w && gy && M > 0 && K > 0 && N > 0, "linear_bwd: bad args");
  const int n = (gx ? M * K : 0) + (gw ? N * K : 0) + (gb ? N : 0);
  if (n == 0) return 0;
  hipLaunchKernelGGL(linear_bwd_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, x, w,
                     gy, gx, gw, gb, M, K, N);
  return evh::check_launch("linear_bwd");
}

extern "C" int ebsdvae_reparam_fwd(const float* mu, const float* logvar, const float* eps, float* z,
                                   float* std, int64_t n, ebsdvae_stream_t stream) {
  EV_REQUIRE(mu && logvar && eps && z && n >= 0, "reparam_fwd: bad args");
  if (n == 0) return 0;
  hipLaunchKernelGGL(reparam_fwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, mu, logvar, eps, z, std, n);
  return evh::check_launch("reparam_fwd");
}

extern "C" int ebsdvae_reparam_bwd(const float* gz, const float* gstd, const float* eps,
                                   const float* std, float* gmu, float* glogvar, int64_t n,
                                   ebsdvae_stream_t stream) {
  EV_REQUIRE(eps && std && n >= 0, "reparam_bwd: bad args");
  if (n == 0) return 0;
  hipLaunchKernelGGL(reparam_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, gz, gstd, eps, std, gmu, glogvar, n);
  return evh::check_launch("reparam_bwd");
}

extern "C" int ebsdvae_normal_fill(float* out, int64_t n, uint64_t seed, uint64_t offset,
                                   uint64_t* counter, ebsdvae_stream_t stream) {
  EV_REQUIRE(out && n >= 0, "normal_fill: bad args");
  if (n == 0) return 0;
  const int64_t threads = (n + 3) / 4;
  if (counter) hipLaunchKernelGGL(normal_tick_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, counter);
  hipLaunchKernelGGL(normal_fill_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, out, n, seed, offset, counter);
  return evh::check_launch("normal_fill");
}
