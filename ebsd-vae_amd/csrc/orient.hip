// Batched orientation consensus: the reference's per-query
// `find_best_orientation` (latice/index/faiss_db.py:258-372, identical in chroma_db.py:261-375)
// for many queries in one launch, one wave per query, one lane per candidate.  Float64
// throughout, restating scipy 1.15 `Rotation` (the reference's dependency) arithmetic:
//
//   from_euler("zxz", deg)  extrinsic: q = q_z(c) (x) q_x(b) (x) q_z(a), scalar-last quats
//   p * q                   Hamilton product p (x) q (q applied first)
//   inv()                   conjugate;   magnitude() = 2 atan2(|v|, |w|)
//   mean()                  the eigenvector of the largest eigenvalue of sum q q^T
//   as_euler("zxz", deg)    Bernardes & Viollet (2022), scipy's algorithm incl. its
//                           gimbal-lock branches (third angle 0) and the wrap to [-180, 180]
//
// Per query (candidates = the orientations of its top-n cosine matches, in match order):
//   for it < min(max_iter, n): ref = cand[it]; similar = {j : angle(ref^-1 cand_j) < thr}
//     if |similar| >= min_matches: each similar candidate is replaced by the one of its 24
//       cubic-symmetry equivalents QUAT_SYM_i (x) cand_j closest to ref (first minimum,
//       faiss_db.py:374-398); mean of those -> Euler; success; stop.
//   best = mean on success, else cand[0]; similar = the last iteration's set (a bit mask).
// The symmetric equivalents are kept as quaternions; the reference round-trips them through
// Euler angles before the mean, which moves the result by ~1e-12 degrees.
#include "common.h"
#include "../../include/ebsdvae.h"

namespace ev {

struct Q4 {
  double x, y, z, w;   // scalar-last, as scipy
};

EV_DEVINL Q4 qmul(const Q4& p, const Q4& q) {
  // scipy _compose_quat: v = pw qv + qw pv + pv x qv ; w = pw qw - pv . qv
  Q4 r;
  r.x = p.w * q.x + q.w * p.x + (p.y * q.z - p.z * q.y);
  r.y = p.w * q.y + q.w * p.y + (p.z * q.x - p.x * q.z);
  r.z = p.w * q.z + q.w * p.z + (p.x * q.y - p.y * q.x);
  r.w = p.w * q.w - (p.x * q.x + p.y * q.y + p.z * q.z);
  return r;
}

EV_DEVINL Q4 qconj(const Q4& q) { return Q4{-q.x, -q.y, -q.z, q.w}; }

EV_DEVINL double qmag(const Q4& q) {
  return 2.0 * atan2(sqrt(q.x * q.x + q.y * q.y + q.z * q.z), fabs(q.w));
}

EV_DEVINL Q4 qnormalize(const Q4& q) {
  const double n = sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
  return Q4{q.x / n, q.y / n, q.z / n, q.w / n};
}

constexpr double kPi = 3.14159265358979323846;
constexpr double kDeg = kPi / 180.0;

// from_euler("zxz", [a, b, c], degrees=True), extrinsic
EV_DEVINL Q4 from_euler_zxz(double a, double b, double c) {
  a *= kDeg; b *= kDeg; c *= kDeg;
  const Q4 qa{0.0, 0.0, sin(a / 2), cos(a / 2)};
  const Q4 qb{sin(b / 2), 0.0, 0.0, cos(b / 2)};
  const Q4 qc{0.0, 0.0, sin(c / 2), cos(c / 2)};
  return qmul(qc, qmul(qb, qa));
}

// as_euler("zxz", degrees=True) of a unit quaternion (scipy's quaternion algorithm for a
// proper, extrinsic sequence: i = k = z, j = x, third axis y, even permutation sign;
// checked against scipy 1.15 in tests/test_index_oracle.py, gimbal-lock branches included)
EV_DEVINL void as_euler_zxz(const Q4& q, double out[3]) {
  // permuted elements for the symmetric sequence z-x-z: a = w, b = q[i=z], c = q[j=x],
  // d = q[k=y] * sign, sign = (i-j)(j-k)(k-i)/2 with (i, j, k) = (2, 0, 1) -> +1
  const double a = q.w, b = q.z, c = q.x, d = q.y;
  double ang[3];
  ang[1] = 2.0 * atan2(hypot(c, d), hypot(a, b));
  const double eps = 1e-7;
  int cs = 0;
  if (fabs(ang[1]) <= eps) cs = 1;
  else if (fabs(ang[1] - kPi) <= eps) cs = 2;
  const double half_sum = atan2(b, a), half_diff = atan2(d, c);
  if (cs == 0) {
    ang[0] = half_sum - half_diff;
    ang[2] = half_sum + half_diff;
  } else {
    ang[2] = 0.0;
    ang[0] = (cs == 1) ? 2.0 * half_sum : -2.0 * half_diff;   // extrinsic: 2 half_diff * -1
  }
  // (scipy swaps the first and third angles only for intrinsic sequences)
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    if (ang[i] < -kPi) ang[i] += 2.0 * kPi;
    else if (ang[i] > kPi) ang[i] -= 2.0 * kPi;
    out[i] = ang[i] / kDeg;
  }
}

// QUAT_SYM (latice/utils/constants.py:13-39), scalar-last, normalised at use as
// scipy's Rotation.from_quat does
__constant__ double kCubic[24][4] = {
    {1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1},
    {0.5, 0.5, 0.5, 0.5}, {0.5, -0.5, -0.5, -0.5}, {0.5, 0.5, -0.5, 0.5}, {0.5, -0.5, 0.5, -0.5},
    {0.5, -0.5, 0.5, 0.5}, {0.5, 0.5, -0.5, -0.5}, {0.5, -0.5, -0.5, 0.5}, {0.5, 0.5, 0.5, -0.5},
    {0.70710678118654746, 0.70710678118654746, 0, 0}, {0.70710678118654746, 0, 0.70710678118654746, 0},
    {0.70710678118654746, 0, 0, 0.70710678118654746}, {0.70710678118654746, -0.70710678118654746, 0, 0},
    {0.70710678118654746, 0, -0.70710678118654746, 0}, {0.70710678118654746, 0, 0, -0.70710678118654746},
    {0, 0.70710678118654746, 0.70710678118654746, 0}, {0, -0.70710678118654746, 0.70710678118654746, 0},
    {0, 0, 0.70710678118654746, 0.70710678118654746}, {0, 0, -0.70710678118654746, 0.70710678118654746},
    {0, 0.70710678118654746, 0, 0.70710678118654746}, {0, -0.70710678118654746, 0, 0.70710678118654746},
};

EV_DEVINL double wsum64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// largest-eigenvalue eigenvector of a symmetric 4x4 (cyclic Jacobi, float64)
EV_DEVINL Q4 top_eigvec(double A[4][4]) {
  double V[4][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}};
  for (int sweep = 0; sweep < 30; ++sweep) {
    double off = 0.0;
    for (int p = 0; p < 4; ++p)
      for (int r = p + 1; r < 4; ++r) off += A[p][r] * A[p][r];
    if (off < 1e-300) break;
    for (int p = 0; p < 3; ++p)
      for (int r = p + 1; r < 4; ++r) {
        if (fabs(A[p][r]) < 1e-300) continue;
        const double theta = (A[r][r] - A[p][p]) / (2.0 * A[p][r]);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
        for (int k = 0; k < 4; ++k) {   // A <- J^T A J
          const double akp = A[k][p], akr = A[k][r];
          A[k][p] = c * akp - s * akr;
          A[k][r] = s * akp + c * akr;
        }
        for (int k = 0; k < 4; ++k) {
          const double apk = A[p][k], ark = A[r][k];
          A[p][k] = c * apk - s * ark;
          A[r][k] = s * apk + c * ark;
        }
        for (int k = 0; k < 4; ++k) {
          const double vkp = V[k][p], vkr = V[k][r];
          V[k][p] = c * vkp - s * vkr;
          V[k][r] = s * vkp + c * vkr;
        }
      }
  }
  int best = 0;
  for (int k = 1; k < 4; ++k)
    if (A[k][k] > A[best][best]) best = k;
  return qnormalize(Q4{V[0][best], V[1][best], V[2][best], V[3][best]});
}

__global__ __launch_bounds__(64) void orient_consensus_kernel(
    const double* __restrict__ ori, const long long* __restrict__ idx, int n, double thr_deg,
    int min_matches, int max_iter, double* __restrict__ best, double* __restrict__ mean,
    int* __restrict__ success, unsigned long long* __restrict__ similar) {
  const int q = blockIdx.x, lane = threadIdx.x;
  const bool live = lane < n;
  long long row = live ? idx[(size_t)q * n + lane] : -1;
  if (row < 0) row = 0;
  const double* e = ori + row * 3;
  const Q4 cq = live ? from_euler_zxz(e[0], e[1], e[2]) : Q4{0, 0, 0, 1};
  const int iters = min(max_iter, n);
  unsigned long long mask = 0;
  int ok = 0;
  double mean_e[3] = {NAN, NAN, NAN};
  for (int it = 0; it < iters; ++it) {
    const Q4 ref{__shfl(cq.x, it, 64), __shfl(cq.y, it, 64), __shfl(cq.z, it, 64), __shfl(cq.w, it, 64)};
    const Q4 rinv = qconj(ref);
    const double ang = qmag(qmul(rinv, cq)) / kDeg;
    mask = __ballot(live && ang < thr_deg);
    if (__popcll(mask) >= min_matches) {
      const bool mine = (mask >> lane) & 1ull;
      Q4 s{0, 0, 0, 1};
      if (mine) {   // closest cubic-symmetry equivalent to ref (first minimum)
        double bm = 1e300;
        for (int k = 0; k < 24; ++k) {
          const Q4 sym = qnormalize(Q4{kCubic[k][0], kCubic[k][1], kCubic[k][2], kCubic[k][3]});
          const Q4 eq = qmul(sym, cq);
          const double m = qmag(qmul(rinv, eq));
          if (m < bm) { bm = m; s = eq; }
        }
      }
      // mean: K = sum q q^T over the similar set (scipy Rotation.mean, unit weights)
      const double f = mine ? 1.0 : 0.0;
      const double qv[4] = {s.x, s.y, s.z, s.w};
      double K[4][4];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = a; b < 4; ++b) {
          K[a][b] = wsum64(f * qv[a] * qv[b]);
          K[b][a] = K[a][b];
        }
      const Q4 m = top_eigvec(K);
      as_euler_zxz(m, mean_e);
      ok = 1;
      break;
    }
  }
  if (lane == 0) {
    success[q] = ok;
    similar[q] = mask;
    double b[3];
    if (ok) {
      b[0] = mean_e[0]; b[1] = mean_e[1]; b[2] = mean_e[2];
    } else {
      b[0] = e[0]; b[1] = e[1]; b[2] = e[2];   // the closest match (candidate 0)
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      best[(size_t)q * 3 + i] = b[i];
      mean[(size_t)q * 3 + i] = mean_e[i];
    }
  }
}

}  // namespace ev

using namespace ev;

extern "C" int ebsdvae_orient_consensus(const double* orientations, const long long* cand_idx,
                                        int Q, int n, double threshold_deg, int min_matches,
                                        int max_iterations, double* best, double* mean,
                                        int* success, unsigned long long* similar_mask,
                                        ebsdvae_stream_t stream) {
  EV_REQUIRE(orientations && cand_idx && best && mean && success && similar_mask,
             "orient_consensus: null pointer");
  EV_REQUIRE(Q >= 0 && n >= 1 && n <= 64, "orient_consensus: n=%d (1..64)", n);
  if (Q == 0) return 0;
  hipLaunchKernelGGL(orient_consensus_kernel, dim3(Q), dim3(64), 0, (hipStream_t)stream, orientations,
                     cand_idx, n, threshold_deg, min_matches, max_iterations, best, mean, success,
                     similar_mask);
  return evh::check_launch("orient_consensus");
}
