// libzkfl: MI355X-native Groth16 prover (BN254) behind the C ABI in include/zkfl.h.
//
// Replaces `snarkjs groth16 prove` [ext] as invoked by the reference harness
// (tests/full_system_simulation.mjs:773-776).  Algorithm per proof (snarkjs groth16_prove,
// restated in oracle/groth16.py::prove):
//   1. buildABC1: a = A.w, b = B.w over the domain rows (zkey section 4 coefficients),
//      c = a o b                                           -> k_abc (CSR rows, Montgomery)
//   2. a,b,c: ifft -> * inc^i -> fft  (odd coset)          -> ntt_coset_shift (3 vectors)
//   3. joinABC: h = a*b - c, from Montgomery               -> k_join
//   4. multiExpAffine A(w), B1(w), B2(w), C(w_priv), H(h)  -> msm_run (G1 x4, G2 x1)
//   5. pi_a = A + alpha1 + r delta1, pi_b = B2 + beta2 + s delta2,
//      pi_c = C + H + s pi_a + r (B1 + beta1 + s delta1) - r s delta1
//      The constant terms are folded into the MSMs as extra bases (alpha1/delta1 on A,
//      beta1/delta1 on B1, beta2/delta2 on B2, delta1 with scalar -rs on C); only
//      s*pi_a + r*B1 remains for k_assemble (GLV halves, windowed, one wave each), then affine.
// Everything from the device-resident witness to the 256-byte proof runs on the GPU; the host
// only parses files, uploads, and launches.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/random.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "curve.h"
#include "glv.h"
#include "host_parse.h"
#include "field.h"
#include "field29.h"
#include "merkle.h"
#include "msm_api.h"
#include "ntt.h"
#include "pairing.h"
#include "row29.h"
#include "prof.h"
#include "setup.h"
#include "verify.h"
#include "witness.h"
#include "wtrace.h"
#include "zkfl.h"

using namespace zkfl;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

int hip_fail(hipError_t e, const char* where) {
  g_err = std::string(where) + ": " + hipGetErrorString(e);
  return e == hipErrorOutOfMemory ? ZKFL_E_OOM : ZKFL_E_DEVICE;
}

#define HIP_TRY(x, where)                      \
  do {                                         \
    hipError_t _e = (x);                       \
    if (_e != hipSuccess) return hip_fail(_e, where); \
  } while (0)

const uint32_t R_LIMBS[8] = {0xf0000001u, 0x43e1f593u, 0x79b97091u, 0x2833e848u,
                             0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
const uint32_t Q_LIMBS[8] = {0xd87cfd47u, 0x3c208c16u, 0x6871ca8du, 0x97816a91u,
                             0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};

bool lt_r(const uint32_t* v) {  // v < r
  for (int i = 7; i >= 0; i--) {
    if (v[i] != R_LIMBS[i]) return v[i] < R_LIMBS[i];
  }
  return false;
}

bool lt_q(const uint32_t* v) {  // v < q (base field)
  for (int i = 7; i >= 0; i--) {
    if (v[i] != Q_LIMBS[i]) return v[i] < Q_LIMBS[i];
  }
  return false;
}

int parse_wtns(const uint8_t* buf, size_t len, WtnsView& out) {
  std::string err;
  int rc = wtns_parse(buf, len, out, err);  // csrc/host_parse.cc
  return rc ? fail(rc, err) : ZKFL_OK;
}

// ---------------------------------------------------------------------------
// Kernels
// ---------------------------------------------------------------------------
// ABC as a segmented sum over the flat term array (A rows then B rows; rp[0..2n] row pointers).
// coef raw = coef * R^2 mod r (snarkjs zkey section 4), w std form, so
// mont_mul(coef_raw, w) = coef * w * R = Montgomery form of coef*w.  Rows range from 1 to ~130
// terms (Poseidon S-box inputs carry ~61-term combinations), so one lane per row leaves ~2/3 of
// the lanes idle; instead lane c takes the ABC_L terms [c*L, c*L+L), emitting the sum of its
// first row segment to head[c], of its last to tail[c], and rows wholly inside the chunk
// straight to abc[row]; k_abc_rows stitches rows j and n+j and forms c = a*b.
constexpr uint32_t ABC_L = 16;

// Terms are either packed (col | coefficient-dictionary index << cshift in one u32: circuits
// with few distinct coefficients, e.g. 1,971 among the 7.0 M A/B terms of the training circuit;
// 4 B per term instead of 36 B, the dictionary stays in cache) or wide (cols[] + coefs[]).
struct AbcTerms {
  const uint32_t* cols;  // packed terms, or column indices (wide)
  const Fr* coefs;       // dictionary (packed) or one coefficient per term (wide)
  uint32_t cshift;       // 0: wide
};

template <bool PACKED>
__global__ void __launch_bounds__(64) k_abc_chunks(const uint32_t* __restrict__ rp, uint32_t nrows, AbcTerms T,
                                                   const Fr* __restrict__ w, uint32_t K, Fr* __restrict__ head,
                                                   Fr* __restrict__ tail, Fr* __restrict__ abc) {
  ZK_WT(WT_ABC);
  ZK_LIGHT();
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t p0 = c * ABC_L;
  if (p0 >= K) return;
  const uint32_t p1 = p0 + ABC_L < K ? p0 + ABC_L : K;
  const uint32_t* __restrict__ cols = T.cols;
  const Fr* __restrict__ coefs = T.coefs;
  const uint32_t cmask = PACKED ? (1u << T.cshift) - 1u : 0xFFFFFFFFu;
  auto coef_of = [&](uint32_t t, uint32_t p) { return PACKED ? coefs[t >> T.cshift] : coefs[p]; };
  // row containing p0: largest r with rp[r] <= p0 (empty rows share their start with the next)
  auto row_of = [&](uint32_t p, uint32_t lo) {
    uint32_t hi = nrows - 1;
    while (lo < hi) {
      const uint32_t mid = (lo + hi + 1) >> 1;
      if (rp[mid] <= p) lo = mid;
      else hi = mid - 1;
    }
    return lo;
  };
  uint32_t r = row_of(p0, 0), rend = rp[r + 1];
  Fr acc = fp_zero<FrP>();
  bool first = true;
  // software-pipelined: term p+1's witness gather (and p+2's term word) are in flight while
  // term p is multiplied
  uint32_t t1 = (p0 + 1 < p1) ? cols[p0 + 1] : 0u;
  const uint32_t t0 = cols[p0];
  Fr wv = w[t0 & cmask], cf = coef_of(t0, p0);
  for (uint32_t p = p0; p < p1; p++) {
    Fr wn, cn;
    uint32_t t2 = 0;
    if (p + 1 < p1) {
      wn = w[t1 & cmask];
      cn = coef_of(t1, p + 1);
    }
    if (p + 2 < p1) t2 = cols[p + 2];
    if (p == rend) {  // row boundary inside the chunk
      if (first) head[c] = acc;
      else abc[r] = acc;
      first = false;
      acc = fp_zero<FrP>();
      // next non-empty row: usually r + 1; a run of empty rows (the domain padding after the
      // last constraint: ~241 K rows at 2^19) is skipped by binary search, not walked row by row
      r++;
      rend = rp[r + 1];
      if (rend == p) {
        r = row_of(p, r);
        rend = rp[r + 1];
      }
    }
    acc = fp_add(acc, fp_mul(cf, wv));
    wv = wn;
    cf = cn;
    t1 = t2;
  }
  if (first) head[c] = acc;
  else tail[c] = acc;
}

__device__ __forceinline__ Fr abc_row(const uint32_t* __restrict__ rp, uint32_t r, uint32_t K,
                                      const Fr* __restrict__ head, const Fr* __restrict__ tail,
                                      const Fr* __restrict__ abc) {
  const uint32_t s = rp[r], e = rp[r + 1];
  if (s == e) return fp_zero<FrP>();
  const uint32_t c0 = s / ABC_L, c1 = (e - 1) / ABC_L;
  const bool starts = (s == c0 * ABC_L);
  if (c0 == c1) {
    const uint32_t cend = (c0 + 1) * ABC_L < K ? (c0 + 1) * ABC_L : K;
    if (starts) return head[c0];
    if (e == cend) return tail[c0];
    return abc[r];  // wholly inside the chunk: written by k_abc_chunks
  }
  Fr acc = starts ? head[c0] : tail[c0];
  for (uint32_t c = c0 + 1; c <= c1; c++) acc = fp_add(acc, head[c]);
  return acc;
}

__global__ void __launch_bounds__(256) k_abc_rows(const uint32_t* __restrict__ rp, size_t n, uint32_t K,
                                                  const Fr* __restrict__ head, const Fr* __restrict__ tail,
                                                  Fr* __restrict__ abc) {
  ZK_WT(WT_ABC_ROWS);
  ZK_LIGHT();
  const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const Fr a = abc_row(rp, (uint32_t)j, K, head, tail, abc);
  const Fr b = abc_row(rp, (uint32_t)(n + j), K, head, tail, abc);
  abc[j] = a;
  abc[n + j] = b;
  abc[2 * n + j] = fp_mul(a, b);
}

// h = a*b - c (coset evaluations), to standard form for the H MSM.
__global__ void k_join(const Fr* __restrict__ abc, size_t n, Fr* __restrict__ h) {
  ZK_WT(WT_JOIN);
  ZK_LIGHT();
  size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
#if ZK_KNOCKOUT & 4
  // NTT knock-out (timing only): a*b - c vanishes on the domain, so without the coset shift h would
  // be zero and the H MSM would lose its digits too; a*b + c keeps h a full-size scalar vector
  Fr v = fp_add(fp_mul(abc[j], abc[n + j]), abc[2 * n + j]);
#else
  Fr v = fp_sub(fp_mul(abc[j], abc[n + j]), abc[2 * n + j]);
#endif
  h[j] = fp_from_mont(v);
}

// Blinding scalar slots referenced by the compacted bases' index maps (std form):
// extra = [1, r, s, -r*s].  plain -> all zero (parity hook: pure MSMs).
// The tails a proof chain empties at its start (k_proof_start): up to 4 G1 and 1 G2, each as
// its bucket array (16-B vectors), nnz counter and liveness flags.
struct ProofStart {
  uint4* buckets[5];
  uint32_t nvec[5];
  uint32_t* nnz[5];
  uint32_t* live[5];
  int n;
  // graph replay: the proof's witness, copied into the slot's stage (w_dst, w_nvec 16-B vectors)
  // from the device address the host left in the pinned buffer (w_src_host); w_dst null: none
  const uint64_t* w_src_host;
  uint4* w_dst;
  uint32_t w_nvec;
};

// A proof chain's first kernel, one launch for what were up to four: the augmentation scalars
// (1, r, s, -rs) of the merged MSMs, res[3] = infinity (the merged C + H leaves the H slot
// empty), and the proof's MSM tails emptied (buckets, nnz, liveness: blockIdx.y = tail).
// rs_host: the slot's pinned r | s | GLV halves (host memory, coherent), copied to d_rs for the
// assembly; the augmentation scalars are computed from the host copy directly.
constexpr int RS_WORDS = (64 + 4 * (int)sizeof(GlvScalar)) / 4;
__global__ void __launch_bounds__(256) k_proof_start(const uint32_t* __restrict__ rs_host, uint32_t* __restrict__ d_rs,
                                                     Fr* __restrict__ extra, int plain, uint32_t* __restrict__ res3,
                                                     const ProofStart ps) {
  ZK_WT(WT_SET_EXTRA);
  ZK_LIGHT();
  const int y = blockIdx.y;
  if (ps.w_dst) {  // uniform per launch
    __shared__ const uint4* src;
    if (threadIdx.x == 0) src = reinterpret_cast<const uint4*>(*ps.w_src_host);
    __syncthreads();
    const size_t nb = (size_t)gridDim.x * gridDim.y * blockDim.x;
    for (size_t i = ((size_t)y * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x; i < ps.w_nvec; i += nb)
      ps.w_dst[i] = src[i];
  }
  if (y == 0 && blockIdx.x == 2 && threadIdx.x < RS_WORDS) d_rs[threadIdx.x] = rs_host[threadIdx.x];
  if (y == 0 && blockIdx.x == 0 && threadIdx.x == 0) {
    const Fr* rs = reinterpret_cast<const Fr*>(rs_host);
    Fr one = fp_zero<FrP>();
    one.v[0] = plain ? 0u : 1u;
    Fr r = plain ? fp_zero<FrP>() : rs[0];
    Fr s = plain ? fp_zero<FrP>() : rs[1];
    extra[0] = one;
    extra[1] = r;
    extra[2] = s;
    extra[3] = fp_from_mont(fp_neg(fp_mul(fp_to_mont(r), fp_to_mont(s))));
  }
  if (y == 0 && blockIdx.x == 1 && res3 && threadIdx.x < sizeof(G1P) / 4) res3[threadIdx.x] = 0u;  // ZZ = 0
  if (y >= ps.n) return;
  uint4* b = ps.buckets[y];
  const size_t nv = ps.nvec[y];
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (size_t)gridDim.x * blockDim.x)
    b[i] = make_uint4(0, 0, 0, 0);
  if (blockIdx.x == 0 && threadIdx.x == 0) *ps.nnz[y] = 0;
  if (blockIdx.x == 0 && threadIdx.x < MSM_LIVE_LEVELS) ps.live[y][threadIdx.x] = 0;
}

template <class F>
__device__ void store_affine_std(const Affine<F>& a, uint32_t* out);

template <>
__device__ void store_affine_std<FqOps>(const Affine<FqOps>& a, uint32_t* out) {
  Fq x = fp_from_mont(a.x), y = fp_from_mont(a.y);
  for (int i = 0; i < 8; i++) {
    out[i] = x.v[i];
    out[8 + i] = y.v[i];
  }
}

template <>
__device__ void store_affine_std<Fq2Ops>(const Affine<Fq2Ops>& a, uint32_t* out) {
  Fq2 x = f2_from_mont(a.x), y = f2_from_mont(a.y);
  for (int i = 0; i < 8; i++) {
    out[i] = x.c0.v[i];
    out[8 + i] = x.c1.v[i];
    out[16 + i] = y.c0.v[i];
    out[24 + i] = y.c1.v[i];
  }
}

// ---------------------------------------------------------------------------
// Quad-cooperative G1 point operations (k_assemble): four lanes evaluate one XYZZ doubling or
// addition together.  The products of each dependency level are spread over the quad (lane q
// computes product q) and broadcast by DPP quad_perm moves; every lane keeps the whole point, so all
// control flow stays uniform inside a quad.  A chain of point operations then costs one
// multiply latency per level (doubling 3, addition 4) instead of one per product (9 / 14).
// ---------------------------------------------------------------------------
// The quad operations are written once over a field policy QF (T, mul, add, sub<K>, dbl,
// is_zero<K>, zero, one, bcast<K>, pick4).  k_assemble runs them on Q29: the 29-bit engine's
// limbs and Montgomery domain (field29.h), a product one f29_mul (81 + 81 v_mad_u64_u32, two
// column chains: ~2.5x shorter single-lane latency than the 32-bit fp_mul).  Values are LAZY
// (normalized limbs, below a small multiple of p, tracked per site in the formulas' comments):
//   mul(a, b) < p + a b / 2^261 < 2p whenever a b < 169 p^2 (2^261 ~ 169.3 p);
//   add(a, b) < bound(a) + bound(b);  sub<K>(a, b) = a + K p - b for b < K p, < bound(a) + K p;
//   is_zero<K>(a) for a < K p (a == 0, p, .., (K-1) p).
// A quad operation keeps X < 8p, Y < 4p, ZZ, ZZZ < 2p (in and out), so no product or sum is
// brought below p on the chain: the canonical (< p) form is taken once, when a point leaves
// (g1q_to).  The round-4 canonical policy spent a conditional subtraction (~40 VALU) after every
// product, sum and difference of the chain.
// lane K of the caller's quad to all four lanes: DPP quad_perm [K,K,K,K] (a VALU move, no
// LDS-path round trip as with ds_bpermute)
template <int K, int N>
ZK_DEV void quad_bcast_words(const uint32_t (&v)[N], uint32_t (&r)[N]) {
#pragma unroll
  for (int i = 0; i < N; i++) r[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)v[i], K * 0x55, 0xF, 0xF, false);
}
template <int N>
ZK_DEV void pick4_words(int q, const uint32_t (&a)[N], const uint32_t (&b)[N], const uint32_t (&c)[N],
                        const uint32_t (&d)[N], uint32_t (&r)[N]) {
#pragma unroll
  for (int i = 0; i < N; i++) r[i] = (q & 2) ? ((q & 1) ? d[i] : c[i]) : ((q & 1) ? b[i] : a[i]);
}

struct Q29 {
  using T = F29;
  // ZKFL_Q29_ACC: accumulators per product column of the assembly's quad operations (an A/B knob:
  // one wave alone on its SIMD might issue from more chains; 4 measured 2,075 vs 2,106 config-5
  // proofs/s and 4.05 vs 4.00 ms alone, 3 same-box alternations, profiles/r05_ab_q29_acc.log: the
  // extra joins cost what the shorter spine saves)
#ifndef ZKFL_Q29_ACC
#define ZKFL_Q29_ACC 2
#endif
  static ZK_DEV T mul(const T& a, const T& b) { return f29_mul_acc<ZKFL_Q29_ACC>(a, b); }
  static ZK_DEV T add(const T& a, const T& b) {
    T r = f29_add_lazy(a, b);
    f29_norm(r);
    return r;
  }
  template <int K>
  static ZK_DEV T sub(const T& a, const T& b) {
    constexpr Limbs9 k = p29_times(K, true);
    T r;
#pragma unroll
    for (int i = 0; i < 9; i++) r.v[i] = a.v[i] + k.v[i] - b.v[i];
    f29_norm(r);
    return r;
  }
  static ZK_DEV T dbl(const T& a) { return add(a, a); }
  template <int K>
  static ZK_DEV bool is_zero(const T& a) {
    bool z = false;
#pragma unroll
    for (int m = 0; m < K; m++) {
      const Limbs9 mp = p29_times(m, false);
      uint32_t d = 0;
#pragma unroll
      for (int i = 0; i < 9; i++) d |= a.v[i] ^ mp.v[i];
      z = z || d == 0;
    }
    return z;
  }
  // a < 8p -> canonical (< p)
  static ZK_DEV T canon(const T& a) { return f29_canon_sub<7>(a); }
  static ZK_DEV T zero() { return f29_zero(); }
  static ZK_DEV T one() { return f29_const(P29::ONE); }
  template <int K>
  static ZK_DEV T bcast(const T& v) {
    T r;
    quad_bcast_words<K, 9>(v.v, r.v);
    return r;
  }
  // operands by value: over references the select chain becomes a select of addresses, which
  // pins every operand to the stack
  static ZK_DEV T pick4(int q, T a, T b, T c, T d) {
    T r;
    pick4_words<9>(q, a.v, b.v, c.v, d.v, r.v);
    return r;
  }
  // Fq (Montgomery 2^256, canonical) <-> this representation
  static ZK_DEV T from_fq(const Fq& x) {
    Fq c;
#pragma unroll
    for (int i = 0; i < 8; i++) c.v[i] = P29::C261[i];
    return f29_pack(fp_mul(x, c).v);  // X 2^256 -> X 2^261, canonical
  }
  static ZK_DEV Fq to_fq(const T& x) {
    Fq r, k = fp_zero<FqP>();
    f29_unpack(r.v, x);
    k.v[7] = 1u << 27;  // 2^251: X 2^261 -> X 2^256
    return fp_mul(r, k);
  }
};

// The row policy of the GLV chains (glv_row_mul): row29.h over Fq
using Row29 = RowF<P29>;

template <class QF>
struct QPoint {
  typename QF::T X, Y, ZZ, ZZZ;
};
template <class QF>
ZK_DEV bool qp_is_inf(const QPoint<QF>& p) { return QF::template is_zero<2>(p.ZZ); }  // ZZ < 2p
template <class QF>
ZK_DEV QPoint<QF> qp_inf() { return {QF::one(), QF::one(), QF::zero(), QF::zero()}; }
using G1Q = QPoint<Q29>;
ZK_DEV G1Q g1q_from(const G1P& p) {
  return {Q29::from_fq(p.X), Q29::from_fq(p.Y), Q29::from_fq(p.ZZ), Q29::from_fq(p.ZZZ)};
}
ZK_DEV G1P g1q_to(const G1Q& p) {  // canonical coordinates out
  return {Q29::to_fq(Q29::canon(p.X)), Q29::to_fq(Q29::canon(p.Y)), Q29::to_fq(Q29::canon(p.ZZ)),
          Q29::to_fq(Q29::canon(p.ZZZ))};
}

// dbl-2008-s-1 by levels: {U^2, X^2} -> {U V, X V, V ZZ, M^2} -> {M (S - X3), W Y, W ZZZ}
// Bounds (X < 8p, Y < 4p, ZZ, ZZZ < 2p in): U < 8p; V, X2 < 2p (64 p^2); M < 6p; W, S, ZZ3, M2
// < 2p (36 p^2); X3 < 6p; S - X3 < 8p; Y3's products < 2p (48 p^2), Y3 < 4p.
// CHECK = false: the operands are known to be finite and distinct (the row chains of glv_row_mul),
// so the special cases are not tested (the row policy has no is_zero)
template <class QF, bool CHECK = true>
ZK_DEV QPoint<QF> quad_dbl(const QPoint<QF>& p, int q) {
  using T = typename QF::T;
  if constexpr (CHECK) {
    if (qp_is_inf(p)) return p;
  }
  const T U = QF::dbl(p.Y);
  const T a1 = QF::pick4(q & 1, U, p.X, U, p.X);
  T t = QF::mul(a1, a1);
  const T V = QF::template bcast<0>(t), X2 = QF::template bcast<1>(t);
  const T M = QF::add(QF::dbl(X2), X2);
  t = QF::mul(QF::pick4(q, U, p.X, p.ZZ, M), QF::pick4(q, V, V, V, M));
  const T W = QF::template bcast<0>(t), S = QF::template bcast<1>(t), ZZ3 = QF::template bcast<2>(t),
          M2 = QF::template bcast<3>(t);
  QPoint<QF> r;
  r.X = QF::template sub<4>(M2, QF::dbl(S));
  t = QF::mul(QF::pick4(q, M, W, W, W), QF::pick4(q, QF::template sub<6>(S, r.X), p.Y, p.ZZZ, p.ZZZ));
  r.Y = QF::template sub<2>(QF::template bcast<0>(t), QF::template bcast<1>(t));
  r.ZZ = ZZ3;
  r.ZZZ = QF::template bcast<2>(t);
  return r;
}

// add-2008-s by levels: {U1, U2, S1, S2} -> {P^2, R^2, ZZ1 ZZ2, ZZZ1 ZZZ2} -> {P PP, U1 PP, ZZ PP}
// -> {R (Q - X3), S1 PPP, ZZZ PPP}
// Bounds (both points X < 8p, Y < 4p, ZZ, ZZZ < 2p): U1, U2, S1, S2 < 2p (16 p^2); P, R < 4p;
// PP, R2, Z12, ZZZ12 < 2p; PPP, Q, ZZ3 < 2p; X3 < 8p; Q - X3 < 10p; Y3's products < 2p
// (40 p^2), Y3 < 4p.
template <class QF, bool CHECK = true>
ZK_DEV QPoint<QF> quad_add(const QPoint<QF>& p, const QPoint<QF>& o, int q) {
  using T = typename QF::T;
  if constexpr (CHECK) {
    if (qp_is_inf(o)) return p;
    if (qp_is_inf(p)) return o;
  }
  T t = QF::mul(QF::pick4(q, p.X, o.X, p.Y, o.Y), QF::pick4(q, o.ZZ, p.ZZ, o.ZZZ, p.ZZZ));
  const T U1 = QF::template bcast<0>(t), U2 = QF::template bcast<1>(t), S1 = QF::template bcast<2>(t),
          S2 = QF::template bcast<3>(t);
  const T P = QF::template sub<2>(U2, U1), R = QF::template sub<2>(S2, S1);
  if constexpr (CHECK) {
    if (QF::template is_zero<4>(P)) {
      if (QF::template is_zero<4>(R)) return quad_dbl<QF>(p, q);
      return qp_inf<QF>();
    }
  }
  t = QF::mul(QF::pick4(q, P, R, p.ZZ, p.ZZZ), QF::pick4(q, P, R, o.ZZ, o.ZZZ));
  const T PP = QF::template bcast<0>(t), R2 = QF::template bcast<1>(t), Z12 = QF::template bcast<2>(t),
          ZZZ12 = QF::template bcast<3>(t);
  t = QF::mul(QF::pick4(q, P, U1, Z12, P), PP);
  const T PPP = QF::template bcast<0>(t), Q = QF::template bcast<1>(t);
  QPoint<QF> r;
  r.ZZ = QF::template bcast<2>(t);
  r.X = QF::template sub<4>(QF::template sub<2>(R2, PPP), QF::dbl(Q));
  const T QX = QF::template sub<8>(Q, r.X);
  t = QF::mul(QF::pick4(q, R, S1, ZZZ12, R), QF::pick4(q, QX, PPP, PPP, QX));
  r.Y = QF::template sub<2>(QF::template bcast<0>(t), QF::template bcast<1>(t));
  r.ZZZ = QF::template bcast<2>(t);
  return r;
}

// Fq inverse on one lane (f29_inv_divsteps): Montgomery 2^256 form in and out (0 -> 0).  The
// proof's last affine conversion (pi_c) sits on the assembly's critical path.
ZK_DEV Fq fq_inv29(const Fq& a) {
  Fq c, k = fp_zero<FqP>();
#pragma unroll
  for (int i = 0; i < 8; i++) c.v[i] = P29::C261[i];
  const Fq a261 = fp_mul(a, c);  // A 2^256 -> A 2^261 (the 29-bit engine's Montgomery domain)
  Fq r;
  const F29 a29 = f29_pack(a261.v);
  f29_unpack(r.v, f29_inv_divsteps(a29));  // A^-1 2^261, canonical
  k.v[7] = 1u << 27;  // 2^251: x 2^261 -> x 2^256
  return fp_mul(r, k);
}

ZK_DEV Affine<FqOps> g1_to_affine29(const G1P& p) {
  if (xyzz_is_inf<FqOps>(p)) return {fp_zero<FqP>(), fp_zero<FqP>()};
  const Fq iZZZ = fq_inv29(p.ZZZ);
  const Fq iZ = fp_mul(p.ZZ, iZZZ);  // ZZ / ZZZ = 1 / Z
  return {fp_mul(p.X, fp_mul(iZ, iZ)), fp_mul(p.Y, iZZZ)};
}

// G2 likewise: (a0 + a1 u)^-1 = (a0 - a1 u) / (a0^2 + a1^2), one Fq inverse
ZK_DEV Affine<Fq2Ops> g2_to_affine29(const G2P& p) {
  if (xyzz_is_inf<Fq2Ops>(p)) return {f2_zero(), f2_zero()};
  const Fq2& z = p.ZZZ;
  const Fq ni = fq_inv29(fp_add(fp_sqr(z.c0), fp_sqr(z.c1)));
  const Fq2 iZZZ = {fp_mul(z.c0, ni), fp_neg(fp_mul(z.c1, ni))};
  const Fq2 iZ = f2_mul(p.ZZ, iZZZ);
  return {f2_mul(p.X, f2_sqr(iZ)), f2_mul(p.Y, iZZZ)};
}

// One GLV half of the assembly's scalar multiplications, on one whole wave in the row policy (Row29):
// wave g < 4 computes k_g * P_g for (s1, A'), (s2, phi(A')), (r1, B1'), (r2, phi(B1')) (res[0] =
// A', res[1] = B1'), the GLV halves of s and r (glv.h): 128-bit scalars in signed 4-bit windows
// over a table of 1P..8P in LDS, the wave's four rows evaluating each level's products side by
// side (a quad chain in one wave, the round-4..6 form, took 664 us per assembly under config 5's
// load against 405 us: profiles/r06_ab_row_assembly.log).  No special cases are tested, and
// none can occur: P' = +-P or +-phi(P) is finite (checked) of prime order r; the table j P'
// (j <= 8) is built by one doubling and additions (j - 1) P' + P', j >= 3; the accumulator starts
// at the first nonzero window and is then m P' with m >= 1 -- the signed base-16 prefix of a
// non-negative scalar is >= 0, and 16 m' + d >= 9 once m' >= 1 -- so every addition adds
// d P' (|d| <= 8) to 16 m' P' with 16 <= 16 m' < 2^133 < r - 8 (never equal, opposite or
// infinity), and a doubling never meets a point of order 2.  The proof bytes are the quad
// chain's (same integers: the row product is the same Montgomery reduction).
// tab: this wave's LDS table, 8 points x 4 coordinates x 64 lanes.
ZK_DEV G1Q glv_row_mul(const G1P* __restrict__ res, const GlvScalar* __restrict__ ks, uint32_t* tab, int g) {
  using RPt = QPoint<Row29>;
  G1P P = res[g >> 1];
  if (g & 1) {  // phi(X/ZZ, Y/ZZZ) = (beta X/ZZ, Y/ZZZ)
    Fq beta;
#pragma unroll
    for (int i = 0; i < 8; i++) beta.v[i] = GLV_BETA[i];
    P.X = fp_mul(P.X, fp_to_mont(beta));
  }
  const GlvScalar k = ks[g];
  if (k.neg) P = xyzz_neg<FqOps>(P);
  const G1Q P29 = g1q_from(P);
  if (qp_is_inf(P29)) return qp_inf<Q29>();
  const int lane = (int)__lane_id(), q = lane >> 4;
  const RPt Pr = {Row29::from(P29.X), Row29::from(P29.Y), Row29::from(P29.ZZ), Row29::from(P29.ZZZ)};
  auto put = [&](int e, const RPt& t) {
    tab[(4 * e + 0) * 64 + lane] = t.X.v;
    tab[(4 * e + 1) * 64 + lane] = t.Y.v;
    tab[(4 * e + 2) * 64 + lane] = t.ZZ.v;
    tab[(4 * e + 3) * 64 + lane] = t.ZZZ.v;
  };
  put(0, Pr);
  RPt Q = quad_dbl<Row29, false>(Pr, q);
  put(1, Q);
#pragma unroll 1
  for (int e = 2; e < 8; e++) {
    Q = quad_add<Row29, false>(Q, Pr, q);
    put(e, Q);
  }
  // signed base-16 digits d_0..d_32 in [-7, 8], packed as nibbles (d & 15): word i holds
  // d_8i .. d_8i+7, word 4 holds d_32 (the final carry)
  uint32_t dg[5] = {0, 0, 0, 0, 0};
  uint32_t carry = 0;
  for (int w = 0; w < 32; w++) {
    const uint32_t v = ((k.mag[w >> 3] >> (4 * (w & 7))) & 15u) + carry;
    carry = v > 8 ? 1u : 0u;
    dg[w >> 3] |= (carry ? (v - 16) & 15u : v) << (4 * (w & 7));
  }
  dg[4] = carry;
  bool inf = true;
  RPt acc = Pr;
#pragma unroll 1
  for (int w = 32; w >= 0; w--) {
    if (!inf)
      for (int i = 0; i < 4; i++) acc = quad_dbl<Row29, false>(acc, q);
    const int wi = w >> 3;
    const uint32_t word = wi == 0 ? dg[0] : wi == 1 ? dg[1] : wi == 2 ? dg[2] : wi == 3 ? dg[3] : dg[4];
    const uint32_t nib = (word >> (4 * (w & 7))) & 15u;
    if (nib) {
      const int d = nib >= 9 ? (int)nib - 16 : (int)nib;
      const int e = (d < 0 ? -d : d) - 1;
      RPt t = {{tab[(4 * e + 0) * 64 + lane]}, {tab[(4 * e + 1) * 64 + lane]}, {tab[(4 * e + 2) * 64 + lane]},
               {tab[(4 * e + 3) * 64 + lane]}};
      if (d < 0) t.Y = Row29::sub<4>(Row29::zero(), t.Y);  // Y < 4p
      if (inf)
        acc = t;
      else
        acc = quad_add<Row29, false>(acc, t, q);
      inf = false;
    }
  }
  if (inf) return qp_inf<Q29>();
  return {Row29::to(acc.X), Row29::to(acc.Y), Row29::to(acc.ZZ), Row29::to(acc.ZZZ)};
}

constexpr int ASM_THREADS = 64 * 5;    // k_assemble: four chain waves + the C' + H wave
constexpr int ASM_T_THREADS = 64 * 4;  // k_assemble_t: four chain waves

struct AsmLds {
  uint32_t rtab[4][8 * 4 * 64];  // the chains' tables
  G1Q part[6];                   // the four products, C' + H, then the sum of parts 2 + 3
};

// After the chains (part[0..3] in LDS, a barrier behind): quads 0 and 1 of wave 0 add parts 0 + 1
// and 2 + 3 in one pass (the same instructions, operands by quad); quad 1 leaves its sum in part[5]
// for the caller's next barrier.  -> quad 0's sum of parts 0 + 1.
ZK_DEV G1Q asm_pair_sums(AsmLds& sh, int g, int q) {
  const int h = g & 1;
  const G1Q s = quad_add<Q29>(sh.part[2 * h], sh.part[2 * h + 1], q);
  if (g == 1 && q == 0) sh.part[5] = s;
  return s;
}

// Proof assembly, one block (replaces snarkjs's final
// pi_c = C + H + s*A + r*B1 - rs*delta; the rs*delta term is already in the C MSM):
//   waves 0..3: the four GLV halves (glv_row_mul) -> part[0..3]; wave 4: C' + H meanwhile;
//   then wave 0 sums the parts (asm_pair_sums, then quad 0 adds 2 + 3 and C' + H) and writes pi_c
//   -> proof[48..63], while lane 0 of wave 1 / wave 2 converts pi_a / pi_b -> proof[0..15] /
//   proof[16..47] -- after the chains, so that no inversion shares a SIMD with a chain
// The critical path is 132 doublings + 33 additions on the chains, 3 quad additions and one
// inversion; the quad operations run in the 29-bit engine (Q29), the inversions by divsteps.
__global__ void __launch_bounds__(ASM_THREADS) k_assemble(const G1P* __restrict__ res, const G2P* __restrict__ resB2,
                                                          const GlvScalar* __restrict__ ks, uint32_t* __restrict__ proof) {
  ZK_WT(WT_ASSEMBLE);
  ZK_LIGHT();
  // one block per proof: block b reads res[5b..], resB2[b], ks[4b..] and writes proof[64b..]
  res += 5 * blockIdx.x;
  resB2 += blockIdx.x;
  ks += 4 * blockIdx.x;
  proof += 64 * blockIdx.x;
  __shared__ AsmLds sh;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), lane = threadIdx.x & 63;
  const int g = lane >> 2, q = lane & 3;
  if (wave < 4) {
    const G1Q acc = glv_row_mul(res, ks, sh.rtab[wave], wave);
    if (lane == 0) sh.part[wave] = acc;
  } else if (g == 0) {  // wave 4: C' + H
    const G1Q c = quad_add<Q29>(g1q_from(res[2]), g1q_from(res[3]), q);
    if (q == 0) sh.part[4] = c;
  }
  __syncthreads();
  G1Q t01 = qp_inf<Q29>();
  if (wave == 0) t01 = asm_pair_sums(sh, g, q);
  __syncthreads();
  if (wave == 0 && g == 0) {
    const G1Q C = quad_add<Q29>(quad_add<Q29>(t01, sh.part[5], q), sh.part[4], q);
    if (q == 0) store_affine_std<FqOps>(g1_to_affine29(g1q_to(C)), proof + 48);
  } else if (wave == 1 && lane == 0) {
    store_affine_std<FqOps>(g1_to_affine29(res[0]), proof);
  } else if (wave == 2 && lane == 0) {
    store_affine_std<Fq2Ops>(g2_to_affine29(resB2[0]), proof + 16);
  }
}

// The same assembly in two launches for the low-latency schedule (enqueue_proof, one proof alone):
// k_assemble_t runs as soon as A' and B1' are final, beside the ABC / NTT / C + H chain:
// T = s pi_A + r B1 -> res[4] (XYZZ, Montgomery 2^256) and pi_a -> proof[0..15];
// k_assemble_c at the end: pi_c = (C' + H) + T -> proof[48..63] and pi_b -> proof[16..47].
// pi_c is the same point as k_assemble's (the group sum does not depend on the order), so the
// proof bytes are identical.
__global__ void __launch_bounds__(ASM_T_THREADS) k_assemble_t(G1P* __restrict__ res, const GlvScalar* __restrict__ ks,
                                                              uint32_t* __restrict__ proof) {
  ZK_WT(WT_ASSEMBLE);
  ZK_LIGHT();
  __shared__ AsmLds sh;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), lane = threadIdx.x & 63;
  const int g = lane >> 2, q = lane & 3;
  const G1Q acc = glv_row_mul(res, ks, sh.rtab[wave], wave);
  if (lane == 0) sh.part[wave] = acc;
  __syncthreads();
  G1Q t01 = qp_inf<Q29>();
  if (wave == 0) t01 = asm_pair_sums(sh, g, q);
  __syncthreads();
  if (wave == 0 && g == 0) {
    const G1Q T = quad_add<Q29>(t01, sh.part[5], q);
    if (q == 0) res[4] = g1q_to(T);
  } else if (wave == 1 && lane == 0) {
    store_affine_std<FqOps>(g1_to_affine29(res[0]), proof);
  }
}

// Parity hook for the assembly's scalar multiplications (zkfl_debug_g1_glv_mul): block b computes
// k_b P_b as k_assemble computes s pi_A' -- two row chains (glv_row_mul over (k1, P) and
// (k2, phi(P)), the GLV halves of k), their sum by a quad addition, affine by the divsteps inverse.
// pts: affine std (x, y), (0, 0) = infinity; out: affine std, infinity as zeros.
__global__ void __launch_bounds__(128) k_debug_glv_mul(const uint32_t* __restrict__ pts,
                                                       const GlvScalar* __restrict__ ks, uint32_t* __restrict__ out) {
  const uint32_t* pa = pts + 16 * blockIdx.x;
  ks += 2 * blockIdx.x;
  out += 16 * blockIdx.x;
  __shared__ uint32_t rtab[2][8 * 4 * 64];
  __shared__ G1Q part[2];
  __shared__ G1P P;
  if (threadIdx.x == 0) {
    Fq x, y;
    uint32_t z = 0;
    for (int i = 0; i < 8; i++) {
      x.v[i] = pa[i];
      y.v[i] = pa[8 + i];
      z |= x.v[i] | y.v[i];
    }
    P = z ? G1P{fp_to_mont(x), fp_to_mont(y), fp_one<FqP>(), fp_one<FqP>()} : xyzz_inf<FqOps>();
  }
  __syncthreads();
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), lane = threadIdx.x & 63;
  const G1Q acc = glv_row_mul(&P, ks, rtab[wave], wave);
  if (lane == 0) part[wave] = acc;
  __syncthreads();
  if (wave == 0 && lane < 4) {
    const G1Q S = quad_add<Q29>(part[0], part[1], lane & 3);
    if (lane == 0) store_affine_std<FqOps>(g1_to_affine29(g1q_to(S)), out);
  }
}

__global__ void __launch_bounds__(128) k_assemble_c(const G1P* __restrict__ res, const G2P* __restrict__ resB2,
                                                    uint32_t* __restrict__ proof) {
  ZK_WT(WT_ASSEMBLE);
  ZK_LIGHT();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int g = lane >> 2, q = lane & 3;
  if (wave == 0 && g == 0) {
    const G1Q C = quad_add<Q29>(quad_add<Q29>(g1q_from(res[2]), g1q_from(res[3]), q), g1q_from(res[4]), q);
    if (q == 0) store_affine_std<FqOps>(g1_to_affine29(g1q_to(C)), proof + 48);
  } else if (wave == 1 && lane == 0) {
    store_affine_std<Fq2Ops>(g2_to_affine29(resB2[0]), proof + 16);
  }
}

// Parts of a split proof (zkfl_groth16_prove_part_batch / zkfl_groth16_assemble): a shard's MSM
// results as XYZZ points, every coordinate in standard form (so the parts cross process boundaries
// in a defined encoding without an inversion per point): A' (32 words) | B1' (32) | B2' (64: each
// coordinate c0, c1) | C' (32) | H (32); ZZ = 0 is infinity.
constexpr int PART_WORDS = 192;  // 768 B
__device__ constexpr int PART_OFF[5] = {0, 32, 128, 160, 64};  // A', B1', C', H (G1), B2' (G2)

__device__ void st_std(const Fq& a, uint32_t* out) {
  const Fq x = fp_from_mont(a);
  for (int i = 0; i < 8; i++) out[i] = x.v[i];
}
__device__ void st_std(const Fq2& a, uint32_t* out) {
  st_std(a.c0, out);
  st_std(a.c1, out + 8);
}
__device__ void ld_std(Fq& a, const uint32_t* in) {
  for (int i = 0; i < 8; i++) a.v[i] = in[i];
  a = fp_to_mont(a);
}
__device__ void ld_std(Fq2& a, const uint32_t* in) {
  ld_std(a.c0, in);
  ld_std(a.c1, in + 8);
}
template <class F>
__device__ void st_xyzz_std(const XYZZ<F>& p, uint32_t* out) {
  constexpr int w = sizeof(typename F::T) / 4;
  st_std(p.X, out);
  st_std(p.Y, out + w);
  st_std(p.ZZ, out + 2 * w);
  st_std(p.ZZZ, out + 3 * w);
}
template <class F>
__device__ XYZZ<F> ld_xyzz_std(const uint32_t* in) {
  constexpr int w = sizeof(typename F::T) / 4;
  XYZZ<F> p;
  ld_std(p.X, in);
  ld_std(p.Y, in + w);
  ld_std(p.ZZ, in + 2 * w);
  ld_std(p.ZZZ, in + 3 * w);
  return p;
}

// the slot's MSM results -> its part (one lane per point)
__global__ void __launch_bounds__(64) k_part_out(const G1P* __restrict__ res, const G2P* __restrict__ resB2,
                                                 uint32_t* __restrict__ out) {
  const int lane = threadIdx.x;
  if (lane < 4) st_xyzz_std<FqOps>(res[lane], out + PART_OFF[lane]);
  else if (lane == 4) st_xyzz_std<Fq2Ops>(resB2[0], out + PART_OFF[4]);
}

// A part's point crossed a process boundary: it must be infinity (ZZ = ZZZ = 0) or a well-formed
// XYZZ point of the curve y^2 = x^3 + b: ZZ, ZZZ != 0, ZZ^3 = ZZZ^2 and (with x = X/ZZ, y = Y/ZZZ,
// multiplied through by ZZ^3 = ZZZ^2) Y^2 = X^3 + b ZZ^3.  A malformed one (say ZZ = 1, ZZZ = 0)
// would otherwise reach the assembly's inversions.
template <class F>
ZK_DEV bool xyzz_part_ok(const XYZZ<F>& p, const typename F::T& b) {
  const bool zz0 = F::is_zero(p.ZZ), zzz0 = F::is_zero(p.ZZZ);
  if (zz0 || zzz0) return zz0 && zzz0;
  const typename F::T zz3 = F::mul(F::sqr(p.ZZ), p.ZZ);
  if (!F::eq(zz3, F::sqr(p.ZZZ))) return false;
  return F::eq(F::sqr(p.Y), F::add(F::mul(F::sqr(p.X), p.X), F::mul(b, zz3)));
}

// block b sums the n_parts parts of proof b (parts[b][j]) into res[5b + {0, 1, 2, 3}] (A', B1', C',
// H) and resB2[b]: lanes 0..3 the G1 points, lane 4 the G2 point, a serial sum over the world size.
// A point that is not on its curve sets *bad (and is left out).
__global__ void __launch_bounds__(64) k_parts_sum(const uint32_t* __restrict__ parts, int n_parts,
                                                  G1P* __restrict__ res, G2P* __restrict__ resB2,
                                                  uint32_t* __restrict__ bad) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const uint32_t* p = parts + (size_t)b * n_parts * PART_WORDS;
  if (lane < 4) {
    Fq b3;
#pragma unroll
    for (int i = 0; i < 8; i++) b3.v[i] = FQ_THREE[i];
    G1P acc = xyzz_inf<FqOps>();
    for (int j = 0; j < n_parts; j++) {
      const G1P q = ld_xyzz_std<FqOps>(p + j * PART_WORDS + PART_OFF[lane]);
      if (xyzz_part_ok<FqOps>(q, b3)) acc = xyzz_add<FqOps>(acc, q);
      else *bad = 1u;
    }
    res[5 * b + lane] = acc;
  } else if (lane == 4) {
    const Fq2 bt = load_fq2(TWIST_B);
    G2P acc = xyzz_inf<Fq2Ops>();
    for (int j = 0; j < n_parts; j++) {
      const G2P q = ld_xyzz_std<Fq2Ops>(p + j * PART_WORDS + PART_OFF[4]);
      if (xyzz_part_ok<Fq2Ops>(q, bt)) acc = xyzz_add<Fq2Ops>(acc, q);
      else *bad = 1u;
    }
    resB2[b] = acc;
  }
}

// MSM result(s) -> std affine bytes (parity hooks)
template <class F>
__global__ void __launch_bounds__(64) k_point_out(const XYZZ<F>* __restrict__ p, int n, uint32_t* __restrict__ out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  constexpr int words = sizeof(Affine<F>) / 4;
  store_affine_std<F>(xyzz_to_affine<F>(p[i]), out + i * words);
}

__global__ void k_fr_std_to_mont(Fr* __restrict__ a, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  a[i] = fp_to_mont(a[i]);
}

__global__ void k_fr_mont_to_std(Fr* __restrict__ a, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  a[i] = fp_from_mont(a[i]);
}

// Dev ceremony: out[i] = k_i * G (mont affine)
template <class F>
__global__ void __launch_bounds__(64) k_gen_mul(const uint32_t* __restrict__ scalars, size_t n, Affine<F> gen_mont,
                          Affine<F>* __restrict__ out) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t k[8];
  for (int j = 0; j < 8; j++) k[j] = scalars[i * 8 + j];
  XYZZ<F> g = xyzz_from_affine<F>(gen_mont);
  out[i] = xyzz_to_affine<F>(xyzz_scalar_mul<F>(g, k));
}

__global__ void k_g1_gen_mont(G1Aff* out) {
  Fq x = fp_zero<FqP>(), y = fp_zero<FqP>();
  x.v[0] = 1;
  y.v[0] = 2;
  out->x = fp_to_mont(x);
  out->y = fp_to_mont(y);
}

__global__ void k_g2_gen_mont(G2Aff* out) {
  // snarkjs/ethereum bn128 G2 generator (std form limbs)
  const uint32_t xc0[8] = {0xd992f6edu, 0x46debd5cu, 0xf75edaddu, 0x674322d4u, 0x5e5c4479u, 0x426a0066u, 0x121f1e76u, 0x1800deefu};
  const uint32_t xc1[8] = {0xaef312c2u, 0x97e485b7u, 0x35a9e712u, 0xf1aa4933u, 0x31fb5d25u, 0x7260bfb7u, 0x920d483au, 0x198e9393u};
  const uint32_t yc0[8] = {0x66fa7daau, 0x4ce6cc01u, 0x0c43d37bu, 0xe3d1e769u, 0x8dcb408fu, 0x4aab7180u, 0xdb8c6debu, 0x12c85ea5u};
  const uint32_t yc1[8] = {0xd122975bu, 0x55acdadcu, 0x70b38ef3u, 0xbc4b3133u, 0x690c3395u, 0xec9e99adu, 0x585ff075u, 0x090689d0u};
  Fq a, b, c, d;
  for (int i = 0; i < 8; i++) {
    a.v[i] = xc0[i];
    b.v[i] = xc1[i];
    c.v[i] = yc0[i];
    d.v[i] = yc1[i];
  }
  out->x = {fp_to_mont(a), fp_to_mont(b)};
  out->y = {fp_to_mont(c), fp_to_mont(d)};
}

}  // namespace

// ---------------------------------------------------------------------------
// Context / key / witness objects
// ---------------------------------------------------------------------------
struct zkfl_ctx {
  int device = 0;
  hipStream_t st = nullptr;  // primitives, key loading, verification
  Profiler prof;
  VkDev* vk = nullptr;       // last prepared verification key (reused while the vk bytes repeat)
  PosTables* pos = nullptr;  // Poseidon constants of every width (first hashing call)
  void* asm_buf = nullptr;   // zkfl_groth16_assemble's device buffers (grown on demand, reused)
  size_t asm_cap = 0;
  WtBuf wt;                  // wave-timeline records (ZK_WTRACE builds, zkfl_debug_wtrace)
  // Lifetime: the caller's handle holds one reference and every key and witness program made on
  // the context holds one more, so zkfl_ctx_destroy and the children's frees may come in any
  // order (the N-API finalizers run in an unspecified order); the device state goes with the last.
  std::atomic<int> refs{1};
};

// One in-flight proof: its own streams, scratch and per-proof vectors.
struct ProofSlot {
  hipStream_t st_main = nullptr, st_g2 = nullptr;
  hipEvent_t ev_ready = nullptr, ev_b2 = nullptr, ev_done = nullptr;
  MsmScratch<FqOps> g1s;   // digit/sort scratch shared by the four G1 MSMs
#if ZK_KNOCKOUT & 2
  MsmScratch<FqOps> g1s_ko[3];  // sort knock-out (timing only): A, B, C+H keep their first sort
#endif
  MsmTail<FqOps> g1t[4];   // A, B1, C, H: accumulated, finished by one batched tail
  MsmScratch<Fq2Ops> g2s;
  MsmTail<Fq2Ops> g2t;
  Fr* extra = nullptr;  // [4] blinding scalars 1, r, s, -rs (= h + n: the extra slots follow h)
  Fr* abc = nullptr;  // [3n]
  Fr* abc_head = nullptr;  // [ceil(K / ABC_L)] ABC segmented-sum partials
  Fr* abc_tail = nullptr;
  Fr* h = nullptr;    // [n]
  G1P* res = nullptr;     // [5]: A', B1', C', H, T
  G2P* resB2 = nullptr;   // [1]
  Fr* d_rs = nullptr;     // r, s (64 B) | GLV halves s1, s2, r1, r2 (4 x 32 B)
  uint32_t* d_parts = nullptr;  // [96]: this rank's part of a split proof (A'|B1'|B2'|C'|H, std affine)
  uint8_t* pinned = nullptr;    // proof (256) | r, s (64) | GLV halves (128) | witness address (8, at
                                // W_PTR_OFF) | pad | part (768 at 512)
  // the low-latency schedule (enqueue_proof_lowlat, one proof alone): two side streams, their
  // events (B sorted and B1 accumulated | B2 final | T = s pi_A + r B1 final) and B's own sort
  // scratch, so C + H can sort on the main stream while B2 still reads B's pairs; made on first use
  hipStream_t st_lat[2] = {nullptr, nullptr};
  hipEvent_t ev_lat[3] = {nullptr, nullptr, nullptr};
  MsmScratch<FqOps> g1s_b;
  MsmScratch<FqOps> g1s_a;  // A's sort scratch in the overlapped schedule (A beside C + H)
  // graph replay (default on; ZKFL_GRAPH=0 off): the one-stream proof chain captured once per witness address
  struct Graph {
    const Fr* w = nullptr;
    hipGraph_t g = nullptr;
    hipGraphExec_t ex = nullptr;
  };
  std::vector<Graph> graphs;
  // the graph's witness: each graph-replayed proof first copies its witness here (nVars x 32 B,
  // a few us of HBM time), so one graph per slot serves every witness buffer
  Fr* w_stage = nullptr;
  uint32_t direct_proofs = 0;     // proofs this slot ran kernel by kernel (the first one: no capture)
  // B2 shares B1's digit sort, so its tail counts with B1's nnz (g2t.nnz == g1t[1].nnz, owned
  // by g1t[1]): no copy between them
  bool nnz_alias = false;
  bool busy = false;
  int index = 0;                  // position among its key's slots
  size_t job = 0;                 // index of the in-flight proof in its batch
  uint8_t* out_proof = nullptr;   // where its 256 proof bytes go (nullable)
  uint8_t* out_part = nullptr;    // split proofs: where the 768 part bytes go (nullable)
};

#ifndef ZK_NO_SHARE_B
#define ZK_NO_SHARE_B 0  // 1: B2 sorts its own digits (A/B builds)
#endif
#ifndef MSM_MERGE_CH
#define MSM_MERGE_CH 1   // 0: C and H as two MSMs with their own sorts and tails (A/B builds)
#endif
struct zkfl_key {
  zkfl_ctx* ctx = nullptr;
  uint32_t nVars = 0, nPub = 0, n = 0;
  int logn = 0;
  size_t nC = 0;  // C query length
  size_t K = 0;
  uint32_t* rows = nullptr;  // [2n+1]: A rows then B rows over one term array
  uint32_t* cols = nullptr;  // [K]
  Fr* coefs = nullptr;       // [K] (wide) or the coefficient dictionary (packed)
  uint32_t cshift = 0;       // packed terms: col | dict index << cshift in cols[]; 0 = wide
  MsmBases<FqOps> bA, bB1, bC, bH;
  MsmBases<Fq2Ops> bB2;
  // C and H as ONE MSM (MSM_MERGE_CH): pi_C only needs their sum, so one sort and one tail serve
  // both queries.  Bases: C's (scalars: the private wires) then H's (scalars: h, addressed through
  // the extra pointer = the slot's h vector, whose extra slots 1, r, s, -rs follow it).  bC / bH
  // stay for the parity hook (zkfl_debug_prove_parts returns C and H apart).
  MsmBases<FqOps> bCH;
  // the parity hook's zeros (zkfl_debug_prove_parts, first call): with C and H merged it runs the
  // C + H MSM twice, once with a zero h (C alone) and once with a zero witness (H alone), so the key
  // holds no separate C and H bases (they were ~0.5 GB of expanded bases per key at 2^18)
  Fr* dbg_zero = nullptr;
  bool share_b = false;  // B1 and B2 have the same base index map: one digit sort serves both
  // small keys (domain <= 2^16, config 5's circuits): a proof sorts A, B1 and C + H in the same four
  // launches and accumulates them in one (msm_sort_multi / msm_accumulate_sorted_multi), after ABC /
  // NTT; the slots hold A's and B's sort scratch for it (g1s_a, g1s_b)
  bool front = false;
  int msm_c = MSM_C;     // window bits of every base set of the key (msm_pick_c of its largest)
  NttPlan ntt;
  std::vector<ProofSlot*> slots;
  int max_slots = 3;
  // Split proofs (zkfl_zkey_load_shard): this key holds base i of every query only when
  // i % nshards == shard, and the alpha/beta/delta augmentation bases only on shard 0, so its
  // MSMs are this shard's share of each proof's sums.
  uint32_t shard = 0, nshards = 1;
  struct WitPipe* wpipe = nullptr;  // batched witnesses of the single-key full-prove entry points
};

struct zkfl_witness {
  const zkfl_key* key = nullptr;
  Fr* d = nullptr;  // nVars std-form elements
  std::vector<uint8_t> pub;  // nPub x 32 B
};

struct zkfl_wprog {
  zkfl_ctx* ctx = nullptr;
  WProg* p = nullptr;
};

static void ctx_retain(zkfl_ctx* ctx);
static void ctx_release(zkfl_ctx* ctx);

namespace {

constexpr size_t W_PTR_OFF = 448;  // pinned: the graph-replayed proof's witness address

// the proof's 256 bytes go straight into the slot's pinned buffer (k_assemble*)
inline uint32_t* proof_out(ProofSlot* s) { return reinterpret_cast<uint32_t*>(s->pinned); }

void slot_release(ProofSlot* s) {
  if (!s) return;
  for (hipStream_t st : {s->st_main, s->st_g2})
    if (st) (void)hipStreamSynchronize(st);
  if (s->nnz_alias) s->g2t.nnz = nullptr;
  msm_scratch_free_g1(s->g1s);
#if ZK_KNOCKOUT & 2
  for (MsmScratch<FqOps>& x : s->g1s_ko) msm_scratch_free_g1(x);
#endif
  for (auto& t : s->g1t) msm_tail_free_g1(t);
  msm_scratch_free_g2(s->g2s);
  msm_tail_free_g2(s->g2t);
  void* ptrs[] = {s->abc, s->abc_head, s->abc_tail, s->h, s->res, s->resB2, s->d_rs, s->d_parts,
                  s->w_stage};  // extra lives in h
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (s->pinned) (void)hipHostFree(s->pinned);
  for (hipStream_t st : s->st_lat)
    if (st) (void)hipStreamSynchronize(st);
  msm_scratch_free_g1(s->g1s_b);
  msm_scratch_free_g1(s->g1s_a);
  for (auto& gr : s->graphs) {
    if (gr.ex) (void)hipGraphExecDestroy(gr.ex);
    if (gr.g) (void)hipGraphDestroy(gr.g);
  }
  s->graphs.clear();
  for (hipEvent_t e : {s->ev_ready, s->ev_b2, s->ev_done, s->ev_lat[0], s->ev_lat[1], s->ev_lat[2]})
    if (e) (void)hipEventDestroy(e);
  for (hipStream_t st : {s->st_main, s->st_g2, s->st_lat[0], s->st_lat[1]})
    if (st) (void)hipStreamDestroy(st);
  delete s;
}

int graph_mode();

// Release a slot's latency-schedule streams and events (made again on its next batch of one).
void slot_drop_lowlat(ProofSlot* s) {
  for (hipStream_t& st : s->st_lat)
    if (st) {
      (void)hipStreamSynchronize(st);
      (void)hipStreamDestroy(st);
      st = nullptr;
    }
  for (hipEvent_t& e : s->ev_lat)
    if (e) {
      (void)hipEventDestroy(e);
      e = nullptr;
    }
}

hipError_t slot_create(zkfl_key* k, ProofSlot** out) {
  ProofSlot* s = new ProofSlot();
  *out = s;
  const size_t nV = k->nVars, n = k->n;
  const size_t cap1 = std::max<size_t>({k->bA.n, k->bB1.n, k->bC.n, k->bH.n, k->bCH.n});
  hipStream_t st = k->ctx->st;
  ZK_CHECK(hipStreamCreateWithFlags(&s->st_main, hipStreamNonBlocking));
  // One stream per slot by default: a slot's proof is a serial chain and throughput comes from
  // many slots (measured on MI355X, 24 HW queues: 16 slots x 1 stream 238-241 proofs/s vs
  // 8 slots x 3 streams 216-217).  ZKFL_SLOT_STREAMS=2 runs the G2 MSM on a second stream.
  static const int streams = getenv("ZKFL_SLOT_STREAMS") ? atoi(getenv("ZKFL_SLOT_STREAMS")) : 1;
  if (streams > 1) ZK_CHECK(hipStreamCreateWithFlags(&s->st_g2, hipStreamNonBlocking));
  for (hipEvent_t* e : {&s->ev_ready, &s->ev_b2, &s->ev_done})
    ZK_CHECK(hipEventCreateWithFlags(e, hipEventDisableTiming));
  const int c = k->msm_c;
  ZK_CHECK(msm_scratch_alloc_g1(s->g1s, cap1, c, st));
#if ZK_KNOCKOUT & 2
  for (MsmScratch<FqOps>& x : s->g1s_ko) {  // zeroed: an index past a stale sort is base 0
    ZK_CHECK(msm_scratch_alloc_g1(x, cap1, c, st));
    ZK_CHECK(hipMemsetAsync(x.keys_out, 0, cap1 * msm_w_of(c) * sizeof(uint16_t), st));
    ZK_CHECK(hipMemsetAsync(x.vals_out, 0, cap1 * msm_w_of(c) * sizeof(uint32_t), st));
  }
#endif
  // tail 3 is H's; with C and H merged the parity hook uses it for the C + H MSM
  const size_t caps[4] = {k->bA.n, k->bB1.n, std::max(k->bC.n, k->bCH.n), std::max(k->bH.n, k->bCH.n)};
  for (int i = 0; i < 4; i++) ZK_CHECK(msm_tail_alloc_g1(s->g1t[i], caps[i], c));
  ZK_CHECK(msm_scratch_alloc_g2(s->g2s, k->bB2.n, c, st));
  ZK_CHECK(msm_tail_alloc_g2(s->g2t, k->bB2.n, c));
  if (k->share_b && !s->st_g2 && !ZK_KNOCKOUT) {
    ZK_CHECK(hipFree(s->g2t.nnz));
    s->g2t.nnz = s->g1t[1].nnz;
    s->nnz_alias = true;
  }
  if (graph_mode()) ZK_CHECK(hipMalloc(&s->w_stage, nV * 32));
  if (k->front) {  // A's and B's own sort scratch (C + H sorts in g1s)
    ZK_CHECK(msm_scratch_alloc_g1(s->g1s_a, k->bA.n, c, st));
    ZK_CHECK(msm_scratch_alloc_g1(s->g1s_b, k->bB1.n, c, st));
  }
  ZK_CHECK(hipMalloc(&s->h, (n + 4) * 32));   // h, then the extra slots (the merged C+H MSM's scalars)
  s->extra = s->h + n;
  ZK_CHECK(hipMalloc(&s->abc, n * 3 * 32));
  const size_t abc_chunks = (k->K + ABC_L - 1) / ABC_L + 1;
  ZK_CHECK(hipMalloc(&s->abc_head, abc_chunks * 32));
  ZK_CHECK(hipMalloc(&s->abc_tail, abc_chunks * 32));
  ZK_CHECK(hipMalloc(&s->res, 5 * sizeof(G1P)));
  ZK_CHECK(hipMalloc(&s->resB2, sizeof(G2P)));
  ZK_CHECK(hipMalloc(&s->d_rs, 2 * 32 + 4 * sizeof(GlvScalar)));
  ZK_CHECK(hipMalloc(&s->d_parts, PART_WORDS * 4));
  // coherent (fine-grained): the proof chain reads r, s and the GLV halves from it and writes the
  // proof into it directly (k_proof_start, k_assemble*), so no copy launches open or close a proof
  ZK_CHECK(hipHostMalloc(&s->pinned, 2048, hipHostMallocCoherent));
  return hipStreamSynchronize(st);
}

int get_slot(zkfl_key* k, size_t idx, ProofSlot** out) {
  size_t want = idx % (size_t)k->max_slots;
  while (k->slots.size() <= want) {
    ProofSlot* s = nullptr;
    hipError_t e = slot_create(k, &s);
    if (e != hipSuccess) {
      slot_release(s);
      return hip_fail(e, "proof slot allocation");
    }
    s->index = (int)k->slots.size();
    k->slots.push_back(s);
  }
  *out = k->slots[want];
  return ZKFL_OK;
}

}  // namespace

// Witnesses of the single-key full-prove entry points, computed G (= the key's slots) jobs at a
// time by ONE batched launch sequence of the witness engine on the key's witness stream, ahead of
// the slots that prove them: group g is computed into buffer set g % 3 while the slots prove
// group g - 1 (when group g + 1 is enqueued, the slots have drained group g - 2, so its set is
// free).  Per-slot witnesses cost ~25 small launches per proof on the slot's stream, each a
// permutation-latency chain; batched, a group's 15 levels cost as much as one witness's.
// Witness sets of a key's pipe: group g uses set g % WIT_SETS; groups run up to WIT_SETS - 2 ahead
// of the group the key's slots start (full_prove_piped)
constexpr int WIT_SETS = 4;
struct WitPipe {
  struct Set {
    Fr* W = nullptr;          // [G][nw] Montgomery scratch
    Fr* d = nullptr;          // [G][nw] std-form witnesses = the proofs' scalars
    uint32_t* in = nullptr;   // [G][n_in x 8]
    uint32_t* fail = nullptr; // [G]
    Fr** outs = nullptr;      // [G] device pointers into d
    uint8_t* pin_in = nullptr;
    hipEvent_t ev = nullptr;  // the group's witnesses are complete
  };
  size_t G = 0, nw = 0, n_in = 0;
  hipStream_t st = nullptr;
  Set set[WIT_SETS];
};

namespace {

void wpipe_release(WitPipe* p) {
  if (!p) return;
  if (p->st) (void)hipStreamSynchronize(p->st);
  for (auto& b : p->set) {
    for (void* q : {(void*)b.W, (void*)b.d, (void*)b.in, (void*)b.fail, (void*)b.outs})
      if (q) (void)hipFree(q);
    if (b.pin_in) (void)hipHostFree(b.pin_in);
    if (b.ev) (void)hipEventDestroy(b.ev);
  }
  if (p->st) (void)hipStreamDestroy(p->st);
  delete p;
}

// The key's pipe for groups of G witnesses of nw wires and n_in inputs (kept between calls).
hipError_t wpipe_get(zkfl_key* k, size_t G, size_t nw, size_t n_in, WitPipe** out) {
  WitPipe* p = k->wpipe;
  if (p && p->G == G && p->nw == nw && p->n_in == n_in) {
    *out = p;
    return hipSuccess;
  }
  wpipe_release(p);
  k->wpipe = p = new WitPipe();
  p->G = G;
  p->nw = nw;
  p->n_in = n_in;
  ZK_CHECK(hipStreamCreateWithFlags(&p->st, hipStreamNonBlocking));
  for (auto& b : p->set) {
    ZK_CHECK(hipMalloc(&b.W, G * nw * 32));
    ZK_CHECK(hipMalloc(&b.d, G * nw * 32));
    ZK_CHECK(hipMalloc(&b.in, G * n_in * 32 + 16));
    ZK_CHECK(hipMalloc(&b.fail, G * 4));
    ZK_CHECK(hipMalloc(&b.outs, G * sizeof(Fr*)));
    ZK_CHECK(hipHostMalloc(&b.pin_in, G * n_in * 32 + 16));
    ZK_CHECK(hipEventCreateWithFlags(&b.ev, hipEventDisableTiming));
    std::vector<Fr*> ptrs(G);
    for (size_t j = 0; j < G; j++) ptrs[j] = b.d + j * nw;
    ZK_CHECK(hipMemcpy(b.outs, ptrs.data(), G * sizeof(Fr*), hipMemcpyHostToDevice));
  }
  *out = p;
  return hipSuccess;
}

void key_release(zkfl_key* k) {
  if (!k) return;
  wpipe_release(k->wpipe);
  k->wpipe = nullptr;
  for (ProofSlot* s : k->slots) slot_release(s);
  k->slots.clear();
  msm_bases_free_g1(k->bA);
  msm_bases_free_g1(k->bB1);
  msm_bases_free_g1(k->bC);
  msm_bases_free_g1(k->bH);
  msm_bases_free_g1(k->bCH);
  msm_bases_free_g2(k->bB2);
  if (k->dbg_zero) (void)hipFree(k->dbg_zero);
  ntt_plan_free(k->ntt);
  void* ptrs[] = {k->rows, k->cols, k->coefs};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  zkfl_ctx* ctx = k->ctx;
  delete k;
  if (ctx) ctx_release(ctx);  // the key's reference (taken when it was made)
}

int get_rs(const uint8_t* rs, uint32_t out[16]) {
  if (rs) {
    memcpy(out, rs, 64);
    if (!lt_r(out) || !lt_r(out + 8)) return fail(ZKFL_E_ARG, "r/s must be < r");
    return ZKFL_OK;
  }
  // CSPRNG, rejection-sample below r (snarkjs: Fr.random())
  for (int k = 0; k < 2; k++) {
    for (int tries = 0;; tries++) {
      uint8_t b[32];
      if (getrandom(b, 32, 0) != 32) return fail(ZKFL_E_DEVICE, "getrandom failed");
      b[31] &= 0x3f;  // < 2^254
      memcpy(out + 8 * k, b, 32);
      if (lt_r(out + 8 * k)) break;
      if (tries > 64) return fail(ZKFL_E_DEVICE, "rng");
    }
  }
  return ZKFL_OK;
}

// Enqueue one proof on a slot (asynchronous).  Stream graph (with 1 stream per slot, the
// default, both are the slot's one stream):
//   main : r, s + GLV halves, scalar vectors, [ev_ready] accumulate A, B1, C, ABC, coset NTT x3,
//          join, accumulate H, the four G1 tails as one batch, wait(ev_b2), assembly (T, pi_a,
//          pi_b, pi_c), proof D2H [ev_done]
//   g2   : wait(ev_ready) MSM B2 [ev_b2]
// plain = 1 (parity hook): alpha/beta/delta/r/s terms zeroed, nothing assembled.
// plain = 2 (split proof): the full augmentation (on shard 0's bases), no assembly; the part
// A' | B1' | B2' | C' + H | infinity goes to pinned + 512 (zkfl_groth16_prove_part_batch).
// ABC (a, b, c on the domain), the coset NTT of all three and h = a b - c (std form: the H MSM's
// scalars) for one proof on stream st.
int enqueue_abc_ntt(zkfl_key* k, ProofSlot* s, const Fr* d_w, hipStream_t st, Profiler* prof) {
  const size_t n = k->n;
  int pi = prof->begin("abc", st);
  if (k->K) {
    const uint32_t K = (uint32_t)k->K;
    const AbcTerms T = {k->cols, k->coefs, k->cshift};
    if (k->cshift)
      hipLaunchKernelGGL(k_abc_chunks<true>, dim3(zk_grid((K + ABC_L - 1) / ABC_L, 64)), dim3(64), 0, st, k->rows,
                         (uint32_t)(2 * n), T, d_w, K, s->abc_head, s->abc_tail, s->abc);
    else
      hipLaunchKernelGGL(k_abc_chunks<false>, dim3(zk_grid((K + ABC_L - 1) / ABC_L, 64)), dim3(64), 0, st, k->rows,
                         (uint32_t)(2 * n), T, d_w, K, s->abc_head, s->abc_tail, s->abc);
  }
  hipLaunchKernelGGL(k_abc_rows, dim3(zk_grid(n, 256)), dim3(256), 0, st, k->rows, n, (uint32_t)k->K, s->abc_head,
                     s->abc_tail, s->abc);
  prof->end(pi, st, (double)k->K);
  pi = prof->begin("ntt", st);
  if (!(ZK_KNOCKOUT & 4)) HIP_TRY(ntt_coset_shift(k->ntt, s->abc, 3, n, st), "ntt");
  prof->end(pi, st, 3.0 * (double)n);
  hipLaunchKernelGGL(k_join, dim3(zk_grid(n, 256)), dim3(256), 0, st, s->abc, n, s->h);
  return ZKFL_OK;
}

// The latency schedules reduce their buckets with the shorter-chain reduction (msm.h
// MSM_WSUM_Q_FAST); ZKFL_FAST_WSUM=0 keeps the throughput form (A/B).
bool lowlat_fast_wsum() {
  static const bool on = !getenv("ZKFL_FAST_WSUM") || atoi(getenv("ZKFL_FAST_WSUM")) != 0;
  return on;
}

// Small keys (domain <= 2^ZKFL_FAST_WSUM_LOGN, default 2^16: config 5's circuits) take the
// shorter-chain reduction in batches too: their proofs are chains of small latency-bound kernels
// that leave most of the GPU idle (config-5 wave trace: SIMD share 0.135 with a wave resident 99%
// of the time), so the reduction's extra waves are free and its shorter chain is not.
bool small_key_fast_wsum(const zkfl_key* k) {
  static const int logn = getenv("ZKFL_FAST_WSUM_LOGN") ? atoi(getenv("ZKFL_FAST_WSUM_LOGN")) : 16;
  return lowlat_fast_wsum() && k->logn <= logn;
}

// One proof alone (a batch of one: the CLI's `groth16 prove`, the API's prove): its latency is
// the metric, and the GPU is mostly idle along the one-stream chain, so the two long chains start
// at once on streams of their own:
//   main : r, s, tails reset [ev_ready] ABC, coset NTT, join, C + H (sort + accumulate), its tail,
//          wait(B2, T), k_assemble_c, proof D2H [ev_done]
//   lat0 : wait(ev_ready) B sort (own scratch) [ev B sorted] B2 + its tail [ev B2]
//   lat1 : wait(ev B sorted) B1, A (sort into its own scratch + accumulate), the tails of A and
//          B1, k_assemble_t (T = s pi_A + r B1, pi_a) [ev T]
// Same proof bytes as the one-stream schedule (k_assemble_t / _c form the same points).  The
// round-4 schedule ran A and B1 on the main stream ahead of ABC / NTT (4.10 vs 4.16 ms then); with
// the row assembly and the divsteps inversions the overlap wins: 3.586 vs 3.712 ms, 3 same-box
// alternations (profiles/r06_ab_lowlat2.log), and the round-4 one was deleted, with its
// per-segment graph replay (ZKFL_GRAPH=2: no gain, profiles/r04_ab_lowlat_seg_graphs.log).

// ZKFL_GRAPH (default 1): graph replay of the one-stream proof chain (0: launch kernel by kernel)
int graph_mode() {
  static const int m = getenv("ZKFL_GRAPH") ? atoi(getenv("ZKFL_GRAPH")) : 1;
  return m;
}

// (the schedule above)
int enqueue_proof_lowlat(zkfl_ctx* ctx, zkfl_key* k, ProofSlot* s, const Fr* d_w) {
  Profiler* prof = &ctx->prof;
  hipStream_t st = s->st_main;
  for (int i = 0; i < 2; i++)
    if (!s->st_lat[i]) HIP_TRY(hipStreamCreateWithFlags(&s->st_lat[i], hipStreamNonBlocking), "stream");
  for (int i = 0; i < 3; i++)
    if (!s->ev_lat[i]) HIP_TRY(hipEventCreateWithFlags(&s->ev_lat[i], hipEventDisableTiming), "event");
  if (!s->g1s_b.keys_out) HIP_TRY(msm_scratch_alloc_g1(s->g1s_b, k->bB1.n, k->msm_c, st), "B sort scratch");
  if (!s->g1s_a.keys_out) HIP_TRY(msm_scratch_alloc_g1(s->g1s_a, k->bA.n, k->msm_c, st), "A sort scratch");
  hipStream_t sb = s->st_lat[0], sa = s->st_lat[1];
  // ev_lat[0] marks "ready" then (re-recorded on lat0) "B sorted": each wait is enqueued before
  // the next record, so every wait sees the record it was meant for
  hipEvent_t ev = s->ev_lat[0], ev_b2 = s->ev_lat[1], ev_t = s->ev_lat[2];
  const uint32_t* W = (const uint32_t*)d_w;
  const uint32_t* E = (const uint32_t*)s->extra;
  MsmTail<FqOps>* tails[3] = {&s->g1t[0], &s->g1t[1], &s->g1t[2]};
  MsmTail<Fq2Ops>* t2 = &s->g2t;
  G2P* o2 = s->resB2;
  HIP_TRY(hipEventRecord(ev, st), "event");  // (tails emptied by k_proof_start)
  // lat0: B's sort, then B2 and its tail
  HIP_TRY(hipStreamWaitEvent(sb, ev, 0), "wait");
  HIP_TRY(msm_sort_g1(k->bB1, s->g1s_b, s->g1t[1].nnz, W, E, sb), "msm B sort");
  if (!s->nnz_alias)
    HIP_TRY(hipMemcpyAsync(s->g2t.nnz, s->g1t[1].nnz, sizeof(uint32_t), hipMemcpyDeviceToDevice, sb), "nnz");
  HIP_TRY(hipEventRecord(ev, sb), "event");
  HIP_TRY(hipStreamWaitEvent(sa, ev, 0), "wait");
  HIP_TRY(msm_accumulate_sorted_g2(k->bB2, s->g1s_b.keys_out, s->g1s_b.vals_out, s->g2t, sb, prof,
                                   "msm_accumulate_g2"), "msm B2");
  HIP_TRY(msm_tails_g2(&t2, &o2, 1, sb, lowlat_fast_wsum()), "msm B2 tail");
  HIP_TRY(hipEventRecord(ev_b2, sb), "event");
  // lat1: B1 (B's pairs), A, their tails, then T = s pi_A + r B1 and pi_a
  HIP_TRY(msm_accumulate_sorted_g1(k->bB1, s->g1s_b.keys_out, s->g1s_b.vals_out, s->g1t[1], sa, prof,
                                   "msm_accumulate_g1"), "msm B1");
  HIP_TRY(msm_accumulate_g1(k->bA, s->g1s_a, s->g1t[0], W, E, sa, prof, "msm_accumulate_g1"), "msm A");
  {
    G1P* outs[2] = {s->res + 0, s->res + 1};
    HIP_TRY(msm_tails_g1(tails, outs, 2, sa, lowlat_fast_wsum()), "msm tails A, B1");
  }
  hipLaunchKernelGGL(k_assemble_t, dim3(1), dim3(ASM_T_THREADS), 0, sa, s->res,
                     reinterpret_cast<const GlvScalar*>(reinterpret_cast<const uint8_t*>(s->d_rs) + 64), proof_out(s));
  HIP_TRY(hipEventRecord(ev_t, sa), "event");
  // main: ABC / NTT / h, C + H and its tail, then pi_c and pi_b
  {
    const int rc = enqueue_abc_ntt(k, s, d_w, st, prof);
    if (rc) return rc;
  }
  HIP_TRY(msm_accumulate_g1(k->bCH, s->g1s, s->g1t[2], W, (const uint32_t*)s->h, st, prof, "msm_accumulate_g1"),
          "msm C+H");
  {
    G1P* out2 = s->res + 2;
    HIP_TRY(msm_tails_g1(&tails[2], &out2, 1, st, lowlat_fast_wsum()), "msm tail C+H");
  }
  HIP_TRY(hipStreamWaitEvent(st, ev_b2, 0), "wait");
  HIP_TRY(hipStreamWaitEvent(st, ev_t, 0), "wait");
  const int pa = prof->begin("assemble", st);
  hipLaunchKernelGGL(k_assemble_c, dim3(1), dim3(128), 0, st, s->res, s->resB2, proof_out(s));
  prof->end(pa, st, 1.0);
  return ZKFL_OK;
}

// The device work of one proof on the slot's streams, after the host has put r, s and the GLV
// halves into the pinned buffer.  graph: being captured (one stream): the events that only order
// the one stream against itself are left out.
int enqueue_proof_body(zkfl_ctx* ctx, zkfl_key* k, ProofSlot* s, const Fr* d_w, int plain, int lowlat, bool graph) {
  Profiler* prof = &ctx->prof;
  hipStream_t st = s->st_main;
  hipStream_t st_g2 = (prof->serialize || !s->st_g2) ? st : s->st_g2;
  const size_t n = k->n;
  int pp = prof->begin("prove", st);
  const bool lowlat_path =
      lowlat && plain == 0 && MSM_MERGE_CH && k->share_b && !prof->serialize && !s->st_g2 && !ZK_KNOCKOUT;
  {
    // the tails this chain accumulates into: G1 A, B1, C (+ H), [H]; G2 B2 when it shares B1's sort
    // on this stream (a separate G2 stream's msm_run empties its own).  The condition is the body's
    // `share` below: a slot with a second stream under serialized profiling shares too.
    const int ng1 = lowlat_path || (MSM_MERGE_CH && plain != 1) ? 3 : 4;
    const bool g2 = lowlat_path || (k->share_b && st_g2 == st && !(ZK_KNOCKOUT & 32));
    ProofStart ps = {};
    auto add = [&](void* buckets, size_t bytes, uint32_t* nnz, uint32_t* live) {
      ps.buckets[ps.n] = static_cast<uint4*>(buckets);
      ps.nvec[ps.n] = (uint32_t)(bytes / sizeof(uint4));
      ps.nnz[ps.n] = nnz;
      ps.live[ps.n] = live;
      ps.n++;
    };
    const size_t nb = msm_nb_of(k->msm_c);
    for (int i = 0; i < ng1; i++) add(s->g1t[i].buckets, nb * sizeof(G1P), s->g1t[i].nnz, s->g1t[i].live);
    if (g2) add(s->g2t.buckets, nb * sizeof(G2P), s->g2t.nnz, s->g2t.live);
    uint32_t* res3 = MSM_MERGE_CH && plain != 1 ? reinterpret_cast<uint32_t*>(s->res + 3) : nullptr;
    if (s->w_stage && d_w == s->w_stage) {  // graph replay (enqueue_proof): stage the witness here
      ps.w_src_host = reinterpret_cast<const uint64_t*>(s->pinned + W_PTR_OFF);
      ps.w_dst = reinterpret_cast<uint4*>(s->w_stage);
      ps.w_nvec = (uint32_t)((size_t)k->nVars * 32 / sizeof(uint4));
    }
    hipLaunchKernelGGL(k_proof_start, dim3(128, ps.n), dim3(256), 0, st, reinterpret_cast<const uint32_t*>(s->pinned + 256),
                       reinterpret_cast<uint32_t*>(s->d_rs), s->extra, plain == 1, res3, ps);
  }
  if (lowlat_path) {
    const int rc = enqueue_proof_lowlat(ctx, k, s, d_w);
    if (rc) return rc;
    prof->end(pp, st, 1.0);
    return ZKFL_OK;
  }
  const uint32_t* W = (const uint32_t*)d_w;
  const uint32_t* E = (const uint32_t*)s->extra;
  if (!graph) HIP_TRY(hipEventRecord(s->ev_ready, st), "event");
  MsmTail<FqOps>* tails[4] = {&s->g1t[0], &s->g1t[1], &s->g1t[2], &s->g1t[3]};
  // C + H as one MSM into tail 2 (res[2] = C' + H, res[3] = infinity); the parity hook (plain)
  // keeps them apart
  const bool merge = MSM_MERGE_CH && plain != 1;
  // the parity hook on merged bases: C = the C + H MSM over (witness, zero h), H = over (zero witness, h)
  const bool split_ch = MSM_MERGE_CH && plain == 1;
  if (split_ch && !k->dbg_zero) return fail(ZKFL_E_ARG, "parity hook: zeros not allocated");
  const uint32_t* Z = (const uint32_t*)k->dbg_zero;
  const int ntails = merge ? 3 : 4;
  // Stage order.  Every slot runs the same chain, so under load the slots move as a convoy: the
  // accumulations fill the GPU one at a time, and the slots that leave them together reach ABC +
  // NTT together -- the wave timeline (tools/wtrace.py) showed stretches of ~4 ms with no
  // accumulation resident at all.  Staggered (the default; ZKFL_STAGGER=0 turns it off): odd slots
  // run ABC + NTT before their witness-scalar MSMs instead of after, so their light phase falls
  // beside the others' heavy one (+2.3 %, 407.5 vs 398.6 proofs/s, 3 same-box alternations).
  static const int stagger = getenv("ZKFL_STAGGER") ? atoi(getenv("ZKFL_STAGGER")) : 1;
  const bool light_first = stagger && (s->index & 1) && !prof->serialize;
  // One stream (the default): B1's digit sort also serves B2 (same scalars, same index map), so
  // B2 runs right after B1 on the main stream, before C reuses the sort scratch.
  const bool share = k->share_b && st_g2 == st && !(ZK_KNOCKOUT & 32);
  // Small keys: the G2 tail joins the G1 tails' launches (msm_tails_joint) instead of running right
  // after B2 -- config 5 2,712 vs 2,385 proofs/s (3 same-box alternations); the metric key keeps the
  // separate tails (M 433 vs 439 and 431 vs 433 with them joint, two boxes:
  // profiles/r06_ab_joint_tails.log, r06_ab_front.log)
  const bool joint = share && k->front;
  if (!share) {  // G2 stream
    HIP_TRY(hipStreamWaitEvent(st_g2, s->ev_ready, 0), "wait");
    if (!(ZK_KNOCKOUT & 32))
      HIP_TRY(msm_run_g2(k->bB2, s->g2s, s->g2t, W, E, s->resB2, st_g2, prof, "msm_accumulate_g2"), "msm B2");
    HIP_TRY(hipEventRecord(s->ev_b2, st_g2), "event");
  }
  auto abc_ntt = [&]() { return enqueue_abc_ntt(k, s, d_w, st, prof); };
  // main: the witness-scalar G1 MSMs, then ABC / NTT / H, then all four G1 tails in one batch
#if ZK_KNOCKOUT & 2
  MsmScratch<FqOps>&sA = s->g1s_ko[0], &sB = s->g1s_ko[1], &sCH = s->g1s_ko[2];
#else
  MsmScratch<FqOps>&sA = s->g1s, &sB = s->g1s, &sCH = s->g1s;
#endif
  // small keys: ABC / NTT, then A, B1 and C + H sorted together and accumulated in one launch, B2
  // from B1's pairs (their proofs are chains of latency-bound launches: fewer links, shorter chain;
  // config 5 2,802 vs 2,748 proofs/s, 3 same-box alternations, profiles/r06_ab_front.log)
  const bool front = joint && merge && !(ZK_KNOCKOUT & 2) && s->g1s_a.keys_out && s->g1s_b.keys_out;
  if (front) {
    const int rc = abc_ntt();
    if (rc) return rc;
    const MsmBases<FqOps>* bs[3] = {&k->bA, &k->bB1, &k->bCH};
    MsmScratch<FqOps>* ss[3] = {&s->g1s_a, &s->g1s_b, &s->g1s};
    uint32_t* nn[3] = {s->g1t[0].nnz, s->g1t[1].nnz, s->g1t[2].nnz};
    const uint32_t* sc[3] = {W, W, W};
    const uint32_t* ex[3] = {E, E, (const uint32_t*)s->h};
    HIP_TRY(msm_sort_multi_g1(bs, ss, nn, sc, ex, 3, st), "msm A, B1, C+H sorts");
    const uint16_t* kk[3] = {ss[0]->keys_out, ss[1]->keys_out, ss[2]->keys_out};
    const uint32_t* vv[3] = {ss[0]->vals_out, ss[1]->vals_out, ss[2]->vals_out};
    HIP_TRY(msm_accumulate_sorted_multi_g1(bs, kk, vv, tails, 3, st), "msm A, B1, C+H");
    if (!s->nnz_alias)
      HIP_TRY(hipMemcpyAsync(s->g2t.nnz, s->g1t[1].nnz, sizeof(uint32_t), hipMemcpyDeviceToDevice, st), "nnz");
    HIP_TRY(msm_accumulate_sorted_g2(k->bB2, ss[1]->keys_out, ss[1]->vals_out, s->g2t, st, prof, "msm_accumulate_g2"),
            "msm B2");
  }
  if (light_first && !front) {
    const int rc = abc_ntt();
    if (rc) return rc;
  }
  if (!front) HIP_TRY(msm_accumulate_g1(k->bA, sA, s->g1t[0], W, E, st, prof, "msm_accumulate_g1"), "msm A");
  if (front) {
  } else if (share) {
    MsmTail<Fq2Ops>* t2 = &s->g2t;
    G2P* o2 = s->resB2;
    HIP_TRY(msm_sort_g1(k->bB1, sB, s->g1t[1].nnz, W, E, st), "msm B1 sort");
    HIP_TRY(msm_accumulate_sorted_g1(k->bB1, sB.keys_out, sB.vals_out, s->g1t[1], st, prof,
                                     "msm_accumulate_g1"), "msm B1");
    if (!s->nnz_alias)
      HIP_TRY(hipMemcpyAsync(s->g2t.nnz, s->g1t[1].nnz, sizeof(uint32_t), hipMemcpyDeviceToDevice, st), "nnz");
    HIP_TRY(msm_accumulate_sorted_g2(k->bB2, sB.keys_out, sB.vals_out, s->g2t, st, prof,
                                     "msm_accumulate_g2"), "msm B2");
    if (!joint) {
      HIP_TRY(msm_tails_g2(&t2, &o2, 1, st, small_key_fast_wsum(k)), "msm B2 tail");
      if (!graph) HIP_TRY(hipEventRecord(s->ev_b2, st), "event");
    }
  } else {
    HIP_TRY(msm_accumulate_g1(k->bB1, sB, s->g1t[1], W, E, st, prof, "msm_accumulate_g1"), "msm B1");
  }
  if (split_ch)
    HIP_TRY(msm_accumulate_g1(k->bCH, s->g1s, s->g1t[2], W, Z, st, prof, "msm_accumulate_g1"), "msm C");
  else if (!merge)
    HIP_TRY(msm_accumulate_g1(k->bC, s->g1s, s->g1t[2], W, E, st, prof, "msm_accumulate_g1"), "msm C");
  if (!light_first && !front) {
    const int rc = abc_ntt();
    if (rc) return rc;
  }
  if (front) {
  } else if (merge) {
    HIP_TRY(msm_accumulate_g1(k->bCH, sCH, s->g1t[2], W, (const uint32_t*)s->h, st, prof, "msm_accumulate_g1"),
            "msm C+H");
  } else if (split_ch) {
    HIP_TRY(msm_accumulate_g1(k->bCH, s->g1s, s->g1t[3], Z, (const uint32_t*)s->h, st, prof, "msm_accumulate_g1"),
            "msm H");
  } else {
    HIP_TRY(msm_accumulate_g1(k->bH, s->g1s, s->g1t[3], (const uint32_t*)s->h, nullptr, st, prof, "msm_accumulate_g1"),
            "msm H");
  }
  {
    G1P* outs[4] = {s->res + 0, s->res + 1, s->res + 2, s->res + 3};
    if (joint) {
      MsmTail<Fq2Ops>* t2 = &s->g2t;
      G2P* o2 = s->resB2;
      HIP_TRY(msm_tails_joint(tails, outs, ntails, &t2, &o2, 1, st, small_key_fast_wsum(k)), "msm tails (G1 + G2)");
    } else {
      HIP_TRY(msm_tails_g1(tails, outs, ntails, st, small_key_fast_wsum(k)), "msm tails");
    }
  }
  if (!graph && !joint) HIP_TRY(hipStreamWaitEvent(st, s->ev_b2, 0), "wait");
  if (plain == 2) {
    hipLaunchKernelGGL(k_part_out, dim3(1), dim3(64), 0, st, s->res, s->resB2, s->d_parts);
    HIP_TRY(hipMemcpyAsync(s->pinned + 512, s->d_parts, PART_WORDS * 4, hipMemcpyDeviceToHost, st), "download part");
  }
  if (!plain && !(ZK_KNOCKOUT & 1)) {
    const int pa = prof->begin("assemble", st);
    hipLaunchKernelGGL(k_assemble, dim3(1), dim3(ASM_THREADS), 0, st, s->res, s->resB2,
                       reinterpret_cast<const GlvScalar*>(reinterpret_cast<const uint8_t*>(s->d_rs) + 64),
                       proof_out(s));
    prof->end(pa, st, 1.0);
  }
  prof->end(pp, st, 1.0);
  return ZKFL_OK;
}

// Graph replay of the one-stream chain (the default; ZKFL_GRAPH=0 launches kernel by kernel;
// config 5 +3.5%, 1894 vs 1831 proofs/s, M +0.6% inside the spread, 3 same-box alternations,
// profiles/r04_ab_c5_small_keys.log, r04_ab_m_graph_target.log): a slot captures its proof's ~40 launches
// once per witness address (enqueue_proof passes the slot's witness stage, so once per slot) and
// then launches the graph -- one host call per proof instead of one per kernel.  Kernel arguments
// are the slot's own buffers, the key's and the witness address, all fixed per cache entry; r and s
// reach the device through the captured copy from the slot's pinned buffer.
int enqueue_proof_graph(zkfl_ctx* ctx, zkfl_key* k, ProofSlot* s, const Fr* d_w, int plain) {
  hipStream_t st = s->st_main;
  ProofSlot::Graph* gr = nullptr;
  for (auto& x : s->graphs)
    if (x.w == d_w) gr = &x;
  if (!gr) {
    if (s->graphs.size() >= 8) {  // bounded cache: drop the oldest
      ProofSlot::Graph& o = s->graphs.front();
      if (o.ex) (void)hipGraphExecDestroy(o.ex);
      if (o.g) (void)hipGraphDestroy(o.g);
      s->graphs.erase(s->graphs.begin());
    }
    ProofSlot::Graph ng;
    ng.w = d_w;
    HIP_TRY(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal), "begin capture");
    const int rc = enqueue_proof_body(ctx, k, s, d_w, plain, 0, true);
    const hipError_t ec = hipStreamEndCapture(st, &ng.g);
    if (rc) {
      if (ng.g) (void)hipGraphDestroy(ng.g);
      return rc;
    }
    HIP_TRY(ec, "end capture");
    const hipError_t ei = hipGraphInstantiate(&ng.ex, ng.g, nullptr, nullptr, 0);
    if (ei != hipSuccess) {
      (void)hipGraphDestroy(ng.g);
      return hip_fail(ei, "graph instantiate");
    }
    s->graphs.push_back(ng);
    gr = &s->graphs.back();
  }
  HIP_TRY(hipGraphLaunch(gr->ex, st), "graph launch");
  return ZKFL_OK;
}

int enqueue_proof(zkfl_ctx* ctx, zkfl_key* k, ProofSlot* s, const Fr* d_w, const uint32_t rs_host[16], int plain,
                  int lowlat = 0) {
  Profiler* prof = &ctx->prof;
  memcpy(s->pinned + 256, rs_host, 64);
  GlvScalar* ks = reinterpret_cast<GlvScalar*>(s->pinned + 320);
  glv_split(rs_host + 8, ks[0], ks[1]);  // s -> s1, s2 (for pi_A, phi(pi_A))
  glv_split(rs_host, ks[2], ks[3]);      // r -> r1, r2 (for B1, phi(B1))
  // graph replay from a slot's second proof on (a one-off proof pays no capture); the witness is
  // staged into the slot's own buffer so the captured kernel arguments hold for every witness
  const bool graph = graph_mode() && s->w_stage && !lowlat && plain == 0 && !prof->on && !prof->serialize &&
                     !s->st_g2 && k->share_b && !ZK_KNOCKOUT && s->direct_proofs > 0;
  int rc;
  if (graph) {
    // k_proof_start copies the witness into the stage from the address left here
    const uint64_t src = reinterpret_cast<uint64_t>(d_w);
    memcpy(s->pinned + W_PTR_OFF, &src, sizeof(src));
    rc = enqueue_proof_graph(ctx, k, s, s->w_stage, plain);
  } else {
    s->direct_proofs++;
    rc = enqueue_proof_body(ctx, k, s, d_w, plain, lowlat, false);
  }
  if (rc) return rc;
  HIP_TRY(hipEventRecord(s->ev_done, s->st_main), "event");
  HIP_TRY(hipGetLastError(), "launch");
  return ZKFL_OK;
}

// Host wait for a device event.  hipEventSynchronize on these (non-blocking-sync) events spins a
// host core for the whole wait: it was most of config 5's host CPU per proof (0.55-0.57 ms, 1.2
// cores busy at ~2,100 proofs/s).  A batch (poll = true) polls instead, sleeping ZKFL_WAIT_US
// (default 50) microseconds between queries: 0.13-0.16 ms per proof, 0.3 cores, throughput within
// the spread (2,091 vs 2,095 proofs/s, 3 same-box alternations, profiles/r05_ab_c5_fold_wait.log,
// which A/Bs the waits beside a since-removed fold knob);
// the scheduler refills a freed slot up to that much later, ~0.1% of an M step.  A proof alone (the
// latency path) keeps the spin.  ZKFL_WAIT_US=0 spins everywhere.
static hipError_t host_wait(hipEvent_t ev, bool poll) {
  static const int us = getenv("ZKFL_WAIT_US") ? atoi(getenv("ZKFL_WAIT_US")) : 50;
  if (us <= 0 || !poll) return hipEventSynchronize(ev);
  for (;;) {
    const hipError_t e = hipEventQuery(ev);
    if (e != hipErrorNotReady) return e;
    std::this_thread::sleep_for(std::chrono::microseconds(us));
  }
}

int wait_slot(ProofSlot* s, bool poll = false) {
  HIP_TRY(host_wait(s->ev_done, poll), "sync");
  if (s->out_proof) memcpy(s->out_proof, s->pinned, 256);
  if (s->out_part) memcpy(s->out_part, s->pinned + 512, PART_WORDS * 4);
  s->busy = false;
  return ZKFL_OK;
}

// One proof of a batch: a device-resident witness, complete once w_ready is (nullptr: already).
// Jobs of one batch may use different keys.
struct Job {
  zkfl_key* key = nullptr;
  const Fr* w = nullptr;
  hipEvent_t w_ready = nullptr;  // the witness group of the full-prove pipe (full_prove_piped)
  const uint8_t* rs = nullptr;  // 64 B or nullptr (CSPRNG)
  uint8_t* proof_out = nullptr;
  uint8_t* part_out = nullptr;  // split proof: this shard's part instead of a proof
};

// The batch scheduler behind every prove entry point: job i goes to the next slot of its key
// (round robin per key), a busy slot is drained first, so up to max_slots proofs per key are in
// flight and proofs of different keys (e.g. the training and secure-aggregation circuits of one
// federated round) overlap on the device.  job(i, Job&) fills the i-th job.
template <class GetJob>
int run_jobs(zkfl_ctx* ctx, size_t n, GetJob job) {
  HIP_TRY(hipSetDevice(ctx->device), "hipSetDevice");
  struct PerKey {
    zkfl_key* key;
    size_t issued = 0;  // proofs issued in this batch
  };
  std::vector<PerKey> cursor;
  // a batch of one proof runs the low-latency schedule (ZKFL_LOWLAT=0: the one-stream chain)
  static const int lowlat = getenv("ZKFL_LOWLAT") ? atoi(getenv("ZKFL_LOWLAT")) : 1;
  // A/B knob: ZKFL_LOWLAT_BATCH=1 runs every proof of a batch on the low-latency schedule
  static const bool lowlat_batch = getenv("ZKFL_LOWLAT_BATCH") && atoi(getenv("ZKFL_LOWLAT_BATCH")) != 0;
  auto issue = [&](PerKey& pk, size_t i, const Job& J, const uint32_t* rsl) -> int {
    ProofSlot* s = nullptr;
    int rc = get_slot(J.key, pk.issued++, &s);
    if (rc) return rc;
    if (s->busy) {
      rc = wait_slot(s, n > 1);
      if (rc) return rc;
    }
    s->job = i;
    s->out_proof = J.part_out ? nullptr : J.proof_out;
    s->out_part = J.part_out;
    if (J.w_ready) {
      hipError_t e = hipStreamWaitEvent(s->st_main, J.w_ready, 0);
      if (e != hipSuccess) return hip_fail(e, "wait for the witness group");
    }
    rc = enqueue_proof(ctx, J.key, s, J.w, rsl, J.part_out ? 2 : 0, (n == 1 || lowlat_batch) ? lowlat : 0);
    if (rc) return rc;
    s->busy = true;
    return ZKFL_OK;
  };
  int rc = ZKFL_OK;
  for (size_t i = 0; i < n && rc == ZKFL_OK; i++) {
    Job J;
    rc = job(i, J);
    if (rc) break;
    if (J.key->nshards != 1 && !J.part_out) {  // its MSMs are one shard's share: no whole proof
      rc = fail(ZKFL_E_ARG, "this key is shard " + std::to_string(J.key->shard) + " of " +
                                std::to_string(J.key->nshards) +
                                " of a split proof: prove parts (zkfl_groth16_prove_part_batch) and assemble them");
      break;
    }
    uint32_t rsl[16];
    rc = get_rs(J.rs, rsl);
    if (rc) break;
    size_t c = 0;
    while (c < cursor.size() && cursor[c].key != J.key) c++;
    if (c == cursor.size()) {
      cursor.emplace_back();
      cursor.back().key = J.key;
    }
    rc = issue(cursor[c], i, J, rsl);
  }
  for (auto& pk : cursor) {
    for (ProofSlot* s : pk.key->slots)
      if (s->busy) {
        int r2 = wait_slot(s, n > 1);
        if (rc == ZKFL_OK) rc = r2;
      }
  }
  return rc;
}

hipError_t msm_run_any(const MsmBases<FqOps>& b, MsmScratch<FqOps>& s, MsmTail<FqOps>& t, const uint32_t* sc,
                       G1P* o, hipStream_t st, Profiler* p) {
  return msm_run_g1(b, s, t, sc, nullptr, o, st, p, "msm_accumulate_g1");
}
hipError_t msm_run_any(const MsmBases<Fq2Ops>& b, MsmScratch<Fq2Ops>& s, MsmTail<Fq2Ops>& t, const uint32_t* sc,
                       G2P* o, hipStream_t st, Profiler* p) {
  return msm_run_g2(b, s, t, sc, nullptr, o, st, p, "msm_accumulate_g2");
}
hipError_t bases_alloc_any(MsmBases<FqOps>& b, size_t n, int c) { return msm_bases_alloc_g1(b, n, c); }
hipError_t bases_alloc_any(MsmBases<Fq2Ops>& b, size_t n, int c) { return msm_bases_alloc_g2(b, n, c); }
hipError_t bases_set_any(MsmBases<FqOps>& b, const G1Aff* src, hipStream_t st) {
  return msm_bases_set_g1(b, src, nullptr, 0xFFFFFFFFu, st);
}
hipError_t bases_set_any(MsmBases<Fq2Ops>& b, const G2Aff* src, hipStream_t st) {
  return msm_bases_set_g2(b, src, nullptr, 0xFFFFFFFFu, st);
}
hipError_t bases_set_map_any(MsmBases<FqOps>& b, const void* src, const uint32_t* hs, uint32_t x, hipStream_t st) {
  return msm_bases_set_g1(b, (const G1Aff*)src, hs, x, st);
}
hipError_t bases_set_map_any(MsmBases<Fq2Ops>& b, const void* src, const uint32_t* hs, uint32_t x, hipStream_t st) {
  return msm_bases_set_g2(b, (const G2Aff*)src, hs, x, st);
}
void bases_free_any(MsmBases<FqOps>& b) { msm_bases_free_g1(b); }
void bases_free_any(MsmBases<Fq2Ops>& b) { msm_bases_free_g2(b); }
hipError_t scratch_alloc_any(MsmScratch<FqOps>& s, size_t n, int c, hipStream_t st) {
  return msm_scratch_alloc_g1(s, n, c, st);
}
hipError_t scratch_alloc_any(MsmScratch<Fq2Ops>& s, size_t n, int c, hipStream_t st) {
  return msm_scratch_alloc_g2(s, n, c, st);
}
void scratch_free_any(MsmScratch<FqOps>& s) { msm_scratch_free_g1(s); }
void scratch_free_any(MsmScratch<Fq2Ops>& s) { msm_scratch_free_g2(s); }
hipError_t tail_alloc_any(MsmTail<FqOps>& t, size_t n, int c) { return msm_tail_alloc_g1(t, n, c); }
hipError_t tail_alloc_any(MsmTail<Fq2Ops>& t, size_t n, int c) { return msm_tail_alloc_g2(t, n, c); }
void tail_free_any(MsmTail<FqOps>& t) { msm_tail_free_g1(t); }
void tail_free_any(MsmTail<Fq2Ops>& t) { msm_tail_free_g2(t); }

template <class F>
int run_msm_primitive(zkfl_ctx* ctx, const uint8_t* bases, const uint8_t* scalars, size_t n, uint8_t* out) {
  if (!ctx || !bases || !scalars || !out || n == 0) return fail(ZKFL_E_ARG, "msm: bad args");
  hipStream_t st = ctx->st;
  MsmBases<F> mb;
  MsmScratch<F> ms;
  MsmTail<F> mt;
  Affine<F>* d_b = nullptr;
  uint32_t* d_s = nullptr;
  XYZZ<F>* d_r = nullptr;
  uint32_t* d_o = nullptr;
  int rc = ZKFL_OK;
  const int c = msm_pick_c(n);
  hipError_t e = bases_alloc_any(mb, n, c);
  if (e == hipSuccess) e = scratch_alloc_any(ms, n, c, st);
  if (e == hipSuccess) e = tail_alloc_any(mt, n, c);
  if (e == hipSuccess) e = hipMalloc(&d_b, n * sizeof(Affine<F>));
  if (e == hipSuccess) e = hipMalloc(&d_s, n * 32);
  if (e == hipSuccess) e = hipMalloc(&d_r, sizeof(XYZZ<F>));
  if (e == hipSuccess) e = hipMalloc(&d_o, sizeof(Affine<F>));
  if (e == hipSuccess) e = hipMemcpyAsync(d_b, bases, n * sizeof(Affine<F>), hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(d_s, scalars, n * 32, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = bases_set_any(mb, d_b, st);
  if (e == hipSuccess) e = msm_run_any(mb, ms, mt, d_s, d_r, st, &ctx->prof);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_point_out<F>, dim3(1), dim3(1), 0, st, d_r, 1, d_o);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(out, d_o, sizeof(Affine<F>), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) rc = hip_fail(e, "msm primitive");
  bases_free_any(mb);
  scratch_free_any(ms);
  tail_free_any(mt);
  for (void* p : {(void*)d_b, (void*)d_s, (void*)d_r, (void*)d_o})
    if (p) (void)hipFree(p);
  return rc;
}

template <class F>
int run_gen_mul(zkfl_ctx* ctx, const uint8_t* scalars, size_t n, uint8_t* out, bool g2) {
  if (!ctx || !scalars || !out) return fail(ZKFL_E_ARG, "gen_mul: bad args");
  if (n == 0) return ZKFL_OK;
  hipStream_t st = ctx->st;
  uint32_t* d_s = nullptr;
  Affine<F>* d_o = nullptr;
  Affine<F>* d_g = nullptr;
  int rc = ZKFL_OK;
  hipError_t e = hipMalloc(&d_s, n * 32);
  if (e == hipSuccess) e = hipMalloc(&d_o, n * sizeof(Affine<F>));
  if (e == hipSuccess) e = hipMalloc(&d_g, sizeof(Affine<F>));
  if (e == hipSuccess) e = hipMemcpyAsync(d_s, scalars, n * 32, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) {
    if (g2)
      hipLaunchKernelGGL(k_g2_gen_mont, dim3(1), dim3(1), 0, st, (G2Aff*)d_g);
    else
      hipLaunchKernelGGL(k_g1_gen_mont, dim3(1), dim3(1), 0, st, (G1Aff*)d_g);
    e = hipGetLastError();
  }
  Affine<F> g;
  if (e == hipSuccess) e = hipMemcpyAsync(&g, d_g, sizeof(g), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_gen_mul<F>, dim3(zk_grid(n, 64)), dim3(64), 0, st, d_s, n, g, d_o);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(out, d_o, n * sizeof(Affine<F>), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) rc = hip_fail(e, "gen_mul");
  for (void* p : {(void*)d_s, (void*)d_o, (void*)d_g})
    if (p) (void)hipFree(p);
  return rc;
}

}  // namespace

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
namespace {

int pos_ready(zkfl_ctx* ctx) {
  if (ctx->pos) return ZKFL_OK;
  std::string err;
  int rc = pos_tables_create(&ctx->pos, ctx->st, err);
  return rc ? fail(rc, err) : ZKFL_OK;
}

int check_fr_array(const uint8_t* v, size_t count, const char* what) {
  for (size_t i = 0; i < count; i++) {
    uint32_t w[8];
    memcpy(w, v + 32 * i, 32);
    if (!lt_r(w)) return fail(ZKFL_E_ARG, std::string(what) + " " + std::to_string(i) + " is not < r");
  }
  return ZKFL_OK;
}

// device scratch of one hashing call, freed on every exit path
struct DevBufs {
  std::vector<void*> p;
  ~DevBufs() {
    for (void* q : p) (void)hipFree(q);
  }
  hipError_t get(void** out, size_t bytes) {
    *out = nullptr;
    hipError_t e = hipMalloc(out, bytes ? bytes : 32);
    if (e == hipSuccess) p.push_back(*out);
    return e;
  }
};


// leaves (device, Montgomery) -> full padded tree (host, std)
int tree_from_device_leaves(zkfl_ctx* ctx, DevBufs& B, const Fr* d_leaves, size_t n, uint32_t depth,
                            uint8_t* tree_out) {
  hipStream_t st = ctx->st;
  const size_t nodes = ((size_t)2 << depth) - 1;
  Fr *d_work, *d_tree;
  HIP_TRY(B.get((void**)&d_work, merkle_work_size(n, depth) * 32), "alloc");
  HIP_TRY(B.get((void**)&d_tree, nodes * 32), "alloc");
  int pi = ctx->prof.begin("merkle", st);
  HIP_TRY(merkle_build(ctx->pos, d_leaves, n, depth, d_tree, d_work, st), "merkle");
  ctx->prof.end(pi, st, (double)(merkle_work_size(n, depth) - n));
  HIP_TRY(hipMemcpyAsync(tree_out, d_tree, nodes * 32, hipMemcpyDeviceToHost, st), "download");
  HIP_TRY(hipStreamSynchronize(st), "sync");
  return ZKFL_OK;
}

int tree_args(zkfl_ctx* ctx, size_t n, uint32_t depth, const void* in, const void* out) {
  if (!ctx || !out || (n && !in)) return fail(ZKFL_E_ARG, "merkle: null argument");
  if (depth > ZKFL_MERKLE_MAX_DEPTH) return fail(ZKFL_E_ARG, "merkle: depth must be <= 30");
  if (n > ((size_t)1 << depth)) return fail(ZKFL_E_ARG, "merkle: more leaves than 2^depth");
  return ZKFL_OK;
}

}  // namespace

extern "C" {

int zkfl_version(void) { return 1; }

int zkfl_debug_glv_split(const uint8_t k[32], uint8_t out[40]) {
  if (!k || !out) return fail(ZKFL_E_ARG, "null argument");
  uint32_t kk[8];
  memcpy(kk, k, 32);
  if (!lt_r(kk)) return fail(ZKFL_E_ARG, "k must be < r");
  GlvScalar a, b;
  glv_split(kk, a, b);
  memcpy(out, a.mag, 16);
  memcpy(out + 16, &a.neg, 4);
  memcpy(out + 20, b.mag, 16);
  memcpy(out + 36, &b.neg, 4);
  return ZKFL_OK;
}

int zkfl_debug_g1_glv_mul(zkfl_ctx* ctx, size_t n, const uint8_t* points, const uint8_t* scalars, uint8_t* out) {
  if (!ctx || (n && (!points || !scalars || !out))) return fail(ZKFL_E_ARG, "null argument");
  if (n == 0) return ZKFL_OK;
  if (n > (1u << 20)) return fail(ZKFL_E_ARG, "glv mul: n too large");
  std::vector<GlvScalar> ks(2 * n);
  for (size_t i = 0; i < n; i++) {
    uint32_t kk[8];
    memcpy(kk, scalars + 32 * i, 32);
    if (!lt_r(kk)) return fail(ZKFL_E_ARG, "glv mul: scalar " + std::to_string(i) + " is not < r");
    glv_split(kk, ks[2 * i], ks[2 * i + 1]);
  }
  HIP_TRY(hipSetDevice(ctx->device), "hipSetDevice");
  hipStream_t st = ctx->st;
  uint8_t *d_p = nullptr, *d_k = nullptr, *d_o = nullptr;
  int rc = ZKFL_OK;
  hipError_t e = hipMalloc(&d_p, n * 64);
  if (e == hipSuccess) e = hipMalloc(&d_k, ks.size() * sizeof(GlvScalar));
  if (e == hipSuccess) e = hipMalloc(&d_o, n * 64);
  if (e == hipSuccess) e = hipMemcpyAsync(d_p, points, n * 64, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(d_k, ks.data(), ks.size() * sizeof(GlvScalar), hipMemcpyHostToDevice, st);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_debug_glv_mul, dim3((uint32_t)n), dim3(128), 0, st, (const uint32_t*)d_p,
                       (const GlvScalar*)d_k, (uint32_t*)d_o);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(out, d_o, n * 64, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) rc = hip_fail(e, "glv mul");
  for (void* q : {(void*)d_p, (void*)d_k, (void*)d_o})
    if (q) (void)hipFree(q);
  return rc;
}

const char* zkfl_last_error(void) { return g_err.c_str(); }

int zkfl_device_count(int* count) {
  if (!count) return fail(ZKFL_E_ARG, "null");
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) {
    *count = 0;
    return hip_fail(e, "hipGetDeviceCount");
  }
  *count = c;
  return ZKFL_OK;
}

int zkfl_ctx_create(int device, zkfl_ctx** out) {
  if (!out) return fail(ZKFL_E_ARG, "null out");
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess || c == 0) return fail(ZKFL_E_DEVICE, "no HIP device available");
  if (device < 0 || device >= c) return fail(ZKFL_E_ARG, "device index out of range");
  HIP_TRY(hipSetDevice(device), "hipSetDevice");
  zkfl_ctx* ctx = new zkfl_ctx();
  ctx->device = device;
  hipError_t e = hipStreamCreateWithFlags(&ctx->st, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete ctx;
    return hip_fail(e, "hipStreamCreate");
  }
  *out = ctx;
  return ZKFL_OK;
}

static void ctx_retain(zkfl_ctx* ctx) { ctx->refs.fetch_add(1, std::memory_order_relaxed); }

// Drops one reference; the last one tears the context down.
static void ctx_release(zkfl_ctx* ctx) {
  if (ctx->refs.fetch_sub(1, std::memory_order_acq_rel) != 1) return;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->st);
  ctx->prof.reset();
  vk_free(ctx->vk);
  pos_tables_free(ctx->pos);
  if (ctx->asm_buf) (void)hipFree(ctx->asm_buf);
  if (ctx->wt.rec) {  // a wave trace still bound: unbind before its buffer goes
    (void)zkfl_debug_wtrace(ctx, 0, 0, nullptr, nullptr);
  }
  (void)hipStreamDestroy(ctx->st);
  delete ctx;
}

// The caller's handle: after this call the handle is gone, but keys and witness programs still
// alive keep the device state until they are freed.
int zkfl_ctx_destroy(zkfl_ctx* ctx) {
  if (!ctx) return ZKFL_OK;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->st);
  ctx_release(ctx);
  return ZKFL_OK;
}

int zkfl_ctx_set_profiling(zkfl_ctx* ctx, int enabled) {
  if (!ctx) return fail(ZKFL_E_ARG, "null ctx");
  ctx->prof.on = enabled != 0;
  ctx->prof.serialize = enabled == 2;
  return ZKFL_OK;
}

int zkfl_ctx_profile(zkfl_ctx* ctx, const char* name, double* total_ms, uint64_t* launches, double* units,
                     double* median_ms) {
  if (!ctx || !name || !total_ms || !launches) return fail(ZKFL_E_ARG, "null");
  (void)hipSetDevice(ctx->device);
  HIP_TRY(hipDeviceSynchronize(), "sync");
  ctx->prof.query(name, total_ms, launches, units, median_ms);
  return ZKFL_OK;
}

int zkfl_ctx_profile_reset(zkfl_ctx* ctx) {
  if (!ctx) return fail(ZKFL_E_ARG, "null ctx");
  (void)hipStreamSynchronize(ctx->st);
  ctx->prof.reset();
  return ZKFL_OK;
}

int zkfl_ctx_synchronize(zkfl_ctx* ctx) {
  if (!ctx) return fail(ZKFL_E_ARG, "null ctx");
  HIP_TRY(hipSetDevice(ctx->device), "hipSetDevice");
  HIP_TRY(hipDeviceSynchronize(), "sync");  // every stream of this process: the proof slots' too
  return ZKFL_OK;
}

namespace {
// Make a parsed key device-resident.  z's pointers address the key bytes (len of them), which
// stay valid for the call; parse_ms: the parse's duration for the load timing.
int zkey_load_parsed(zkfl_ctx* ctx, const ZkeyHost& z, size_t len, double parse_ms, uint32_t shard, uint32_t nshards,
                     zkfl_key** out) {
  if (!ctx || !out) return fail(ZKFL_E_ARG, "null argument");
  if (nshards < 1 || nshards > 1024 || shard >= nshards) return fail(ZKFL_E_ARG, "shard must be < n_shards <= 1024");
  // ZKFL_LOAD_TIMING=<file>: one JSON line per load with the host-side stages (bench.py cli_prove)
  const char* timing_path = getenv("ZKFL_LOAD_TIMING");
  std::vector<std::pair<std::string, double>> marks;
  auto t_last = std::chrono::steady_clock::now();
  auto mark = [&](const char* what) {
    if (!timing_path) return;
    const auto t = std::chrono::steady_clock::now();
    marks.emplace_back(what, std::chrono::duration<double, std::milli>(t - t_last).count());
    t_last = t;
  };
  if (timing_path) marks.emplace_back("parse", parse_ms);
  const uint32_t nVars = z.nVars, nPub = z.nPub, dom = z.dom;
  const int logn = z.logn;
  const size_t nC = z.nC;
  const size_t ncoef = z.ncoef;
  const uint32_t cshift = z.cshift;
  const std::vector<uint32_t>& rowptr = z.rowptr;
  const std::vector<uint32_t>& cols = z.cols;
  const std::vector<uint32_t>& coefs = z.coefs;
  const uint8_t* pts = z.pts;
  HIP_TRY(hipSetDevice(ctx->device), "hipSetDevice");
  hipStream_t st = ctx->st;
  zkfl_key* k = new zkfl_key();
  k->ctx = ctx;
  ctx_retain(ctx);  // dropped by key_release
  k->nVars = nVars;
  k->nPub = nPub;
  k->n = dom;
  k->logn = logn;
  k->nC = nC;
  k->K = ncoef;
  k->shard = shard;
  k->nshards = nshards;
  auto cleanup = [&](int code) {
    key_release(k);
    return code;
  };
#define KTRY(x, where)                                  \
  do {                                                  \
    hipError_t _e = (x);                                \
    if (_e != hipSuccess) return cleanup(hip_fail(_e, where)); \
  } while (0)
  KTRY(hipMalloc(&k->rows, (2 * (size_t)dom + 1) * 4), "alloc rows");
  KTRY(hipMalloc(&k->cols, (size_t)(ncoef ? ncoef : 1) * 4), "alloc cols");
  k->cshift = cshift;
  const size_t ncoefs_dev = coefs.size() / 8;
  KTRY(hipMalloc(&k->coefs, (ncoefs_dev ? ncoefs_dev : 1) * 32), "alloc coefs");
  // combined row pointers: A rows [0, dom), B rows [dom, 2 dom) over one term array (rowA[dom] == rowB[0])
  KTRY(hipMemcpyAsync(k->rows, rowptr.data(), (size_t)dom * 4, hipMemcpyHostToDevice, st), "upload");
  KTRY(hipMemcpyAsync(k->rows + dom, rowptr.data() + dom + 1, ((size_t)dom + 1) * 4, hipMemcpyHostToDevice, st),
       "upload");
  if (ncoef) {
    KTRY(hipMemcpyAsync(k->cols, cols.data(), (size_t)ncoef * 4, hipMemcpyHostToDevice, st), "upload");
    KTRY(hipMemcpyAsync(k->coefs, coefs.data(), ncoefs_dev * 32, hipMemcpyHostToDevice, st), "upload");
  }
  if (timing_path) KTRY(hipStreamSynchronize(st), "sync");
  mark("qap_upload");
  // MSM bases: infinity points dropped (e.g. ~1/3 of B1/B2 for Poseidon-heavy circuits: x^4
  // wires never appear in B), plus augmentation slots alpha1/delta1 (A), beta1/delta1 (B1),
  // beta2/delta2 (B2), delta1 (C) whose scalars are the proof's extra = [1, r, s, -rs]
  // (index map: extra_start = nVars).
  {
    const uint8_t* alpha1 = pts;
    const uint8_t* beta1 = pts + 64;
    const uint8_t* beta2 = pts + 128;
    const uint8_t* delta1 = pts + 384;
    const uint8_t* delta2 = pts + 448;
    const uint32_t X = nVars;  // extra_start
    auto nonzero = [](const uint8_t* p, size_t len) {
      for (size_t i = 0; i < len; i++)
        if (p[i]) return true;
      return false;
    };
    struct Aug {
      const uint8_t* pt;
      uint32_t sidx;
    };
    // this shard's share of a query: element i when i % nshards == shard; the augmentation
    // bases once, on shard 0
    auto mine = [&](size_t i) { return nshards == 1 || i % nshards == shard; };
    const bool aug_here = shard == 0;
    // H with one shard keeps every point and no index map (scalar j = h[j]); sharded, it is
    // compacted like the others, its map indexing h directly (no extra slots)
    const bool h_identity = nshards == 1;
    // The compacted (host) base images + index maps of every query are built on host threads at
    // once (they only read the key bytes), then uploaded and expanded back to back on the stream
    // with one synchronisation at the end (the images stay alive until then).
    struct Img {
      std::vector<uint8_t> img;
      std::vector<uint32_t> sidx;
    };
    auto image = [&](Img& o, size_t psz, const uint8_t* sec, size_t cnt, uint32_t scalar_off,
                     std::vector<Aug> aug, bool identity) {
      size_t kept = 0;
      for (size_t i = 0; i < cnt; i++) kept += mine(i) && (identity || nonzero(sec + i * psz, psz));
      o.img.resize((kept + aug.size()) * psz);
      o.sidx.reserve(kept + aug.size());
      uint8_t* w = o.img.data();
      for (size_t i = 0; i < cnt; i++) {
        const uint8_t* p = sec + i * psz;
        if (!mine(i) || (!identity && !nonzero(p, psz))) continue;
        memcpy(w, p, psz);
        w += psz;
        o.sidx.push_back(scalar_off + (uint32_t)i);
      }
      if (aug_here)
        for (const Aug& x : aug) {
          memcpy(w, x.pt, psz);
          w += psz;
          o.sidx.push_back(x.sidx);
        }
      o.img.resize((size_t)(w - o.img.data()));
    };
    // C (private wires -> the witness) then H (h_j -> extra[j], the slot's h vector), then delta1
    // with -rs (extra[dom + 3]: the extra slots sit behind h)
    auto image_ch = [&](Img& o) {
      Img c, h;
      image(c, 64, z.secC, nC, nPub + 1, {}, false);
      image(h, 64, z.secH, dom, X, {{delta1, (uint32_t)(X + dom + 3)}}, false);
      o.img.swap(c.img);
      o.img.insert(o.img.end(), h.img.begin(), h.img.end());
      o.sidx.swap(c.sidx);
      o.sidx.insert(o.sidx.end(), h.sidx.begin(), h.sidx.end());
    };
    enum { QA, QB1, QB2, QC, QH, QCH, NQ };
    std::vector<Img> im(NQ);
    {
      std::vector<std::thread> th;
      th.emplace_back([&] { image(im[QA], 64, z.secA, nVars, 0, {{alpha1, X + 0}, {delta1, X + 1}}, false); });
      th.emplace_back([&] { image(im[QB1], 64, z.secB1, nVars, 0, {{beta1, X + 0}, {delta1, X + 2}}, false); });
      th.emplace_back([&] { image(im[QB2], 128, z.secB2, nVars, 0, {{beta2, X + 0}, {delta2, X + 2}}, false); });
      if (MSM_MERGE_CH) {
        th.emplace_back([&] { image_ch(im[QCH]); });
      } else {
        th.emplace_back([&] { image(im[QC], 64, z.secC, nC, nPub + 1, {{delta1, X + 3}}, false); });
        // aug.size() == 0 (H): no extra slots, the map indexes the main scalars only
        th.emplace_back([&] { image(im[QH], 64, z.secH, dom, 0, {}, h_identity); });
      }
      for (auto& t : th) t.join();
    }
    mark("bases_host");
    size_t most = 0;
    for (const Img& o : im) most = std::max(most, o.sidx.size());
    k->msm_c = msm_pick_c(most);
    std::vector<void*> d_imgs;
    auto upload = [&](auto& mb, Img& o, bool identity, uint32_t xs) -> hipError_t {
      hipError_t e = bases_alloc_any(mb, o.sidx.size(), k->msm_c);
      if (e != hipSuccess || o.sidx.empty()) return e;
      void* d_img = nullptr;
      e = hipMalloc(&d_img, o.img.size());
      if (e != hipSuccess) return e;
      d_imgs.push_back(d_img);
      e = hipMemcpyAsync(d_img, o.img.data(), o.img.size(), hipMemcpyHostToDevice, st);
      if (e == hipSuccess) e = bases_set_map_any(mb, d_img, identity ? nullptr : o.sidx.data(), xs, st);
      return e;
    };
    hipError_t e = upload(k->bA, im[QA], false, X);
    if (e == hipSuccess) e = upload(k->bB1, im[QB1], false, X);
    if (e == hipSuccess) e = upload(k->bB2, im[QB2], false, X);
    // B_i(tau) G1 and B_i(tau) G2 vanish together in an honest zkey; the sort is shared only when
    // the two index maps really are equal
    k->share_b = !ZK_NO_SHARE_B && im[QB1].sidx == im[QB2].sidx && !im[QB1].sidx.empty();
    k->front = MSM_MERGE_CH && k->share_b && nshards == 1 && logn <= 16;
    if (e == hipSuccess && MSM_MERGE_CH) e = upload(k->bCH, im[QCH], false, X);
    if (e == hipSuccess && !MSM_MERGE_CH) e = upload(k->bC, im[QC], false, X);
    if (e == hipSuccess && !MSM_MERGE_CH) e = upload(k->bH, im[QH], h_identity, 0xFFFFFFFFu);
    const hipError_t es = hipStreamSynchronize(st);
    if (e == hipSuccess) e = es;
    for (void* d : d_imgs) (void)hipFree(d);
    mark("bases_upload");
    if (e != hipSuccess) return cleanup(hip_fail(e, "base expansion"));
  }
  KTRY(ntt_plan_alloc(k->ntt, logn, st), "ntt plan");
  if (timing_path) KTRY(hipStreamSynchronize(st), "sync");
  mark("ntt_plan");
  {
    ProofSlot* s0 = nullptr;
    int rc0 = get_slot(k, 0, &s0);  // first slot eagerly: surfaces OOM at load time
    if (rc0) return cleanup(rc0);
  }
  KTRY(hipStreamSynchronize(st), "sync");
  mark("first_slot");
  if (timing_path) {
    if (FILE* f = fopen(timing_path, "a")) {
      double total = 0;
      fprintf(f, "{\"bytes\": %zu", len);
      for (auto& m : marks) {
        fprintf(f, ", \"%s_ms\": %.3f", m.first.c_str(), m.second);
        total += m.second;
      }
      fprintf(f, ", \"total_ms\": %.3f}\n", total);
      fclose(f);
    }
  }
#undef KTRY
  *out = k;
  return ZKFL_OK;
}

int zkey_load_impl(zkfl_ctx* ctx, const uint8_t* buf, size_t len, uint32_t shard, uint32_t nshards,
                   zkfl_key** out) {
  if (!ctx || !buf || !out) return fail(ZKFL_E_ARG, "null argument");
  if (nshards < 1 || nshards > 1024 || shard >= nshards) return fail(ZKFL_E_ARG, "shard must be < n_shards <= 1024");
  const auto t0 = std::chrono::steady_clock::now();
  ZkeyHost z;
  std::string err;
  const int rc = zkey_parse(buf, len, z, err);  // csrc/host_parse.cc: header, sections, CSR + dictionary
  if (rc) return fail(rc, err);
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return zkey_load_parsed(ctx, z, len, ms, shard, nshards, out);
}
}  // namespace

struct zkfl_zkey_file {
  int fd = -1;
  void* map = nullptr;
  size_t len = 0;
  ZkeyHost z;
  double parse_ms = 0;
};

int zkfl_zkey_load(zkfl_ctx* ctx, const uint8_t* buf, size_t len, zkfl_key** out) {
  return zkey_load_impl(ctx, buf, len, 0, 1, out);
}

int zkfl_zkey_file_open(const char* path, zkfl_zkey_file** out) {
  if (!path || !out) return fail(ZKFL_E_ARG, "null argument");
  *out = nullptr;
  const auto t0 = std::chrono::steady_clock::now();
  zkfl_zkey_file* f = new zkfl_zkey_file();
  f->fd = open(path, O_RDONLY | O_CLOEXEC);
  struct stat stt;
  if (f->fd < 0 || fstat(f->fd, &stt) != 0) {
    zkfl_zkey_file_close(f);
    return fail(ZKFL_E_ARG, std::string("cannot open ") + path);
  }
  f->len = (size_t)stt.st_size;
  if (f->len) {
    f->map = mmap(nullptr, f->len, PROT_READ, MAP_PRIVATE, f->fd, 0);
    if (f->map == MAP_FAILED) {
      f->map = nullptr;
      zkfl_zkey_file_close(f);
      return fail(ZKFL_E_ARG, std::string("cannot map ") + path);
    }
    (void)madvise(f->map, f->len, MADV_WILLNEED);
  }
  std::string err;
  const int rc = zkey_parse(static_cast<const uint8_t*>(f->map), f->len, f->z, err);
  if (rc) {
    zkfl_zkey_file_close(f);
    return fail(rc, err);
  }
  f->parse_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  *out = f;
  return ZKFL_OK;
}

int zkfl_zkey_load_file(zkfl_ctx* ctx, const zkfl_zkey_file* f, zkfl_key** out) {
  if (!f) return fail(ZKFL_E_ARG, "null argument");
  return zkey_load_parsed(ctx, f->z, f->len, f->parse_ms, 0, 1, out);
}

int zkfl_zkey_file_close(zkfl_zkey_file* f) {
  if (!f) return ZKFL_OK;
  if (f->map) munmap(f->map, f->len);
  if (f->fd >= 0) close(f->fd);
  delete f;
  return ZKFL_OK;
}

int zkfl_zkey_load_shard(zkfl_ctx* ctx, const uint8_t* buf, size_t len, uint32_t shard, uint32_t n_shards,
                         zkfl_key** out) {
  return zkey_load_impl(ctx, buf, len, shard, n_shards, out);
}

int zkfl_key_free(zkfl_key* key) {
  if (!key) return ZKFL_OK;
  (void)hipSetDevice(key->ctx->device);
  (void)hipStreamSynchronize(key->ctx->st);
  key_release(key);
  return ZKFL_OK;
}

int zkfl_key_info(const zkfl_key* key, uint32_t* n_vars, uint32_t* n_public, uint32_t* domain_size) {
  if (!key) return fail(ZKFL_E_ARG, "null key");
  if (n_vars) *n_vars = key->nVars;
  if (n_public) *n_public = key->nPub;
  if (domain_size) *domain_size = key->n;
  return ZKFL_OK;
}

int zkfl_witness_upload(zkfl_ctx* ctx, const zkfl_key* key, const uint8_t* wtns, size_t wtns_len,
                        zkfl_witness** out) {
  if (!ctx || !key || !wtns || !out) return fail(ZKFL_E_ARG, "null argument");
  WtnsView v;
  int rc = parse_wtns(wtns, wtns_len, v);
  if (rc) return rc;
  if (v.n != key->nVars) return fail(ZKFL_E_MISMATCH, "wtns: nWitness != zkey nVars");
  HIP_TRY(hipSetDevice(ctx->device), "hipSetDevice");
  zkfl_witness* w = new zkfl_witness();
  w->key = key;
  hipError_t e = hipMalloc(&w->d, (size_t)v.n * 32);
  if (e == hipSuccess) e = hipMemcpyAsync(w->d, v.data, (size_t)v.n * 32, hipMemcpyHostToDevice, ctx->st);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->st);
  if (e != hipSuccess) {
    if (w->d) (void)hipFree(w->d);
    delete w;
    return hip_fail(e, "witness upload");
  }
  w->pub.assign(v.data + 32, v.data + 32 + (size_t)key->nPub * 32);
  *out = w;
  return ZKFL_OK;
}

int zkfl_witness_free(zkfl_witness* w) {
  if (!w) return ZKFL_OK;
  if (w->d) (void)hipFree(w->d);
  delete w;
  return ZKFL_OK;
}

int zkfl_groth16_prove_resident(zkfl_ctx* ctx, zkfl_key* key, const zkfl_witness* w, const uint8_t* rs,
                                uint8_t proof_out[256]) {
  return zkfl_groth16_prove_batch(ctx, key, 1, &w, rs, proof_out);
}

int zkfl_key_set_slots(zkfl_key* key, int slots) {
  if (!key || slots < 1 || slots > 32) return fail(ZKFL_E_ARG, "slots must be in 1..32");
  (void)hipSetDevice(key->ctx->device);
  for (ProofSlot* s : key->slots) {
    if (s->busy) return fail(ZKFL_E_ARG, "slots busy");
  }
  while ((int)key->slots.size() > slots) {
    slot_release(key->slots.back());
    key->slots.pop_back();
  }
  // a slot's latency-schedule streams (made by a batch of one) hold HW queues: with many slots
  // they would push the slots' own streams past the ~24 HW queues and make slots share them
  // (a latency pass on a one-slot key before a 20-slot run: 395 vs 415 proofs/s)
  if (slots > 1)
    for (ProofSlot* s : key->slots) slot_drop_lowlat(s);
  key->max_slots = slots;
  return ZKFL_OK;
}

int zkfl_groth16_prove_batch(zkfl_ctx* ctx, zkfl_key* key, size_t n, const zkfl_witness* const* w,
                             const uint8_t* rs, uint8_t* proofs_out) {
  if (!ctx || !key || (!w && n) || (!proofs_out && n)) return fail(ZKFL_E_ARG, "null argument");
  for (size_t i = 0; i < n; i++) {
    if (!w[i] || w[i]->key != key) return fail(ZKFL_E_MISMATCH, "witness uploaded for another key");
  }
  return run_jobs(ctx, n, [&](size_t i, Job& J) {
    J.key = key;
    J.w = w[i]->d;
    J.rs = rs ? rs + 64 * i : nullptr;
    J.proof_out = proofs_out + 256 * i;
    return ZKFL_OK;
  });
}

int zkfl_key_shard(const zkfl_key* key, uint32_t* shard, uint32_t* n_shards) {
  if (!key) return fail(ZKFL_E_ARG, "null key");
  if (shard) *shard = key->shard;
  if (n_shards) *n_shards = key->nshards;
  return ZKFL_OK;
}

int zkfl_groth16_prove_part_batch(zkfl_ctx* ctx, zkfl_key* key, size_t n, const zkfl_witness* const* w,
                                  const uint8_t* rs, uint8_t* parts_out) {
  if (!ctx || !key || (n && (!w || !rs || !parts_out))) return fail(ZKFL_E_ARG, "prove_part: null argument");
  for (size_t i = 0; i < n; i++) {
    if (!w[i] || w[i]->key != key) return fail(ZKFL_E_MISMATCH, "witness uploaded for another key");
  }
  return run_jobs(ctx, n, [&](size_t i, Job& J) {
    J.key = key;
    J.w = w[i]->d;
    J.rs = rs + 64 * i;
    J.part_out = parts_out + PART_WORDS * 4 * i;
    return ZKFL_OK;
  });
}

int zkfl_groth16_assemble(zkfl_ctx* ctx, size_t n, size_t n_parts, const uint8_t* parts, const uint8_t* rs,
                          uint8_t* proofs_out) {
  if (!ctx || (n && (!parts || !rs || !proofs_out)) || n_parts < 1 || n_parts > 1024)
    return fail(ZKFL_E_ARG, "assemble: bad arguments");
  if (n == 0) return ZKFL_OK;
  // every coordinate canonical (< q): the parts cross a process boundary
  for (size_t i = 0; i < n * n_parts * (PART_WORDS / 8); i++)
    if (!lt_q(reinterpret_cast<const uint32_t*>(parts + 32 * i)))
      return fail(ZKFL_E_ARG, "assemble: part coordinate " + std::to_string(i) + " is not < q");
  std::vector<uint8_t> ks(n * 4 * sizeof(GlvScalar));
  for (size_t i = 0; i < n; i++) {
    uint32_t rsl[16];
    int rc = get_rs(rs + 64 * i, rsl);
    if (rc) return rc;
    GlvScalar* k = reinterpret_cast<GlvScalar*>(ks.data()) + 4 * i;
    glv_split(rsl + 8, k[0], k[1]);  // s -> pi_A's multiplier
    glv_split(rsl, k[2], k[3]);      // r -> B1's multiplier
  }
  HIP_TRY(hipSetDevice(ctx->device), "hipSetDevice");
  hipStream_t st = ctx->st;
  // one device buffer, carved: parts | res (5 G1P per proof) | resB2 | GLV halves | proofs | bad flag
  auto up = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t o_res = up(n * n_parts * PART_WORDS * 4), o_b2 = o_res + up(n * 5 * sizeof(G1P)),
               o_ks = o_b2 + up(n * sizeof(G2P)), o_pf = o_ks + up(ks.size()), o_bad = o_pf + up(n * 256),
               total = o_bad + 4;
  if (total > ctx->asm_cap) {
    if (ctx->asm_buf) (void)hipFree(ctx->asm_buf);
    ctx->asm_buf = nullptr;
    ctx->asm_cap = 0;
    HIP_TRY(hipMalloc(&ctx->asm_buf, total), "assemble buffers");
    ctx->asm_cap = total;
  }
  uint8_t* base = static_cast<uint8_t*>(ctx->asm_buf);
  void *d_parts = base, *d_res = base + o_res, *d_b2 = base + o_b2, *d_ks = base + o_ks, *d_proof = base + o_pf;
  uint32_t* d_bad = reinterpret_cast<uint32_t*>(base + o_bad);
  uint32_t bad = 0;
  hipError_t e = hipMemcpyAsync(d_parts, parts, n * n_parts * PART_WORDS * 4, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(d_ks, ks.data(), ks.size(), hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemsetAsync(d_bad, 0, 4, st);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_parts_sum, dim3((uint32_t)n), dim3(64), 0, st, (const uint32_t*)d_parts, (int)n_parts,
                       (G1P*)d_res, (G2P*)d_b2, d_bad);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(&bad, d_bad, 4, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return hip_fail(e, "assemble");
  if (bad) return fail(ZKFL_E_ARG, "assemble: a part holds a point that is not on its curve");
  hipLaunchKernelGGL(k_assemble, dim3((uint32_t)n), dim3(ASM_THREADS), 0, st, (const G1P*)d_res, (const G2P*)d_b2,
                     (const GlvScalar*)d_ks, (uint32_t*)d_proof);
  e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpyAsync(proofs_out, d_proof, n * 256, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return hip_fail(e, "assemble");
  return ZKFL_OK;
}

int zkfl_groth16_prove_multi(zkfl_ctx* ctx, size_t n, zkfl_key* const* keys, const zkfl_witness* const* w,
                             const uint8_t* rs, uint8_t* proofs_out) {
  if (!ctx || (n && (!keys || !w || !proofs_out))) return fail(ZKFL_E_ARG, "prove_multi: null argument");
  for (size_t i = 0; i < n; i++) {
    if (!keys[i] || keys[i]->ctx != ctx) return fail(ZKFL_E_ARG, "prove_multi: key of another context");
    if (!w[i] || w[i]->key != keys[i]) return fail(ZKFL_E_MISMATCH, "prove_multi: witness uploaded for another key");
  }
  return run_jobs(ctx, n, [&](size_t i, Job& J) {
    J.key = keys[i];
    J.w = w[i]->d;
    J.rs = rs ? rs + 64 * i : nullptr;
    J.proof_out = proofs_out + 256 * i;
    return ZKFL_OK;
  });
}

static int full_prove_check(const zkfl_ctx* ctx, const zkfl_key* key, const zkfl_wprog* prog, size_t n,
                            const uint8_t* inputs, size_t* n_in) {
  if (!key || !prog || (n && !inputs)) return fail(ZKFL_E_ARG, "full_prove: null argument");
  if (key->ctx != ctx || prog->ctx != ctx) return fail(ZKFL_E_ARG, "full_prove: key/program of another context");
  uint32_t nw = 0, n_in32 = 0, npub = 0;
  wprog_info(prog->p, &nw, &n_in32, &npub);
  if (nw != key->nVars || npub != key->nPub)
    return fail(ZKFL_E_MISMATCH, "witness program does not match the proving key (nVars / nPublic)");
  *n_in = n_in32;
  std::string err;
  if (!wprog_inputs_ok(prog->p, n, inputs, err)) return fail(ZKFL_E_ARG, err);
  return ZKFL_OK;
}

// Full prove through the keys' witness pipes: for each key, groups of G = its slots witnesses one
// group ahead of its slots (WitPipe); a proof waits on its group's event.  Job i uses key_of(i),
// program prog_of(i) (nVars / inputs of that key), get_input(i, &ptr) yields its input vector
// (n_in x 32 B std form, < r; called in increasing i per key), pub_of(i) its public-signal
// destination (nullable).
extern "C++" {
template <class KeyOf, class ProgOf, class GetInput, class PubOf>
int full_prove_piped(zkfl_ctx* ctx, size_t n, KeyOf key_of, ProgOf prog_of, GetInput get_input, const uint8_t* rs,
                     uint8_t* proofs_out, PubOf pub_of) {
  if (n == 0) return ZKFL_OK;
  HIP_TRY(hipSetDevice(ctx->device), "hipSetDevice");
  struct PerKey {
    zkfl_key* key;
    const WProg* prog;
    size_t G = 0, n_in = 0, groups = 0;
    WitPipe* pipe = nullptr;
    std::vector<size_t> jobs;  // global indices, in order
  };
  std::vector<PerKey> ks;
  std::vector<size_t> kidx(n), local(n), off(n + 1, 0);
  for (size_t i = 0; i < n; i++) {
    zkfl_key* k = key_of(i);
    size_t c = 0;
    while (c < ks.size() && ks[c].key != k) c++;
    if (c == ks.size()) {
      PerKey pk;
      pk.key = k;
      pk.prog = prog_of(i);
      uint32_t nw = 0, nin = 0, np = 0;
      wprog_info(pk.prog, &nw, &nin, &np);
      pk.n_in = nin;
      // one group >= the proofs a key holds in flight: the witness sets'
      // reuse (enqueue_group) relies on it.  ZKFL_WIT_GROUP=m: m times that (a witness launch
      // serves m x as many witnesses; its kernels are latency-bound, so they take about as long)
      static const int wg = getenv("ZKFL_WIT_GROUP") ? std::max(1, atoi(getenv("ZKFL_WIT_GROUP"))) : 1;
      pk.G = (size_t)k->max_slots * wg;
      ks.push_back(pk);
    }
    kidx[i] = c;
    local[i] = ks[c].jobs.size();
    ks[c].jobs.push_back(i);
    off[i + 1] = off[i] + 4 + (size_t)k->nPub * 32;  // pinned record: fail flag | public signals
  }
  for (auto& pk : ks) {
    pk.groups = (pk.jobs.size() + pk.G - 1) / pk.G;
    HIP_TRY(wpipe_get(pk.key, pk.G, pk.key->nVars, pk.n_in, &pk.pipe), "witness pipe allocation");
  }
  uint8_t* pin_out = nullptr;
  HIP_TRY(hipHostMalloc(&pin_out, off[n] + 16), "pinned witness outputs");
  // groups enqueued ahead of the one the slots start (ZKFL_WIT_AHEAD, 1..WIT_SETS - 2): a group
  // is computed while the slots run the `ahead` groups before it
  static const size_t ahead = (size_t)std::clamp(getenv("ZKFL_WIT_AHEAD") ? atoi(getenv("ZKFL_WIT_AHEAD")) : 2, 1,
                                                 WIT_SETS - 2);
  auto enqueue_group = [&](PerKey& pk, size_t g) -> int {
    WitPipe* P = pk.pipe;
    WitPipe::Set& b = P->set[g % WIT_SETS];
    const size_t l0 = g * pk.G, m = std::min(pk.G, pk.jobs.size() - l0), nw = pk.key->nVars;
    const size_t npub = pk.key->nPub;
    HIP_TRY(host_wait(b.ev, true), "witness set reuse");  // its group of WIT_SETS groups ago
    for (size_t j = 0; j < m; j++) {
      const uint8_t* in = nullptr;
      int r = get_input(pk.jobs[l0 + j], &in);
      if (r) return r;
      memcpy(b.pin_in + j * pk.n_in * 32, in, pk.n_in * 32);
    }
    if (pk.n_in)
      HIP_TRY(hipMemcpyAsync(b.in, b.pin_in, m * pk.n_in * 32, hipMemcpyHostToDevice, P->st), "upload inputs");
    HIP_TRY(wprog_enqueue(pk.prog, m, b.in, b.W, b.outs, b.fail, P->st), "witness group");
    for (size_t j = 0; j < m; j++) {
      uint8_t* o = pin_out + off[pk.jobs[l0 + j]];
      HIP_TRY(hipMemcpyAsync(o, b.fail + j, 4, hipMemcpyDeviceToHost, P->st), "witness status");
      if (npub) HIP_TRY(hipMemcpyAsync(o + 4, b.d + j * nw + 1, npub * 32, hipMemcpyDeviceToHost, P->st), "publics");
    }
    HIP_TRY(hipEventRecord(b.ev, P->st), "event");
    return ZKFL_OK;
  };
  int rc = ZKFL_OK;
  for (auto& pk : ks)
    for (size_t g = 0; g <= ahead && g < pk.groups && rc == ZKFL_OK; g++) rc = enqueue_group(pk, g);
  if (rc == ZKFL_OK)
    rc = run_jobs(ctx, n, [&](size_t i, Job& J) {
      PerKey& pk = ks[kidx[i]];
      const size_t g = local[i] / pk.G, j = local[i] % pk.G;
      // the key's slots hold its group g - 1 now and have drained group g - 2, whose set (mod
      // WIT_SETS) group g + ahead takes (ahead <= WIT_SETS - 2)
      if (j == 0 && g >= 1 && g + ahead < pk.groups) {
        int r = enqueue_group(pk, g + ahead);
        if (r) return r;
      }
      J.key = pk.key;
      J.w = pk.pipe->set[g % WIT_SETS].d + j * pk.key->nVars;
      J.w_ready = pk.pipe->set[g % WIT_SETS].ev;
      J.rs = rs ? rs + 64 * i : nullptr;
      J.proof_out = proofs_out + 256 * i;
      return ZKFL_OK;
    });
  for (auto& pk : ks) {
    const hipError_t e = hipStreamSynchronize(pk.pipe->st);
    if (rc == ZKFL_OK && e != hipSuccess) rc = hip_fail(e, "witness pipe");
  }
  size_t bad = SIZE_MAX;
  uint32_t bad_assert = 0;
  for (size_t i = 0; rc == ZKFL_OK && i < n; i++) {
    uint32_t f;
    memcpy(&f, pin_out + off[i], 4);
    if (f != 0xFFFFFFFFu) {  // unsatisfied witness: its proof bytes are zeroed
      memset(proofs_out + 256 * i, 0, 256);
      if (bad == SIZE_MAX) {
        bad = i;
        bad_assert = f;
      }
    }
    uint8_t* pub = pub_of(i);
    if (pub) memcpy(pub, pin_out + off[i] + 4, off[i + 1] - off[i] - 4);
  }
  (void)hipHostFree(pin_out);
  if (rc == ZKFL_OK && bad != SIZE_MAX)
    rc = fail(ZKFL_E_CONSTRAINT, "witness " + std::to_string(bad) + ": assert constraint #" +
                                     std::to_string(bad_assert) + " failed (inputs do not satisfy the circuit)");
  return rc;
}
}  // extern "C++"

int zkfl_groth16_full_prove_batch(zkfl_ctx* ctx, zkfl_key* key, const zkfl_wprog* prog, size_t n,
                                  const uint8_t* inputs, const uint8_t* rs, uint8_t* proofs_out, uint8_t* pubs_out) {
  if (!ctx || (n && !proofs_out)) return fail(ZKFL_E_ARG, "full_prove: null argument");
  size_t n_in = 0;
  int rc = full_prove_check(ctx, key, prog, n, inputs, &n_in);
  if (rc) return rc;
  return full_prove_piped(
      ctx, n, [&](size_t) { return key; }, [&](size_t) { return (const WProg*)prog->p; },
      [&](size_t i, const uint8_t** in) {
        *in = inputs + i * n_in * 32;
        return ZKFL_OK;
      },
      rs, proofs_out, [&](size_t i) { return pubs_out ? pubs_out + (size_t)key->nPub * 32 * i : nullptr; });
}

int zkfl_groth16_full_prove_json(zkfl_ctx* ctx, zkfl_key* key, const zkfl_wprog* prog, const char* input_json,
                                 const uint8_t* rs, uint8_t proof_out[256], uint8_t* pub_out) {
  if (!ctx || !key || !prog || !input_json || !proof_out) return fail(ZKFL_E_ARG, "full_prove_json: null argument");
  std::vector<uint32_t> v;
  std::string err;
  int rc = wprog_inputs_json(prog->p, input_json, v, err);  // the loaded program's signal table
  if (rc) return fail(rc, err);
  v.resize(v.size() + 8);  // never empty (a circuit without inputs still proves one witness)
  return zkfl_groth16_full_prove_batch(ctx, key, prog, 1, reinterpret_cast<const uint8_t*>(v.data()), rs, proof_out,
                                       pub_out);
}

// input.json texts -> input vectors on host worker threads, ahead of the slot scheduler that
// consumes them (at most AHEAD parsed vectors held), so parsing overlaps the proofs in flight.
namespace {
struct JsonParsePool {
  static constexpr size_t AHEAD = 64;
  const WProg* prog;
  const char* const* texts;
  size_t n, n_in;
  std::vector<std::vector<uint32_t>> vec;
  std::vector<std::string> err;
  std::vector<int> rc;
  std::vector<uint8_t> done;
  std::atomic<size_t> next{0};
  size_t consumed = 0;
  bool stop = false;
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::thread> th;

  JsonParsePool(const WProg* p, const char* const* t, size_t count, size_t nin)
      : prog(p), texts(t), n(count), n_in(nin), vec(count), err(count), rc(count, 0), done(count, 0) {
    const unsigned hw = std::max(2u, std::thread::hardware_concurrency());
    const size_t workers = std::min<size_t>({count, (size_t)hw / 2, 8});
    for (size_t w = 0; w < workers; w++) th.emplace_back([this] { work(); });
  }
  ~JsonParsePool() {
    {
      std::lock_guard<std::mutex> g(mu);
      stop = true;
    }
    cv.notify_all();
    for (auto& t : th) t.join();
  }
  void work() {
    for (;;) {
      const size_t i = next.fetch_add(1);
      if (i >= n) return;
      {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return stop || i < consumed + AHEAD; });
        if (stop) return;
      }
      std::vector<uint32_t> v;
      std::string e;
      int r = texts[i] ? wprog_inputs_json(prog, texts[i], v, e) : ZKFL_E_ARG;
      if (!texts[i]) e = "null input json";
      if (r == ZKFL_OK && v.size() != n_in * 8) {
        r = ZKFL_E_ARG;
        e = "input json does not fill the program's inputs";
      }
      v.resize(n_in * 8 + 8);  // never empty
      {
        std::lock_guard<std::mutex> g(mu);
        vec[i] = std::move(v);
        err[i] = std::move(e);
        rc[i] = r;
        done[i] = 1;
      }
      cv.notify_all();
    }
  }
  // Job i's vector (blocks until parsed); job i-1's vector is released (its slot copied it).
  int get(size_t i, const uint8_t** out) {
    std::unique_lock<std::mutex> g(mu);
    if (i > 0) std::vector<uint32_t>().swap(vec[i - 1]);
    consumed = i;
    cv.notify_all();
    cv.wait(g, [&] { return done[i] != 0; });
    if (rc[i]) return fail(rc[i], "input " + std::to_string(i) + ": " + err[i]);
    *out = reinterpret_cast<const uint8_t*>(vec[i].data());
    return ZKFL_OK;
  }
};
}  // namespace

int zkfl_groth16_full_prove_json_batch(zkfl_ctx* ctx, zkfl_key* key, const zkfl_wprog* prog, size_t n,
                                       const char* const* input_jsons, const uint8_t* rs, uint8_t* proofs_out,
                                       uint8_t* pubs_out) {
  if (!ctx || (n && (!input_jsons || !proofs_out))) return fail(ZKFL_E_ARG, "full_prove_json_batch: null argument");
  size_t n_in = 0;
  int rc = full_prove_check(ctx, key, prog, 0, nullptr, &n_in);
  if (rc || n == 0) return rc;
  JsonParsePool pool(prog->p, input_jsons, n, n_in);
  // parsed values are < r by construction
  return full_prove_piped(
      ctx, n, [&](size_t) { return key; }, [&](size_t) { return (const WProg*)prog->p; },
      [&](size_t i, const uint8_t** in) { return pool.get(i, in); }, rs, proofs_out,
      [&](size_t i) { return pubs_out ? pubs_out + (size_t)key->nPub * 32 * i : nullptr; });
}

int zkfl_groth16_full_prove_multi(zkfl_ctx* ctx, size_t n, zkfl_key* const* keys, const zkfl_wprog* const* progs,
                                  const uint8_t* const* inputs, const uint8_t* rs, uint8_t* proofs_out,
                                  uint8_t* const* pubs_out) {
  if (!ctx || (n && (!keys || !progs || !inputs || !proofs_out))) return fail(ZKFL_E_ARG, "full_prove_multi: null argument");
  std::vector<size_t> n_in(n);
  for (size_t i = 0; i < n; i++) {
    int rc = full_prove_check(ctx, keys[i], progs[i], 1, inputs[i], &n_in[i]);
    if (rc) return fail(rc, "job " + std::to_string(i) + ": " + g_err);
  }
  std::vector<std::pair<const zkfl_key*, const zkfl_wprog*>> kp;  // a key's jobs share its witness program
  for (size_t i = 0; i < n; i++) {
    size_t c = 0;
    while (c < kp.size() && kp[c].first != keys[i]) c++;
    if (c == kp.size()) kp.push_back({keys[i], progs[i]});
    else if (kp[c].second != progs[i])
      return fail(ZKFL_E_ARG, "full_prove_multi: job " + std::to_string(i) +
                                  " uses its key with another witness program than an earlier job");
  }
  return full_prove_piped(
      ctx, n, [&](size_t i) { return keys[i]; }, [&](size_t i) { return (const WProg*)progs[i]->p; },
      [&](size_t i, const uint8_t** in) {
        *in = inputs[i];
        return ZKFL_OK;
      },
      rs, proofs_out, [&](size_t i) { return pubs_out ? pubs_out[i] : nullptr; });
}

int zkfl_groth16_prove(zkfl_ctx* ctx, zkfl_key* key, const uint8_t* wtns, size_t wtns_len, const uint8_t* rs,
                       uint8_t proof_out[256], uint8_t* pub_out, size_t* npub) {
  zkfl_witness* w = nullptr;
  int rc = zkfl_witness_upload(ctx, key, wtns, wtns_len, &w);
  if (rc) return rc;
  rc = zkfl_groth16_prove_resident(ctx, key, w, rs, proof_out);
  if (rc == ZKFL_OK) {
    if (pub_out) memcpy(pub_out, w->pub.data(), w->pub.size());
    if (npub) *npub = key->nPub;
  }
  zkfl_witness_free(w);
  return rc;
}

int zkfl_debug_wtrace(zkfl_ctx* ctx, int op, uint32_t cap, void* out, uint32_t* count) {
#if !ZK_WTRACE
  (void)ctx;
  (void)op;
  (void)cap;
  (void)out;
  (void)count;
  return fail(ZKFL_E_ARG, "wave trace: this library was built without -DZK_WTRACE=1");
#else
  if (!ctx || op < 0 || op > 2) return fail(ZKFL_E_ARG, "wave trace: bad arguments");
  HIP_TRY(hipSetDevice(ctx->device), "hipSetDevice");
  auto bind_all = [](const WtBuf& b) {
    hipError_t e = zk_wtrace_bind_tu(b);
    if (e == hipSuccess) e = zk_wtrace_bind_g1(b);
    if (e == hipSuccess) e = zk_wtrace_bind_g2(b);
    if (e == hipSuccess) e = zk_wtrace_bind_ntt(b);
    if (e == hipSuccess) e = zk_wtrace_bind_wit(b);
    if (e == hipSuccess) e = zk_wtrace_bind_joint(b);
    return e;
  };
  HIP_TRY(hipDeviceSynchronize(), "wave trace: sync");
  if (op == 2) {
    if (!ctx->wt.rec) return fail(ZKFL_E_ARG, "wave trace: not started");
    uint32_t n = 0;
    HIP_TRY(hipMemcpy(&n, ctx->wt.cnt, 4, hipMemcpyDeviceToHost), "wave trace: count");
    HIP_TRY(bind_all(WtBuf()), "wave trace: unbind");
    const uint32_t m = std::min(n, std::min(cap, ctx->wt.cap));
    if (out && m) HIP_TRY(hipMemcpy(out, ctx->wt.rec, (size_t)m * sizeof(WtRec), hipMemcpyDeviceToHost), "wave trace: read");
    if (count) *count = n;
    return ZKFL_OK;
  }
  HIP_TRY(bind_all(WtBuf()), "wave trace: unbind");
  if (ctx->wt.rec) (void)hipFree(ctx->wt.rec);
  if (ctx->wt.cnt) (void)hipFree(ctx->wt.cnt);
  ctx->wt = WtBuf();
  if (op == 0) return ZKFL_OK;
  if (cap == 0) return fail(ZKFL_E_ARG, "wave trace: cap must be > 0");
  HIP_TRY(hipMalloc(&ctx->wt.rec, (size_t)cap * sizeof(WtRec)), "wave trace: alloc");
  HIP_TRY(hipMalloc(&ctx->wt.cnt, 4), "wave trace: alloc");
  HIP_TRY(hipMemset(ctx->wt.cnt, 0, 4), "wave trace: reset");
  ctx->wt.cap = cap;
  HIP_TRY(bind_all(ctx->wt), "wave trace: bind");
  HIP_TRY(hipDeviceSynchronize(), "wave trace: sync");
  return ZKFL_OK;
#endif
}

int zkfl_debug_prove_parts(zkfl_ctx* ctx, zkfl_key* key, const uint8_t* wtns, size_t wtns_len, uint8_t* h_out,
                           uint8_t* msm_out) {
  zkfl_witness* w = nullptr;
  int rc = zkfl_witness_upload(ctx, key, wtns, wtns_len, &w);
  if (rc) return rc;
  ProofSlot* s = nullptr;
  rc = get_slot(key, 0, &s);
  uint32_t zeros[16] = {0};
  if (rc == ZKFL_OK && MSM_MERGE_CH && !key->dbg_zero) {  // see zkfl_key::dbg_zero
    const size_t bytes = std::max<size_t>(key->nVars, (size_t)key->n + 4) * 32;
    hipError_t e = hipMalloc(&key->dbg_zero, bytes);
    // on the slot's stream and waited for: hipMemset is asynchronous to the host and runs on the
    // null stream, which the slots' non-blocking streams do not wait for -- the MSMs below read
    // the zeros, and a recycled allocation (a freed key's memory) is not zero.  (Found as a
    // parity failure that appeared only after earlier tests had freed large keys.)
    if (e == hipSuccess) e = hipMemsetAsync(key->dbg_zero, 0, bytes, s->st_main);
    if (e == hipSuccess) e = hipStreamSynchronize(s->st_main);
    if (e != hipSuccess) rc = hip_fail(e, "parity hook zeros");
  }
  if (rc == ZKFL_OK && s->busy) rc = wait_slot(s);
  if (rc == ZKFL_OK) {
    s->out_proof = nullptr;
    s->out_part = nullptr;
    rc = enqueue_proof(ctx, key, s, w->d, zeros, 1);
  }
  if (rc == ZKFL_OK) rc = wait_slot(s);
  hipStream_t st = s ? s->st_main : ctx->st;
  uint32_t* d_o = nullptr;
  if (rc == ZKFL_OK && msm_out) {
    hipError_t e = hipMalloc(&d_o, 64 * 4 + 128);
    if (e == hipSuccess) {
      hipLaunchKernelGGL(k_point_out<FqOps>, dim3(1), dim3(4), 0, st, s->res, 4, d_o);
      hipLaunchKernelGGL(k_point_out<Fq2Ops>, dim3(1), dim3(1), 0, st, s->resB2, 1, d_o + 64);
      e = hipGetLastError();
    }
    std::vector<uint8_t> tmp(64 * 4 + 128);
    if (e == hipSuccess) e = hipMemcpyAsync(tmp.data(), d_o, tmp.size(), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) rc = hip_fail(e, "debug parts");
    if (rc == ZKFL_OK) {
      // res order A, B1, C, H ; output order A | B1 | B2 | C | H
      memcpy(msm_out, tmp.data(), 64);
      memcpy(msm_out + 64, tmp.data() + 64, 64);
      memcpy(msm_out + 128, tmp.data() + 256, 128);
      memcpy(msm_out + 256, tmp.data() + 128, 64);
      memcpy(msm_out + 320, tmp.data() + 192, 64);
    }
  }
  if (rc == ZKFL_OK && h_out) {
    hipError_t e = hipMemcpyAsync(h_out, s->h, (size_t)key->n * 32, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) rc = hip_fail(e, "debug h");
  }
  if (d_o) (void)hipFree(d_o);
  zkfl_witness_free(w);
  return rc;
}

int zkfl_msm_g1(zkfl_ctx* ctx, const uint8_t* bases, const uint8_t* scalars, size_t n, uint8_t out[64]) {
  return run_msm_primitive<FqOps>(ctx, bases, scalars, n, out);
}

int zkfl_msm_g2(zkfl_ctx* ctx, const uint8_t* bases, const uint8_t* scalars, size_t n, uint8_t out[128]) {
  return run_msm_primitive<Fq2Ops>(ctx, bases, scalars, n, out);
}

int zkfl_ntt_coset(zkfl_ctx* ctx, uint8_t* data, uint32_t logn) {
  if (!ctx || !data || logn < 1 || logn > 27) return fail(ZKFL_E_ARG, "ntt: bad args");
  hipStream_t st = ctx->st;
  NttPlan pl;
  Fr* d = nullptr;
  const size_t n = (size_t)1 << logn;
  int rc = ZKFL_OK;
  hipError_t e = ntt_plan_alloc(pl, (int)logn, st);
  if (e == hipSuccess) e = hipMalloc(&d, n * 32);
  if (e == hipSuccess) e = hipMemcpyAsync(d, data, n * 32, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_fr_std_to_mont, dim3(zk_grid(n, 256)), dim3(256), 0, st, d, n);
    e = ntt_coset_shift(pl, d, 1, n, st);
  }
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_fr_mont_to_std, dim3(zk_grid(n, 256)), dim3(256), 0, st, d, n);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(data, d, n * 32, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) rc = hip_fail(e, "ntt");
  ntt_plan_free(pl);
  if (d) (void)hipFree(d);
  return rc;
}

int zkfl_setup_g1_gen_mul(zkfl_ctx* ctx, const uint8_t* scalars, size_t n, uint8_t* out) {
  return run_gen_mul<FqOps>(ctx, scalars, n, out, false);
}

int zkfl_setup_g2_gen_mul(zkfl_ctx* ctx, const uint8_t* scalars, size_t n, uint8_t* out) {
  return run_gen_mul<Fq2Ops>(ctx, scalars, n, out, true);
}

// Ceremony primitives (csrc/setup.hip)
static int setup_scale_abi(zkfl_ctx* ctx, const uint8_t* points, const uint8_t* scalars, size_t n, uint8_t* out,
                           bool g2) {
  if (!ctx || (n && (!points || !scalars || !out))) return fail(ZKFL_E_ARG, "setup scale: bad args");
  hipError_t e = setup_scale(g2, ctx->st, points, scalars, n, out);
  return e == hipSuccess ? ZKFL_OK : hip_fail(e, "setup scale");
}

int zkfl_setup_g1_scale(zkfl_ctx* ctx, const uint8_t* points, const uint8_t* scalars, size_t n, uint8_t* out) {
  return setup_scale_abi(ctx, points, scalars, n, out, false);
}

int zkfl_setup_g2_scale(zkfl_ctx* ctx, const uint8_t* points, const uint8_t* scalars, size_t n, uint8_t* out) {
  return setup_scale_abi(ctx, points, scalars, n, out, true);
}

static int setup_lagrange_abi(zkfl_ctx* ctx, const uint8_t* points, uint32_t logn, uint8_t* out, bool g2) {
  if (!ctx || !points || !out) return fail(ZKFL_E_ARG, "setup lagrange: bad args");
  if (logn > 28) return fail(ZKFL_E_ARG, "setup lagrange: logn > 28 (BN254 Fr 2-adicity)");
  hipError_t e = setup_lagrange(g2, ctx->st, points, (int)logn, out);
  return e == hipSuccess ? ZKFL_OK : hip_fail(e, "setup lagrange");
}

int zkfl_setup_g1_lagrange(zkfl_ctx* ctx, const uint8_t* points, uint32_t logn, uint8_t* out) {
  return setup_lagrange_abi(ctx, points, logn, out, false);
}

int zkfl_setup_g2_lagrange(zkfl_ctx* ctx, const uint8_t* points, uint32_t logn, uint8_t* out) {
  return setup_lagrange_abi(ctx, points, logn, out, true);
}

static int setup_lincomb_abi(zkfl_ctx* ctx, const uint8_t* bases, size_t n_bases, size_t n_out,
                             const uint64_t* rowptr, const uint32_t* idx, const uint8_t* coefs, uint8_t* out,
                             bool g2) {
  if (!ctx || !rowptr || (n_out && !out)) return fail(ZKFL_E_ARG, "setup lincomb: bad args");
  if (rowptr[0] != 0) return fail(ZKFL_E_ARG, "setup lincomb: rowptr[0] != 0");
  for (size_t r = 0; r < n_out; r++)
    if (rowptr[r + 1] < rowptr[r]) return fail(ZKFL_E_ARG, "setup lincomb: rowptr not monotonic at " + std::to_string(r));
  const uint64_t nnz = rowptr[n_out];
  if (nnz >= 0xffffffffull) return fail(ZKFL_E_ARG, "setup lincomb: more than 2^32 - 2 terms");
  if (nnz && (!idx || !coefs || !bases)) return fail(ZKFL_E_ARG, "setup lincomb: bad args");
  for (uint64_t t = 0; t < nnz; t++)  // no device access outside the bases
    if (idx[t] >= n_bases) return fail(ZKFL_E_ARG, "setup lincomb: term " + std::to_string(t) + " base index out of range");
  hipError_t e = setup_lincomb(g2, ctx->st, bases, n_bases, n_out, rowptr, idx, coefs, out);
  return e == hipSuccess ? ZKFL_OK : hip_fail(e, "setup lincomb");
}

int zkfl_setup_g1_lincomb(zkfl_ctx* ctx, const uint8_t* bases, size_t n_bases, size_t n_out, const uint64_t* rowptr,
                          const uint32_t* idx, const uint8_t* coefs, uint8_t* out) {
  return setup_lincomb_abi(ctx, bases, n_bases, n_out, rowptr, idx, coefs, out, false);
}

int zkfl_setup_g2_lincomb(zkfl_ctx* ctx, const uint8_t* bases, size_t n_bases, size_t n_out, const uint64_t* rowptr,
                          const uint32_t* idx, const uint8_t* coefs, uint8_t* out) {
  return setup_lincomb_abi(ctx, bases, n_bases, n_out, rowptr, idx, coefs, out, true);
}

// ---------------------------------------------------------------------------
// Verification (csrc/verify.hip)
// ---------------------------------------------------------------------------
static int vk_get(zkfl_ctx* ctx, const uint8_t* vk, size_t vk_len, size_t npub) {
  if (!vk_same(ctx->vk, vk, vk_len)) {
    vk_free(ctx->vk);
    ctx->vk = nullptr;
    std::string err;
    VkDev* p = nullptr;
    int rc = vk_prepare(vk, vk_len, ctx->st, &p, err);
    if (rc != ZKFL_OK) return fail(rc, err);
    ctx->vk = p;
  }
  if (vk_npub(ctx->vk) != npub)
    return fail(ZKFL_E_MISMATCH, "verify: " + std::to_string(npub) + " public signals, key expects " +
                                     std::to_string(vk_npub(ctx->vk)));
  return ZKFL_OK;
}

int zkfl_groth16_verify_batch(zkfl_ctx* ctx, const uint8_t* vk, size_t vk_len, size_t n, const uint8_t* pubs,
                              size_t npub, const uint8_t* proofs, int32_t* results) {
  if (!ctx || !vk || (n && (!proofs || !results || (npub && !pubs)))) return fail(ZKFL_E_ARG, "verify: bad args");
  HIP_TRY(hipSetDevice(ctx->device), "hipSetDevice");
  int rc = vk_get(ctx, vk, vk_len, npub);
  if (rc != ZKFL_OK) return rc;
  std::string err;
  rc = verify_batch(ctx->vk, n, pubs, proofs, results, ctx->st, err);
  return rc == ZKFL_OK ? rc : fail(rc, err);
}

int zkfl_groth16_verify(zkfl_ctx* ctx, const uint8_t* vk, size_t vk_len, const uint8_t* pub, size_t npub,
                        const uint8_t proof[256]) {
  int32_t res = 0;
  int rc = zkfl_groth16_verify_batch(ctx, vk, vk_len, 1, pub, npub, proof, &res);
  return rc == ZKFL_OK ? res : rc;
}

static int pairing_common(zkfl_ctx* ctx, size_t n, const uint8_t* g1, const uint8_t* g2, uint8_t* out, int fe) {
  if (!ctx || (n && (!g1 || !g2 || !out))) return fail(ZKFL_E_ARG, "pairing: bad args");
  HIP_TRY(hipSetDevice(ctx->device), "hipSetDevice");
  std::string err;
  int rc = pairing_batch(n, g1, g2, fe, out, ctx->st, err);
  return rc == ZKFL_OK ? rc : fail(rc, err);
}

int zkfl_pairing(zkfl_ctx* ctx, size_t n, const uint8_t* g1, const uint8_t* g2, uint8_t* gt_out) {
  return pairing_common(ctx, n, g1, g2, gt_out, 1);
}

int zkfl_debug_miller_loop(zkfl_ctx* ctx, size_t n, const uint8_t* g1, const uint8_t* g2, uint8_t* out) {
  return pairing_common(ctx, n, g1, g2, out, 0);
}

// ---------------------------------------------------------------------------
// Witness generation (csrc/witness.hip)
// ---------------------------------------------------------------------------
int zkfl_wprog_load(zkfl_ctx* ctx, const uint8_t* prog, size_t len, zkfl_wprog** out) {
  if (!ctx || !prog || !out) return fail(ZKFL_E_ARG, "wprog_load: null argument");
  HIP_TRY(hipSetDevice(ctx->device), "hipSetDevice");
  std::string err;
  WProg* p = nullptr;
  int rc = wprog_load(prog, len, ctx->st, &p, err);
  if (rc != ZKFL_OK) return fail(rc, err);
  zkfl_wprog* w = new zkfl_wprog();
  w->ctx = ctx;
  ctx_retain(ctx);  // dropped by zkfl_wprog_free
  w->p = p;
  *out = w;
  return ZKFL_OK;
}

int zkfl_wprog_free(zkfl_wprog* prog) {
  if (!prog) return ZKFL_OK;
  zkfl_ctx* ctx = prog->ctx;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->st);
  wprog_free(prog->p);
  delete prog;
  ctx_release(ctx);
  return ZKFL_OK;
}

int zkfl_wprog_info(const zkfl_wprog* prog, uint32_t* n_wires, uint32_t* n_inputs, uint32_t* n_public) {
  if (!prog) return fail(ZKFL_E_ARG, "null program");
  wprog_info(prog->p, n_wires, n_inputs, n_public);
  return ZKFL_OK;
}

size_t zkfl_wtns_size(const zkfl_wprog* prog) {
  uint32_t nw = 0;
  if (prog) wprog_info(prog->p, &nw, nullptr, nullptr);
  return 76 + 32 * (size_t)nw;
}

static void wtns_header(uint8_t* dst, uint32_t nw) {
  const uint32_t h1[3] = {0x736e7477u /* "wtns" */, 2, 2};
  memcpy(dst, h1, 12);
  uint32_t t = 1;
  uint64_t sz = 40;
  memcpy(dst + 12, &t, 4);
  memcpy(dst + 16, &sz, 8);
  uint32_t n8 = 32;
  memcpy(dst + 24, &n8, 4);
  memcpy(dst + 28, R_LIMBS, 32);
  memcpy(dst + 60, &nw, 4);
  t = 2;
  sz = 32ull * nw;
  memcpy(dst + 64, &t, 4);
  memcpy(dst + 68, &sz, 8);
}

int zkfl_witness_compute(zkfl_ctx* ctx, const zkfl_wprog* prog, size_t n, const uint8_t* inputs, uint8_t* wtns_out) {
  if (!ctx || !prog || (n && (!wtns_out || !inputs))) return fail(ZKFL_E_ARG, "witness_compute: null argument");
  if (n == 0) return ZKFL_OK;
  HIP_TRY(hipSetDevice(ctx->device), "hipSetDevice");
  uint32_t nw = 0;
  wprog_info(prog->p, &nw, nullptr, nullptr);
  const size_t img = 76 + 32 * (size_t)nw;
  Fr* d = nullptr;
  HIP_TRY(hipMalloc(&d, n * (size_t)nw * 32), "witness buffer");
  std::vector<Fr*> outs(n);
  for (size_t j = 0; j < n; j++) outs[j] = d + j * nw;
  std::string err;
  int rc = wprog_run(prog->p, n, inputs, outs.data(), ctx->st, err);
  hipError_t e = hipSuccess;
  for (size_t j = 0; rc == ZKFL_OK && e == hipSuccess && j < n; j++) {
    wtns_header(wtns_out + j * img, nw);
    e = hipMemcpyAsync(wtns_out + j * img + 76, outs[j], 32ull * nw, hipMemcpyDeviceToHost, ctx->st);
  }
  if (rc == ZKFL_OK && e == hipSuccess) e = hipStreamSynchronize(ctx->st);
  (void)hipFree(d);
  if (rc != ZKFL_OK) return fail(rc, err);
  if (e != hipSuccess) return hip_fail(e, "witness download");
  return ZKFL_OK;
}

int zkfl_wprog_parse_inputs(const uint8_t* prog, size_t len, const char* input_json, uint8_t* inputs_out, size_t cap,
                            size_t* n_inputs) {
  if (!prog || !input_json || !n_inputs || (cap && !inputs_out)) return fail(ZKFL_E_ARG, "parse_inputs: null argument");
  std::vector<uint32_t> v;
  std::string err;
  int rc = wprog_image_inputs_json(prog, len, input_json, v, err);
  if (rc != ZKFL_OK) return fail(rc, err);
  *n_inputs = v.size() / 8;
  if (*n_inputs > cap) return fail(ZKFL_E_ARG, "parse_inputs: output buffer too small");
  memcpy(inputs_out, v.data(), v.size() * 4);
  return ZKFL_OK;
}

int zkfl_witness_compute_json(zkfl_ctx* ctx, const zkfl_wprog* prog, const char* input_json, uint8_t* wtns_out) {
  if (!ctx || !prog || !input_json || !wtns_out) return fail(ZKFL_E_ARG, "witness_compute_json: null argument");
  std::vector<uint32_t> v;
  std::string err;
  int rc = wprog_inputs_json(prog->p, input_json, v, err);
  if (rc != ZKFL_OK) return fail(rc, err);
  return zkfl_witness_compute(ctx, prog, 1, reinterpret_cast<const uint8_t*>(v.data()), wtns_out);
}

int zkfl_witness_compute_resident(zkfl_ctx* ctx, const zkfl_wprog* prog, const zkfl_key* key, size_t n,
                                  const uint8_t* inputs, zkfl_witness** out) {
  if (!ctx || !prog || !key || (n && (!out || !inputs))) return fail(ZKFL_E_ARG, "witness_compute: null argument");
  uint32_t nw = 0, npub = 0;
  wprog_info(prog->p, &nw, nullptr, &npub);
  if (nw != key->nVars || npub != key->nPub)
    return fail(ZKFL_E_MISMATCH, "witness program does not match the proving key (nVars / nPublic)");
  HIP_TRY(hipSetDevice(ctx->device), "hipSetDevice");
  std::vector<zkfl_witness*> ws(n, nullptr);
  std::vector<Fr*> outs(n, nullptr);
  hipError_t e = hipSuccess;
  for (size_t j = 0; j < n && e == hipSuccess; j++) {
    ws[j] = new zkfl_witness();
    ws[j]->key = key;
    e = hipMalloc(&ws[j]->d, 32ull * nw);
    outs[j] = ws[j]->d;
  }
  std::string err;
  int rc = e == hipSuccess ? wprog_run(prog->p, n, inputs, outs.data(), ctx->st, err) : hip_fail(e, "witness alloc");
  if (rc == ZKFL_OK) {
    // public signals (witness[1..nPub]) for the prove call's public.json
    for (size_t j = 0; j < n && e == hipSuccess; j++) {
      ws[j]->pub.resize(32ull * npub);
      if (npub) e = hipMemcpyAsync(ws[j]->pub.data(), ws[j]->d + 1, 32ull * npub, hipMemcpyDeviceToHost, ctx->st);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->st);
    if (e != hipSuccess) rc = hip_fail(e, "public signals");
  } else if (!err.empty()) {
    rc = fail(rc, err);
  }
  if (rc != ZKFL_OK) {
    for (zkfl_witness* w : ws)
      if (w) {
        if (w->d) (void)hipFree(w->d);
        delete w;
      }
    return rc;
  }
  for (size_t j = 0; j < n; j++) out[j] = ws[j];
  return ZKFL_OK;
}


// ---------------------------------------------------------------------------
// Poseidon / vectorHash / Merkle trees (csrc/merkle.hip)
// ---------------------------------------------------------------------------
int zkfl_poseidon_params(uint32_t t, uint8_t* consts_out, uint8_t* xy_out, uint32_t* rp_out) {
  if (t < 2 || t > 17) return fail(ZKFL_E_ARG, "poseidon width t must be in 2..17");
  pos_params_raw(t, consts_out, xy_out);
  if (rp_out) *rp_out = pos_rp(t);
  return ZKFL_OK;
}

int zkfl_poseidon_batch(zkfl_ctx* ctx, uint32_t arity, size_t n, const uint8_t* inputs, uint8_t* out) {
  if (!ctx || (n && (!inputs || !out))) return fail(ZKFL_E_ARG, "poseidon_batch: null argument");
  if (arity < 1 || arity > POS_MAX_ARITY) return fail(ZKFL_E_ARG, "poseidon arity must be in 1..16");
  int rc = check_fr_array(inputs, n * arity, "poseidon input");
  if (rc || !n) return rc;
  HIP_TRY(hipSetDevice(ctx->device), "hipSetDevice");
  if ((rc = pos_ready(ctx))) return rc;
  DevBufs B;
  Fr *d_in, *d_out;
  HIP_TRY(B.get((void**)&d_in, n * arity * 32), "alloc");
  HIP_TRY(B.get((void**)&d_out, n * 32), "alloc");
  hipStream_t st = ctx->st;
  HIP_TRY(hipMemcpyAsync(d_in, inputs, n * arity * 32, hipMemcpyHostToDevice, st), "upload");
  int pi = ctx->prof.begin("poseidon", st);
  HIP_TRY(poseidon_batch(ctx->pos, arity, n, d_in, d_out, st), "poseidon");
  ctx->prof.end(pi, st, (double)n);
  HIP_TRY(hipMemcpyAsync(out, d_out, n * 32, hipMemcpyDeviceToHost, st), "download");
  HIP_TRY(hipStreamSynchronize(st), "sync");
  return ZKFL_OK;
}

int zkfl_vector_hash_batch(zkfl_ctx* ctx, uint32_t len, size_t n, const uint8_t* values, uint8_t* out) {
  if (!ctx || (n && (!values || !out))) return fail(ZKFL_E_ARG, "vector_hash_batch: null argument");
  if (len < 1 || len > VHASH_CHUNK * VHASH_CHUNK) return fail(ZKFL_E_ARG, "vector length must be in 1..256");
  int rc = check_fr_array(values, n * len, "vector value");
  if (rc || !n) return rc;
  HIP_TRY(hipSetDevice(ctx->device), "hipSetDevice");
  if ((rc = pos_ready(ctx))) return rc;
  DevBufs B;
  Fr *d_in, *d_out, *d_s;
  const size_t nch = (len + VHASH_CHUNK - 1) / VHASH_CHUNK;
  HIP_TRY(B.get((void**)&d_in, n * len * 32), "alloc");
  HIP_TRY(B.get((void**)&d_out, n * 32), "alloc");
  HIP_TRY(B.get((void**)&d_s, n * nch * 32), "alloc");
  hipStream_t st = ctx->st;
  HIP_TRY(hipMemcpyAsync(d_in, values, n * len * 32, hipMemcpyHostToDevice, st), "upload");
  int pi = ctx->prof.begin("vector_hash", st);
  HIP_TRY(vector_hash_batch(ctx->pos, len, n, d_in, d_out, false, d_s, st), "vector hash");
  ctx->prof.end(pi, st, (double)n);
  HIP_TRY(hipMemcpyAsync(out, d_out, n * 32, hipMemcpyDeviceToHost, st), "download");
  HIP_TRY(hipStreamSynchronize(st), "sync");
  return ZKFL_OK;
}

int zkfl_merkle_build(zkfl_ctx* ctx, const uint8_t* leaves, size_t n, uint32_t depth, uint8_t* tree_out) {
  int rc = tree_args(ctx, n, depth, leaves, tree_out);
  if (rc) return rc;
  if ((rc = check_fr_array(leaves, n, "leaf"))) return rc;
  HIP_TRY(hipSetDevice(ctx->device), "hipSetDevice");
  if ((rc = pos_ready(ctx))) return rc;
  DevBufs B;
  Fr *d_raw, *d_leaves;
  HIP_TRY(B.get((void**)&d_raw, n * 32), "alloc");
  HIP_TRY(B.get((void**)&d_leaves, n * 32), "alloc");
  if (n) {
    HIP_TRY(hipMemcpyAsync(d_raw, leaves, n * 32, hipMemcpyHostToDevice, ctx->st), "upload");
    HIP_TRY(fr_to_mont_batch(d_raw, n, d_leaves, ctx->st), "leaves");
  }
  return tree_from_device_leaves(ctx, B, d_leaves, n, depth, tree_out);
}

int zkfl_dataset_commit(zkfl_ctx* ctx, const uint8_t* values, size_t n, uint32_t len, uint32_t depth,
                        uint8_t* tree_out) {
  int rc = tree_args(ctx, n, depth, values, tree_out);
  if (rc) return rc;
  if (len < 1 || len > VHASH_CHUNK * VHASH_CHUNK) return fail(ZKFL_E_ARG, "vector length must be in 1..256");
  if ((rc = check_fr_array(values, n * len, "sample value"))) return rc;
  HIP_TRY(hipSetDevice(ctx->device), "hipSetDevice");
  if ((rc = pos_ready(ctx))) return rc;
  DevBufs B;
  Fr *d_in, *d_leaves, *d_s;
  const size_t nch = (len + VHASH_CHUNK - 1) / VHASH_CHUNK;
  HIP_TRY(B.get((void**)&d_in, n * len * 32), "alloc");
  HIP_TRY(B.get((void**)&d_leaves, n * 32), "alloc");
  HIP_TRY(B.get((void**)&d_s, n * nch * 32), "alloc");
  if (n) {
    HIP_TRY(hipMemcpyAsync(d_in, values, n * len * 32, hipMemcpyHostToDevice, ctx->st), "upload");
    int pi = ctx->prof.begin("vector_hash", ctx->st);
    HIP_TRY(vector_hash_batch(ctx->pos, len, n, d_in, d_leaves, true, d_s, ctx->st), "leaf hashes");
    ctx->prof.end(pi, ctx->st, (double)n);
  }
  return tree_from_device_leaves(ctx, B, d_leaves, n, depth, tree_out);
}

}  // extern "C"
