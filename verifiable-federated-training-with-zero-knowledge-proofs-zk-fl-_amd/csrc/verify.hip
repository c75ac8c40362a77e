// GPU Groth16 verification over BN254 (batched: one lane per proof).
//
// Replaces `snarkjs groth16 verify <vkey> <public> <proof>` [ext] (reference call sites
// tests/full_system_simulation.mjs:865-868, 975-983, 1116-1125), i.e. snarkjs groth16_verify:
//   * every public signal < r (publicInputsAreValid), proof points well formed;
//   * vk_x = IC0 + sum pub_i IC_i;
//   * e(-pi_a, pi_b) e(vk_x, gamma2) e(pi_c, delta2) e(alpha1, beta2) == 1.
// Restated in oracle/groth16.py::verify.  This implementation is stricter on encodings:
// coordinates must be canonical (< q) and pi_b must lie in the order-r subgroup of the twist.
//
// Kernels per batch: k_g2_prepare (pi_b: checks + the 102 Miller-loop line coefficients),
// k_verify_inputs (pi_a, pi_c checks, vk_x by 4-bit windows over per-key tables),
// k_miller (3 prepared pairs + the key's precomputed Miller value of (alpha1, beta2), final
// exponentiation, compare with 1).  Per key (cached by the context): IC window tables and the
// lines of beta2, gamma2, delta2.
#include <hip/hip_runtime.h>
#include <string.h>

#include <cstdio>

#include "common.h"
#include "curve.h"
#include "pairing.h"
#include "verify.h"
#include "zkfl.h"

namespace zkfl {

namespace {

constexpr uint32_t ST_INF = 1u, ST_BAD = 2u;

ZK_DEV bool lt_mod(const uint32_t* v, const uint32_t* P) {
  for (int i = 7; i >= 0; i--)
    if (v[i] != P[i]) return v[i] < P[i];
  return false;
}

// canonical std-form Fq -> Montgomery; false if >= q
ZK_DEV bool fq_load_std(const uint32_t* s, Fq& out) {
  Fq t;
#pragma unroll
  for (int i = 0; i < 8; i++) t.v[i] = s[i];
  if (!lt_mod(t.v, FqP::P)) return false;
  out = fp_to_mont(t);
  return true;
}

ZK_DEV Fq fq_small(uint32_t x) {  // Montgomery form of a small constant
  Fq t = fp_zero<FqP>();
  t.v[0] = x;
  return fp_to_mont(t);
}

// affine G1 from 16 std u32; status bits
ZK_DEV uint32_t g1_load(const uint32_t* s, G1Aff& p) {
  bool ok = fq_load_std(s, p.x) && fq_load_std(s + 8, p.y);
  if (!ok) return ST_BAD;
  if (aff_is_inf(p)) return ST_INF;
  // y^2 == x^3 + 3
  Fq lhs = fp_sqr(p.y);
  Fq rhs = fp_add(fp_mul(fp_sqr(p.x), p.x), fq_small(3));
  return fp_eq(lhs, rhs) ? 0u : ST_BAD;
}

ZK_DEV uint32_t g2_load(const uint32_t* s, G2Aff& q) {
  bool ok = fq_load_std(s, q.x.c0) && fq_load_std(s + 8, q.x.c1) && fq_load_std(s + 16, q.y.c0) &&
            fq_load_std(s + 24, q.y.c1);
  if (!ok) return ST_BAD;
  if (aff_is_inf(q)) return ST_INF;
  Fq2 lhs = f2_sqr(q.y);
  Fq2 rhs = f2_add(f2_mul(f2_sqr(q.x), q.x), load_fq2(TWIST_B));
  return f2_eq(lhs, rhs) ? 0u : ST_BAD;
}

// psi (untwist-Frobenius-twist) on XYZZ coordinates: conj is a field automorphism, so
// psi(X, Y, ZZ, ZZZ) = (conj(X) gx, conj(Y) gy, conj(ZZ), conj(ZZZ))
ZK_DEV G2P g2_psi(const G2P& p) {
  G2P r;
  r.X = f2_mul(f2_conj(p.X), load_fq2(TWIST_FROB_X));
  r.Y = f2_mul(f2_conj(p.Y), load_fq2(TWIST_FROB_Y));
  r.ZZ = f2_conj(p.ZZ);
  r.ZZZ = f2_conj(p.ZZZ);
  return r;
}

ZK_DEV bool g2_eq(const G2P& a, const G2P& b) {
  const bool ia = xyzz_is_inf(a), ib = xyzz_is_inf(b);
  if (ia || ib) return ia && ib;
  return f2_eq(f2_mul(a.X, b.ZZ), f2_mul(b.X, a.ZZ)) && f2_eq(f2_mul(a.Y, b.ZZZ), f2_mul(b.Y, a.ZZZ));
}

// Order-r subgroup membership of a twist point (G2 has a large cofactor), by the BN endomorphism
// criterion [x0+1]P + psi([x0]P) + psi^2([x0]P) == psi^3([2 x0]P), x0 = u (ePrint 2022/348 §5.1):
// a 63-bit scalar multiplication instead of [r]P.  Checked against [r]P on subgroup and
// non-subgroup points in tests (tests/test_gpu_verify.py).
ZK_DEV bool g2_in_subgroup(const G2Aff& q) {
  const uint32_t u[8] = {(uint32_t)BN_U, (uint32_t)(BN_U >> 32), 0, 0, 0, 0, 0, 0};
  const G2P p = xyzz_from_affine<Fq2Ops>(q);
  const G2P xp = xyzz_scalar_mul<Fq2Ops>(p, u);
  const G2P pxp = g2_psi(xp);
  G2P lhs = xyzz_add<Fq2Ops>(xyzz_add<Fq2Ops>(xyzz_add<Fq2Ops>(xp, p), pxp), g2_psi(pxp));
  G2P rhs = g2_psi(g2_psi(g2_psi(xyzz_dbl<Fq2Ops>(xp))));
  return g2_eq(lhs, rhs);
}

__global__ __launch_bounds__(64) void k_g2_prepare(size_t n, const uint32_t* q_std, size_t q_stride, int subgroup,
                                                   LineCoef* lines, uint32_t* qstat) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  G2Aff q;
  uint32_t st = g2_load(q_std + i * q_stride, q);
  if (st == 0 && subgroup && !g2_in_subgroup(q)) st = ST_BAD;
  qstat[i] = st;
  if (st == 0) g2_prepare_lines(q.x, q.y, lines + i * ATE_NLINES);
}

__global__ __launch_bounds__(64) void k_g1_load(size_t n, const uint32_t* p_std, G1Aff* out, uint32_t* pstat) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  G1Aff p;
  uint32_t st = g1_load(p_std + i * 16, p);
  if (st) p.x = p.y = fp_zero<FqP>();
  out[i] = p;
  pstat[i] = st;
}

// j * IC_i for j = 0..15, affine Montgomery (batch inversion over the 15 non-trivial multiples)
__global__ __launch_bounds__(64) void k_ic_tables(uint32_t npub1, const uint32_t* ic_std, G1Aff* table,
                                                  uint32_t* stat) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npub1) return;
  G1Aff p;
  uint32_t st = g1_load(ic_std + i * 16, p);
  stat[i] = st & ST_BAD;
  G1Aff* t = table + (size_t)i * 16;
  t[0].x = t[0].y = fp_zero<FqP>();
  if (st) {  // infinity (or invalid: reported through stat)
    for (int j = 1; j < 16; j++) t[j] = t[0];
    return;
  }
  G1P m[16];
  m[1] = xyzz_from_affine<FqOps>(p);
  for (int j = 2; j < 16; j++) m[j] = xyzz_madd<FqOps>(m[j - 1], p);
  // batch-invert ZZZ (never zero: j*IC != O for 0 < j < r)
  Fq pre[16];
  pre[1] = m[1].ZZZ;
  for (int j = 2; j < 16; j++) pre[j] = fp_mul(pre[j - 1], m[j].ZZZ);
  Fq inv = fp_inv(pre[15]);
  for (int j = 15; j >= 1; j--) {
    Fq iZZZ = (j > 1) ? fp_mul(inv, pre[j - 1]) : inv;
    if (j > 1) inv = fp_mul(inv, m[j].ZZZ);
    Fq iZ = fp_mul(m[j].ZZ, iZZZ);
    t[j].x = fp_mul(m[j].X, fp_sqr(iZ));
    t[j].y = fp_mul(m[j].Y, iZZZ);
  }
}

// Per proof: public-signal range, pi_a / pi_c checks, vk_x; writes the 3 G1 points of the
// pairing product (-pi_a, vk_x, pi_c) and a status (0 ok, else invalid).
__global__ __launch_bounds__(64) void k_verify_inputs(size_t n, uint32_t npub, const uint32_t* pubs,
                                                      const uint32_t* proofs, const G1Aff* ic_table,
                                                      const uint32_t* bstat, G1Aff* P, uint32_t* status) {
  size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const uint32_t* pub = pubs + k * npub * 8;
  const uint32_t* pr = proofs + k * 64;
  uint32_t bad = (bstat[k] & ST_BAD) ? 1u : 0u;
  for (uint32_t i = 0; i < npub; i++)
    if (!lt_mod(pub + i * 8, FrP::P)) bad |= 2u;
  G1Aff a, c;
  uint32_t sa = g1_load(pr, a), sc = g1_load(pr + 48, c);
  if ((sa | sc) & ST_BAD) bad |= 4u;
  G1Aff* out = P + k * 3;
  const G1Aff zero = {fp_zero<FqP>(), fp_zero<FqP>()};
  if (bad) {
    status[k] = bad;
    out[0] = out[1] = out[2] = zero;
    return;
  }
  // pair (-A, B) vanishes when either is infinity
  out[0] = (sa == ST_INF || bstat[k] == ST_INF) ? zero : aff_neg<FqOps>(a);
  out[2] = c;
  // vk_x = IC0 + sum pub_i * IC_i, 4-bit windows, MSB first
  G1P acc = xyzz_inf<FqOps>();
  for (int w = 63; w >= 0; w--) {
    if (w != 63)
      for (int d = 0; d < 4; d++) acc = xyzz_dbl<FqOps>(acc);
    for (uint32_t i = 0; i < npub; i++) {
      uint32_t dig = (pub[i * 8 + (w >> 3)] >> ((w & 7) * 4)) & 15u;
      if (dig) acc = xyzz_madd<FqOps>(acc, ic_table[(size_t)(i + 1) * 16 + dig]);
    }
  }
  acc = xyzz_madd<FqOps>(acc, ic_table[1]);  // 1 * IC0
  out[1] = xyzz_to_affine<FqOps>(acc);
  status[k] = 0;
}

struct PairLines {
  const LineCoef* base[4];
  size_t stride[4];  // in LineCoef units per item (0 = shared by all items)
};

// f = prod over pairs of the Miller loop (prepared lines) [* fmul]; optionally final
// exponentiation; writes f (Montgomery) and/or result = (status ok && f == 1).
__global__ __launch_bounds__(64) void k_miller(size_t n, int npairs, const G1Aff* P, PairLines L,
                                               const Fq12* fmul, const uint32_t* status, int do_final,
                                               Fq12* f_out, int32_t* result) {
  size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  if (status && status[k]) {
    if (result) result[k] = 0;
    return;
  }
  Fq px[4], py[4];
  bool skip[4];
  const LineCoef* lines[4];
  for (int i = 0; i < npairs; i++) {
    G1Aff p = P[k * npairs + i];
    px[i] = p.x;
    py[i] = p.y;
    skip[i] = aff_is_inf(p);
    lines[i] = L.base[i] + k * L.stride[i];
  }
  Fq12 f = miller_prepared(npairs, px, py, lines, skip);
  if (fmul) f = f12_mul(f, *fmul);
  if (do_final) f = final_exp(f);
  if (f_out) f_out[k] = f;
  if (result) result[k] = f12_is_one(f) ? 1 : 0;
}

__global__ void k_fq12_to_std(size_t n, const Fq12* in, uint32_t* out) {
  size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const Fq2* c = reinterpret_cast<const Fq2*>(in + k);  // c0.c0, c0.c1, c0.c2, c1.c0, ... = toObject order
  for (int j = 0; j < 6; j++) {
    Fq a = fp_from_mont(c[j].c0), b = fp_from_mont(c[j].c1);
    for (int l = 0; l < 8; l++) {
      out[k * 96 + j * 16 + l] = a.v[l];
      out[k * 96 + j * 16 + 8 + l] = b.v[l];
    }
  }
}

int hip_err(hipError_t e, const char* where, std::string& err) {
  err = std::string(where) + ": " + hipGetErrorString(e);
  return e == hipErrorOutOfMemory ? ZKFL_E_OOM : ZKFL_E_DEVICE;
}

template <class T>
hipError_t dalloc(T** p, size_t count) {
  return hipMalloc((void**)p, count * sizeof(T) + 16);
}

}  // namespace

struct VkDev {
  std::vector<uint8_t> bytes;
  uint32_t npub = 0;
  G1Aff* ic_table = nullptr;  // (npub+1) x 16; index 1 of row 0 = IC0
  LineCoef* lines = nullptr;  // [3][ATE_NLINES]: beta2, gamma2, delta2
  Fq12* f_ab = nullptr;       // Miller value of (alpha1, beta2), Montgomery
  G1Aff* alpha = nullptr;
};

void vk_free(VkDev* vk) {
  if (!vk) return;
  for (void* p : {(void*)vk->ic_table, (void*)vk->lines, (void*)vk->f_ab, (void*)vk->alpha})
    if (p) (void)hipFree(p);
  delete vk;
}

bool vk_same(const VkDev* vk, const uint8_t* bytes, size_t len) {
  return vk && vk->bytes.size() == len && memcmp(vk->bytes.data(), bytes, len) == 0;
}

uint32_t vk_npub(const VkDev* vk) { return vk->npub; }

int vk_prepare(const uint8_t* vkb, size_t len, hipStream_t st, VkDev** out, std::string& err) {
  if (!vkb || len < 4 + 448 + 64) {
    err = "verification key: truncated";
    return ZKFL_E_FORMAT;
  }
  uint32_t npub;
  memcpy(&npub, vkb, 4);
  if (npub > (1u << 20) || len != 4 + 448 + 64ull * (npub + 1)) {
    err = "verification key: length does not match nPublic";
    return ZKFL_E_FORMAT;
  }
  VkDev* vk = new VkDev();
  vk->bytes.assign(vkb, vkb + len);
  vk->npub = npub;
  uint32_t* d_in = nullptr;   // the vk image without the count (u32 aligned)
  uint32_t* d_stat = nullptr; // [npub+1 IC | 3 G2 | 1 alpha]
  int rc = ZKFL_OK;
  const size_t nwords = (len - 4) / 4;
  hipError_t e = dalloc(&d_in, nwords);
  if (e == hipSuccess) e = dalloc(&d_stat, npub + 5);
  if (e == hipSuccess) e = dalloc(&vk->ic_table, (size_t)(npub + 1) * 16);
  if (e == hipSuccess) e = dalloc(&vk->lines, 3 * (size_t)ATE_NLINES);
  if (e == hipSuccess) e = dalloc(&vk->f_ab, 1);
  if (e == hipSuccess) e = dalloc(&vk->alpha, 1);
  if (e == hipSuccess) e = hipMemcpyAsync(d_in, vkb + 4, len - 4, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemsetAsync(d_stat, 0, (npub + 5) * 4, st);
  if (e == hipSuccess) {
    // layout (u32 words): alpha1 [0,16) beta2 [16,48) gamma2 [48,80) delta2 [80,112) IC [112, ...)
    hipLaunchKernelGGL(k_ic_tables, dim3(zk_grid(npub + 1, 64)), dim3(64), 0, st, npub + 1, d_in + 112,
                       vk->ic_table, d_stat);
    hipLaunchKernelGGL(k_g2_prepare, dim3(1), dim3(64), 0, st, (size_t)3, d_in + 16, (size_t)32, 1, vk->lines,
                       d_stat + npub + 1);
    hipLaunchKernelGGL(k_g1_load, dim3(1), dim3(64), 0, st, (size_t)1, d_in, vk->alpha, d_stat + npub + 4);
    PairLines L = {};
    L.base[0] = vk->lines;  // beta2
    hipLaunchKernelGGL(k_miller, dim3(1), dim3(64), 0, st, (size_t)1, 1, (const G1Aff*)vk->alpha, L,
                       (const Fq12*)nullptr, (const uint32_t*)nullptr, 0, vk->f_ab, (int32_t*)nullptr);
    e = hipGetLastError();
  }
  std::vector<uint32_t> stat(npub + 5);
  if (e == hipSuccess) e = hipMemcpyAsync(stat.data(), d_stat, (npub + 5) * 4, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) {
    rc = hip_err(e, "vk_prepare", err);
  } else {
    for (uint32_t i = 0; i < npub + 5 && rc == ZKFL_OK; i++) {
      // IC entries may be infinity; alpha/beta/gamma/delta must be proper points
      bool bad = (stat[i] & ST_BAD) || (i > npub && stat[i] != 0);
      if (bad) {
        err = "verification key: point off curve / not in subgroup / at infinity";
        rc = ZKFL_E_FORMAT;
      }
    }
  }
  if (d_in) (void)hipFree(d_in);
  if (d_stat) (void)hipFree(d_stat);
  if (rc != ZKFL_OK) {
    vk_free(vk);
    return rc;
  }
  *out = vk;
  return ZKFL_OK;
}

int verify_batch(const VkDev* vk, size_t n, const uint8_t* pubs, const uint8_t* proofs, int32_t* results,
                 hipStream_t st, std::string& err) {
  if (n == 0) return ZKFL_OK;
  const size_t CH = 4096;  // proofs per chunk: 4096 x 102 lines x 192 B = 80 MB of lines
  const size_t cap = n < CH ? n : CH;
  const uint32_t npub = vk->npub;
  uint32_t *d_pub = nullptr, *d_proof = nullptr, *d_bstat = nullptr, *d_status = nullptr;
  LineCoef* d_lines = nullptr;
  G1Aff* d_P = nullptr;
  int32_t* d_res = nullptr;
  hipError_t e = dalloc(&d_pub, cap * npub * 8);
  if (e == hipSuccess) e = dalloc(&d_proof, cap * 64);
  if (e == hipSuccess) e = dalloc(&d_bstat, cap);
  if (e == hipSuccess) e = dalloc(&d_status, cap);
  if (e == hipSuccess) e = dalloc(&d_lines, cap * ATE_NLINES);
  if (e == hipSuccess) e = dalloc(&d_P, cap * 3);
  if (e == hipSuccess) e = dalloc(&d_res, cap);
  for (size_t off = 0; off < n && e == hipSuccess; off += cap) {
    size_t m = (n - off < cap) ? n - off : cap;
    if (npub) e = hipMemcpyAsync(d_pub, pubs + off * npub * 32, m * npub * 32, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipMemcpyAsync(d_proof, proofs + off * 256, m * 256, hipMemcpyHostToDevice, st);
    if (e != hipSuccess) break;
    unsigned g = zk_grid(m, 64);
    hipLaunchKernelGGL(k_g2_prepare, dim3(g), dim3(64), 0, st, m, d_proof + 16, (size_t)64, 1, d_lines, d_bstat);
    hipLaunchKernelGGL(k_verify_inputs, dim3(g), dim3(64), 0, st, m, npub, d_pub, d_proof,
                       (const G1Aff*)vk->ic_table, d_bstat, d_P, d_status);
    PairLines L = {};
    L.base[0] = d_lines;
    L.stride[0] = ATE_NLINES;
    L.base[1] = vk->lines + ATE_NLINES;  // gamma2
    L.base[2] = vk->lines + 2 * ATE_NLINES;  // delta2
    hipLaunchKernelGGL(k_miller, dim3(g), dim3(64), 0, st, m, 3, (const G1Aff*)d_P, L, (const Fq12*)vk->f_ab,
                       (const uint32_t*)d_status, 1, (Fq12*)nullptr, d_res);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(results + off, d_res, m * 4, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
  }
  int rc = (e == hipSuccess) ? ZKFL_OK : hip_err(e, "verify_batch", err);
  for (void* p : {(void*)d_pub, (void*)d_proof, (void*)d_bstat, (void*)d_status, (void*)d_lines, (void*)d_P,
                  (void*)d_res})
    if (p) (void)hipFree(p);
  return rc;
}

int pairing_batch(size_t n, const uint8_t* g1, const uint8_t* g2, int final_exp, uint8_t* out, hipStream_t st,
                  std::string& err) {
  if (n == 0) return ZKFL_OK;
  uint32_t *d_g1 = nullptr, *d_g2 = nullptr, *d_stat = nullptr, *d_out = nullptr;
  LineCoef* d_lines = nullptr;
  G1Aff* d_P = nullptr;
  Fq12* d_f = nullptr;
  hipError_t e = dalloc(&d_g1, n * 16);
  if (e == hipSuccess) e = dalloc(&d_g2, n * 32);
  if (e == hipSuccess) e = dalloc(&d_stat, 2 * n);
  if (e == hipSuccess) e = dalloc(&d_lines, n * ATE_NLINES);
  if (e == hipSuccess) e = dalloc(&d_P, n);
  if (e == hipSuccess) e = dalloc(&d_f, n);
  if (e == hipSuccess) e = dalloc(&d_out, n * 96);
  if (e == hipSuccess) e = hipMemcpyAsync(d_g1, g1, n * 64, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(d_g2, g2, n * 128, hipMemcpyHostToDevice, st);
  std::vector<uint32_t> stat(2 * n);
  if (e == hipSuccess) {
    unsigned g = zk_grid(n, 64);
    hipLaunchKernelGGL(k_g1_load, dim3(g), dim3(64), 0, st, n, d_g1, d_P, d_stat);
    hipLaunchKernelGGL(k_g2_prepare, dim3(g), dim3(64), 0, st, n, d_g2, (size_t)32, 1, d_lines, d_stat + n);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(stat.data(), d_stat, 2 * n * 4, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  int rc = ZKFL_OK;
  if (e == hipSuccess) {
    for (size_t i = 0; i < 2 * n; i++)
      if (stat[i] & ST_BAD) {
        err = "pairing: point " + std::to_string(i % n) + (i < n ? " (G1)" : " (G2)") +
              " is not canonical / not on the curve / not in the subgroup";
        rc = ZKFL_E_ARG;
        break;
      }
    // a G2 point at infinity: mark the G1 side as infinity so the pair contributes 1
    for (size_t i = 0; i < n && rc == ZKFL_OK; i++)
      if (stat[n + i] == ST_INF) e = hipMemsetAsync(d_P + i, 0, sizeof(G1Aff), st);
  }
  if (rc == ZKFL_OK && e == hipSuccess) {
    unsigned g = zk_grid(n, 64);
    PairLines L = {};
    L.base[0] = d_lines;
    L.stride[0] = ATE_NLINES;
    hipLaunchKernelGGL(k_miller, dim3(g), dim3(64), 0, st, n, 1, (const G1Aff*)d_P, L, (const Fq12*)nullptr,
                       (const uint32_t*)nullptr, final_exp, d_f, (int32_t*)nullptr);
    hipLaunchKernelGGL(k_fq12_to_std, dim3(g), dim3(64), 0, st, n, (const Fq12*)d_f, d_out);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(out, d_out, n * 384, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
  }
  if (rc == ZKFL_OK && e != hipSuccess) rc = hip_err(e, "pairing_batch", err);
  for (void* p : {(void*)d_g1, (void*)d_g2, (void*)d_stat, (void*)d_lines, (void*)d_P, (void*)d_f, (void*)d_out})
    if (p) (void)hipFree(p);
  return rc;
}

}  // namespace zkfl
