/*
 * groth16_ref.c — CPU restatement of snarkjs `groth16 prove` over BN254 (TEST INFRASTRUCTURE).
 *
 * Oracle only: linked/loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg, never by the product.  Restates (third-party, absent from /root/reference):
 *   snarkjs ^0.7.5 groth16_prove: buildABC1 -> ifft/batchApplyKey/fft (x3) -> joinABC ->
 *   multiExpAffine A, B1, B2, C, H -> assembly with r, s   (call site
 *   tests/full_system_simulation.mjs:773-776), on ffjavascript ^0.2.63 bn128 arithmetic.
 * Same algorithm as oracle/groth16.py (the pure-Python restatement it is tested against),
 * written for speed: 4 x 64-bit Montgomery limbs, Jacobian coordinates, Pippenger with one
 * OpenMP task per window, iterative radix-2 NTT.
 *
 * Exported: ref_prove(zkey, zkey_len, wtns, wtns_len, rs(64 B) , proof_out(256 B), threads)
 *           -> 0 ok / <0 error.   Proof layout = include/zkfl.h (std affine, LE).
 */
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef struct { uint64_t v[4]; } fe;

static const uint64_t QP[4] = {0x3c208c16d87cfd47ull, 0x97816a916871ca8dull, 0xb85045b68181585dull, 0x30644e72e131a029ull};
static const uint64_t RP[4] = {0x43e1f593f0000001ull, 0x2833e84879b97091ull, 0xb85045b68181585dull, 0x30644e72e131a029ull};
static uint64_t QINV, RINV;   /* -p^-1 mod 2^64 */
static fe Q_ONE, R_ONE, Q_R2, R_R2;

static uint64_t neg_inv64(uint64_t p0) {
  uint64_t x = 1;
  for (int i = 0; i < 7; i++) x *= 2 - p0 * x;
  return (uint64_t)0 - x;
}

static inline int geq(const uint64_t* a, const uint64_t* p) {
  for (int i = 3; i >= 0; i--) {
    if (a[i] != p[i]) return a[i] > p[i];
  }
  return 1;
}

static inline void sub_p(uint64_t* a, const uint64_t* p) {
  u128 b = 0;
  for (int i = 0; i < 4; i++) {
    u128 d = (u128)a[i] - p[i] - b;
    a[i] = (uint64_t)d;
    b = (d >> 127) & 1;
  }
}

static inline void fadd(fe* r, const fe* a, const fe* b, const uint64_t* p) {
  u128 c = 0;
  for (int i = 0; i < 4; i++) {
    c += (u128)a->v[i] + b->v[i];
    r->v[i] = (uint64_t)c;
    c >>= 64;
  }
  if (c || geq(r->v, p)) sub_p(r->v, p);
}

static inline void fsub(fe* r, const fe* a, const fe* b, const uint64_t* p) {
  u128 bw = 0;
  uint64_t t[4];
  for (int i = 0; i < 4; i++) {
    u128 d = (u128)a->v[i] - b->v[i] - bw;
    t[i] = (uint64_t)d;
    bw = (d >> 127) & 1;
  }
  if (bw) {
    u128 c = 0;
    for (int i = 0; i < 4; i++) {
      c += (u128)t[i] + p[i];
      t[i] = (uint64_t)c;
      c >>= 64;
    }
  }
  memcpy(r->v, t, 32);
}

static inline void fmul(fe* r, const fe* a, const fe* b, const uint64_t* p, uint64_t inv) {
  uint64_t t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; i++) {
    u128 c = 0;
    for (int j = 0; j < 4; j++) {
      c += (u128)a->v[j] * b->v[i] + t[j];
      t[j] = (uint64_t)c;
      c >>= 64;
    }
    c += t[4];
    t[4] = (uint64_t)c;
    t[5] = (uint64_t)(c >> 64);
    uint64_t m = t[0] * inv;
    c = (u128)m * p[0] + t[0];
    c >>= 64;
    for (int j = 1; j < 4; j++) {
      c += (u128)m * p[j] + t[j];
      t[j - 1] = (uint64_t)c;
      c >>= 64;
    }
    c += t[4];
    t[3] = (uint64_t)c;
    t[4] = t[5] + (uint64_t)(c >> 64);
  }
  if (t[4] || geq(t, p)) sub_p(t, p);
  memcpy(r->v, t, 32);
}

#define QADD(r, a, b) fadd(r, a, b, QP)
#define QSUB(r, a, b) fsub(r, a, b, QP)
#define QMUL(r, a, b) fmul(r, a, b, QP, QINV)
#define RADD(r, a, b) fadd(r, a, b, RP)
#define RSUB(r, a, b) fsub(r, a, b, RP)
#define RMUL(r, a, b) fmul(r, a, b, RP, RINV)

static inline int fe_zero(const fe* a) { return !(a->v[0] | a->v[1] | a->v[2] | a->v[3]); }

static void fpow(fe* r, const fe* a, const uint64_t* e, const uint64_t* p, uint64_t inv, const fe* one) {
  fe acc = *one;
  for (int i = 3; i >= 0; i--)
    for (int b = 63; b >= 0; b--) {
      fmul(&acc, &acc, &acc, p, inv);
      if ((e[i] >> b) & 1) fmul(&acc, &acc, a, p, inv);
    }
  *r = acc;
}

static void qinv(fe* r, const fe* a) {
  uint64_t e[4];
  memcpy(e, QP, 32);
  e[0] -= 2;
  fpow(r, a, e, QP, QINV, &Q_ONE);
}

static void init_consts(void) {
  static int done = 0;
  if (done) return;
  QINV = neg_inv64(QP[0]);
  RINV = neg_inv64(RP[0]);
  /* R mod p and R^2 mod p by doubling */
  for (int w = 0; w < 2; w++) {
    const uint64_t* p = w ? RP : QP;
    fe x = {{1, 0, 0, 0}};
    for (int i = 0; i < 512; i++) {
      fadd(&x, &x, &x, p);
      if (i == 255) *(w ? &R_ONE : &Q_ONE) = x;
    }
    *(w ? &R_R2 : &Q_R2) = x;
  }
  done = 1;
}

/* ---------------- Fq2 ---------------- */
typedef struct { fe c0, c1; } fe2;
static inline void f2add(fe2* r, const fe2* a, const fe2* b) { QADD(&r->c0, &a->c0, &b->c0); QADD(&r->c1, &a->c1, &b->c1); }
static inline void f2sub(fe2* r, const fe2* a, const fe2* b) { QSUB(&r->c0, &a->c0, &b->c0); QSUB(&r->c1, &a->c1, &b->c1); }
static inline void f2mul(fe2* r, const fe2* a, const fe2* b) {
  fe t0, t1, t2, s0, s1;
  QMUL(&t0, &a->c0, &b->c0);
  QMUL(&t1, &a->c1, &b->c1);
  QADD(&s0, &a->c0, &a->c1);
  QADD(&s1, &b->c0, &b->c1);
  QMUL(&t2, &s0, &s1);
  QSUB(&r->c0, &t0, &t1);
  QSUB(&t2, &t2, &t0);
  QSUB(&r->c1, &t2, &t1);
}
static inline int f2zero(const fe2* a) { return fe_zero(&a->c0) && fe_zero(&a->c1); }
static void f2inv(fe2* r, const fe2* a) {
  fe n, t, ni;
  QMUL(&n, &a->c0, &a->c0);
  QMUL(&t, &a->c1, &a->c1);
  QADD(&n, &n, &t);
  qinv(&ni, &n);
  QMUL(&r->c0, &a->c0, &ni);
  fe z = {{0}};
  QMUL(&t, &a->c1, &ni);
  QSUB(&r->c1, &z, &t);
}

/* ---------------- generic Jacobian arithmetic via macros over (F, ADD, SUB, MUL, ZERO) ---------------- */
#define DEFINE_CURVE(NAME, F, ADD, SUB, MUL, ISZERO)                                           \
  typedef struct { F X, Y, Z; } NAME##_jac;                                                    \
  typedef struct { F x, y; } NAME##_aff;                                                       \
  static inline int NAME##_is_inf(const NAME##_jac* p) { return ISZERO(&p->Z); }              \
  static void NAME##_dbl(NAME##_jac* r, const NAME##_jac* p) {                                 \
    if (NAME##_is_inf(p) || ISZERO(&p->Y)) { memset(r, 0, sizeof(*r)); return; }              \
    F A, B, C, D, E, Fv, t, X3, Y3, Z3;                                                         \
    MUL(&A, &p->X, &p->X);                                                                     \
    MUL(&B, &p->Y, &p->Y);                                                                     \
    MUL(&C, &B, &B);                                                                           \
    ADD(&t, &p->X, &B);                                                                        \
    MUL(&D, &t, &t);                                                                           \
    SUB(&D, &D, &A);                                                                           \
    SUB(&D, &D, &C);                                                                           \
    ADD(&D, &D, &D);                                                                           \
    ADD(&E, &A, &A);                                                                           \
    ADD(&E, &E, &A);                                                                           \
    MUL(&Fv, &E, &E);                                                                          \
    ADD(&t, &D, &D);                                                                           \
    SUB(&X3, &Fv, &t);                                                                         \
    SUB(&t, &D, &X3);                                                                          \
    MUL(&Y3, &E, &t);                                                                          \
    ADD(&C, &C, &C);                                                                           \
    ADD(&C, &C, &C);                                                                           \
    ADD(&C, &C, &C);                                                                           \
    SUB(&Y3, &Y3, &C);                                                                         \
    MUL(&Z3, &p->Y, &p->Z);                                                                    \
    ADD(&Z3, &Z3, &Z3);                                                                        \
    r->X = X3; r->Y = Y3; r->Z = Z3;                                                           \
  }                                                                                            \
  static void NAME##_add(NAME##_jac* r, const NAME##_jac* p, const NAME##_jac* q) {            \
    if (NAME##_is_inf(p)) { *r = *q; return; }                                                 \
    if (NAME##_is_inf(q)) { *r = *p; return; }                                                 \
    F Z1Z1, Z2Z2, U1, U2, S1, S2, H, Rr, H2, H3, U1H2, t, X3, Y3, Z3;                           \
    MUL(&Z1Z1, &p->Z, &p->Z);                                                                  \
    MUL(&Z2Z2, &q->Z, &q->Z);                                                                  \
    MUL(&U1, &p->X, &Z2Z2);                                                                    \
    MUL(&U2, &q->X, &Z1Z1);                                                                    \
    MUL(&t, &p->Y, &q->Z);                                                                     \
    MUL(&S1, &t, &Z2Z2);                                                                       \
    MUL(&t, &q->Y, &p->Z);                                                                     \
    MUL(&S2, &t, &Z1Z1);                                                                       \
    SUB(&H, &U2, &U1);                                                                         \
    SUB(&Rr, &S2, &S1);                                                                        \
    if (ISZERO(&H)) {                                                                          \
      if (ISZERO(&Rr)) { NAME##_dbl(r, p); return; }                                           \
      memset(r, 0, sizeof(*r));                                                                \
      return;                                                                                  \
    }                                                                                          \
    MUL(&H2, &H, &H);                                                                          \
    MUL(&H3, &H2, &H);                                                                         \
    MUL(&U1H2, &U1, &H2);                                                                      \
    MUL(&X3, &Rr, &Rr);                                                                        \
    SUB(&X3, &X3, &H3);                                                                        \
    SUB(&X3, &X3, &U1H2);                                                                      \
    SUB(&X3, &X3, &U1H2);                                                                      \
    SUB(&t, &U1H2, &X3);                                                                       \
    MUL(&Y3, &Rr, &t);                                                                         \
    MUL(&t, &S1, &H3);                                                                         \
    SUB(&Y3, &Y3, &t);                                                                         \
    MUL(&t, &p->Z, &q->Z);                                                                     \
    MUL(&Z3, &t, &H);                                                                          \
    r->X = X3; r->Y = Y3; r->Z = Z3;                                                           \
  }

static inline int qzero(const fe* a) { return fe_zero(a); }
DEFINE_CURVE(g1, fe, QADD, QSUB, QMUL, qzero)
DEFINE_CURVE(g2, fe2, f2add, f2sub, f2mul, f2zero)

static void g1_from_aff(g1_jac* r, const g1_aff* a) {
  if (fe_zero(&a->x) && fe_zero(&a->y)) { memset(r, 0, sizeof(*r)); return; }
  r->X = a->x; r->Y = a->y; r->Z = Q_ONE;
}
static void g2_from_aff(g2_jac* r, const g2_aff* a) {
  if (f2zero(&a->x) && f2zero(&a->y)) { memset(r, 0, sizeof(*r)); return; }
  r->X = a->x; r->Y = a->y; r->Z.c0 = Q_ONE; memset(&r->Z.c1, 0, 32);
}

/* ---------------- Pippenger (unsigned windows; one OpenMP task per window) ---------------- */
#define DEFINE_MSM(NAME)                                                                        \
  static void NAME##_msm(NAME##_jac* out, const NAME##_aff* bases, const fe* sc, size_t n) {    \
    int c = 2;                                                                                  \
    while (c < 16 && ((size_t)1 << (c + 2)) < n) c++;                                           \
    int W = (254 + c - 1) / c;                                                                  \
    NAME##_jac* win = calloc((size_t)W, sizeof(NAME##_jac));                                    \
    _Pragma("omp parallel for schedule(dynamic, 1)")                                             \
    for (int w = 0; w < W; w++) {                                                               \
      size_t nb = ((size_t)1 << c);                                                             \
      NAME##_jac* bk = calloc(nb, sizeof(NAME##_jac));                                          \
      for (size_t i = 0; i < n; i++) {                                                          \
        int bit = w * c;                                                                        \
        uint64_t d = sc[i].v[bit >> 6] >> (bit & 63);                                           \
        if ((bit & 63) + c > 64 && (bit >> 6) < 3) d |= sc[i].v[(bit >> 6) + 1] << (64 - (bit & 63)); \
        d &= nb - 1;                                                                            \
        if (!d) continue;                                                                       \
        NAME##_jac P;                                                                           \
        NAME##_from_aff(&P, &bases[i]);                                                         \
        if (NAME##_is_inf(&P)) continue;                                                        \
        NAME##_add(&bk[d], &bk[d], &P);                                                         \
      }                                                                                         \
      NAME##_jac run, acc;                                                                      \
      memset(&run, 0, sizeof run);                                                              \
      memset(&acc, 0, sizeof acc);                                                              \
      for (size_t d = nb - 1; d >= 1; d--) {                                                    \
        NAME##_add(&run, &run, &bk[d]);                                                         \
        NAME##_add(&acc, &acc, &run);                                                           \
      }                                                                                         \
      win[w] = acc;                                                                             \
      free(bk);                                                                                 \
    }                                                                                           \
    NAME##_jac tot;                                                                             \
    memset(&tot, 0, sizeof tot);                                                                \
    for (int w = W - 1; w >= 0; w--) {                                                          \
      for (int k = 0; k < c; k++) NAME##_dbl(&tot, &tot);                                       \
      NAME##_add(&tot, &tot, &win[w]);                                                          \
    }                                                                                           \
    *out = tot;                                                                                 \
    free(win);                                                                                  \
  }
DEFINE_MSM(g1)
DEFINE_MSM(g2)

static void g1_mul_scalar(g1_jac* r, const g1_jac* p, const fe* k) {
  g1_jac acc;
  memset(&acc, 0, sizeof acc);
  for (int i = 3; i >= 0; i--)
    for (int b = 63; b >= 0; b--) {
      g1_dbl(&acc, &acc);
      if ((k->v[i] >> b) & 1) g1_add(&acc, &acc, p);
    }
  *r = acc;
}

/* ---------------- NTT (Montgomery Fr) ---------------- */
static void r_pow_u64(fe* r, const fe* a, uint64_t e) {
  fe acc = R_ONE, b = *a;
  while (e) {
    if (e & 1) RMUL(&acc, &acc, &b);
    RMUL(&b, &b, &b);
    e >>= 1;
  }
  *r = acc;
}

static void ntt(fe* a, size_t n, const fe* root_mont) {
  int logn = 0;
  while (((size_t)1 << logn) < n) logn++;
  for (size_t i = 1, j = 0; i < n; i++) {
    size_t bit = n >> 1;
    for (; j & bit; bit >>= 1) j ^= bit;
    j ^= bit;
    if (i < j) { fe t = a[i]; a[i] = a[j]; a[j] = t; }
  }
  fe* tw = malloc((n / 2 + 1) * sizeof(fe));
  tw[0] = R_ONE;
  for (size_t i = 1; i < n / 2; i++) RMUL(&tw[i], &tw[i - 1], root_mont);
  for (size_t len = 2; len <= n; len <<= 1) {
    size_t half = len >> 1, step = n / len;
#pragma omp parallel for schedule(static)
    for (size_t k = 0; k < n / 2; k++) {
      size_t blk = k / half, j = k % half;
      size_t i0 = blk * len + j, i1 = i0 + half;
      fe t, u = a[i0];
      RMUL(&t, &a[i1], &tw[j * step]);
      RADD(&a[i0], &u, &t);
      RSUB(&a[i1], &u, &t);
    }
  }
  free(tw);
}

/* roots (std form) computed at init: w[28] = 5^t */
static fe root_std(int power, int inverse) {
  fe five = {{5, 0, 0, 0}}, x;
  RMUL(&five, &five, &R_R2);          /* to mont */
  /* t = (r-1) >> 28 */
  uint64_t t[4];
  memcpy(t, RP, 32);
  t[0] -= 1;
  for (int s = 0; s < 28; s++) {
    t[0] = (t[0] >> 1) | (t[1] << 63);
    t[1] = (t[1] >> 1) | (t[2] << 63);
    t[2] = (t[2] >> 1) | (t[3] << 63);
    t[3] >>= 1;
  }
  fpow(&x, &five, t, RP, RINV, &R_ONE);
  for (int s = 28; s > power; s--) RMUL(&x, &x, &x);
  if (inverse) {
    uint64_t e[4];
    memcpy(e, RP, 32);
    e[0] -= 2;
    fpow(&x, &x, e, RP, RINV, &R_ONE);
  }
  return x; /* mont */
}

/* ---------------- zkey / wtns parsing ---------------- */
typedef struct { const uint8_t* p; uint64_t size; } sec_t;

static int parse_bin(const uint8_t* b, size_t len, const char* magic, sec_t* secs, int maxs) {
  if (len < 12 || memcmp(b, magic, 4)) return -2;
  uint32_t ns;
  memcpy(&ns, b + 8, 4);
  size_t off = 12;
  memset(secs, 0, sizeof(sec_t) * maxs);
  for (uint32_t i = 0; i < ns; i++) {
    uint32_t t;
    uint64_t sz;
    if (off + 12 > len) return -2;
    memcpy(&t, b + off, 4);
    memcpy(&sz, b + off + 4, 8);
    off += 12;
    if (off + sz > len) return -2;
    if ((int)t < maxs && !secs[t].p) { secs[t].p = b + off; secs[t].size = sz; }
    off += sz;
  }
  return 0;
}

static void to_mont_r(fe* x) { RMUL(x, x, &R_R2); }
static void from_mont_r(fe* x) { fe one = {{1, 0, 0, 0}}; RMUL(x, x, &one); }
static void from_mont_q(fe* x) { fe one = {{1, 0, 0, 0}}; QMUL(x, x, &one); }

static void g1_to_std_aff(uint8_t* out, const g1_jac* p) {
  if (g1_is_inf(p)) { memset(out, 0, 64); return; }
  fe zi, zi2, zi3, x, y;
  qinv(&zi, &p->Z);
  QMUL(&zi2, &zi, &zi);
  QMUL(&zi3, &zi2, &zi);
  QMUL(&x, &p->X, &zi2);
  QMUL(&y, &p->Y, &zi3);
  from_mont_q(&x);
  from_mont_q(&y);
  memcpy(out, x.v, 32);
  memcpy(out + 32, y.v, 32);
}

static void g2_to_std_aff(uint8_t* out, const g2_jac* p) {
  if (g2_is_inf(p)) { memset(out, 0, 128); return; }
  fe2 zi, zi2, zi3, x, y;
  f2inv(&zi, &p->Z);
  f2mul(&zi2, &zi, &zi);
  f2mul(&zi3, &zi2, &zi);
  f2mul(&x, &p->X, &zi2);
  f2mul(&y, &p->Y, &zi3);
  from_mont_q(&x.c0); from_mont_q(&x.c1); from_mont_q(&y.c0); from_mont_q(&y.c1);
  memcpy(out, x.c0.v, 32); memcpy(out + 32, x.c1.v, 32);
  memcpy(out + 64, y.c0.v, 32); memcpy(out + 96, y.c1.v, 32);
}

/* Full proof plus the deterministic core for parity checks: h_out (n x 32 B std, the H-MSM
 * scalars) and msm_out (A 64 | B1 64 | B2 128 | C 64 | H 64, std affine, without the
 * alpha/beta/delta/r/s terms), both nullable: the layout of zkfl_debug_prove_parts. */
int ref_prove_ex(const uint8_t* zk, size_t zlen, const uint8_t* wt, size_t wlen, const uint8_t* rs, uint8_t* proof,
                 int threads, uint8_t* h_out, uint8_t* msm_out) {
  init_consts();
  if (threads > 0) omp_set_num_threads(threads);
  sec_t s[16], w[4];
  if (parse_bin(zk, zlen, "zkey", s, 16) || parse_bin(wt, wlen, "wtns", w, 4)) return -2;
  const uint8_t* h = s[2].p;
  uint32_t nVars, nPub, n;
  memcpy(&nVars, h + 72, 4);
  memcpy(&nPub, h + 76, 4);
  memcpy(&n, h + 80, 4);
  const uint8_t* pts = h + 84;
  uint32_t nw;
  memcpy(&nw, w[1].p + 36, 4);
  if (nw != nVars) return -4;
  const fe* wit = (const fe*)w[2].p;   /* std form */
  int power = 0;
  while ((1u << power) < n) power++;

  /* ABC (Montgomery): coef raw = coef*R^2, mont_mul(raw, w_std) = coef*w in mont */
  fe* abc = calloc((size_t)3 * n, sizeof(fe));
  fe *A = abc, *B = abc + n, *C = abc + 2 * (size_t)n;
  uint32_t nc;
  memcpy(&nc, s[4].p, 4);
  for (uint32_t i = 0; i < nc; i++) {
    const uint8_t* e = s[4].p + 4 + (size_t)i * 44;
    uint32_t m, c, sg;
    memcpy(&m, e, 4); memcpy(&c, e + 4, 4); memcpy(&sg, e + 8, 4);
    fe coef, t;
    memcpy(coef.v, e + 12, 32);
    RMUL(&t, &coef, &wit[sg]);
    fe* dst = m ? &B[c] : &A[c];
    RADD(dst, dst, &t);
  }
  for (uint32_t i = 0; i < n; i++) RMUL(&C[i], &A[i], &B[i]);

  /* coset evaluations */
  fe wf = root_std(power, 0), wi = root_std(power, 1);
  fe inc = power == 28 ? (fe){{25, 0, 0, 0}} : root_std(power + 1, 0);
  if (power == 28) to_mont_r(&inc);
  fe ninv = {{n, 0, 0, 0}};
  to_mont_r(&ninv);
  {
    uint64_t e[4];
    memcpy(e, RP, 32);
    e[0] -= 2;
    fpow(&ninv, &ninv, e, RP, RINV, &R_ONE);
  }
  for (int v = 0; v < 3; v++) {
    fe* x = abc + (size_t)v * n;
    ntt(x, n, &wi);
#pragma omp parallel for schedule(static)
    for (uint32_t i = 0; i < n; i++) {
      fe f;
      r_pow_u64(&f, &inc, i);
      RMUL(&f, &f, &ninv);
      RMUL(&x[i], &x[i], &f);
    }
    ntt(x, n, &wf);
  }
  fe* hs = malloc((size_t)n * sizeof(fe));
#pragma omp parallel for schedule(static)
  for (uint32_t i = 0; i < n; i++) {
    fe t;
    RMUL(&t, &A[i], &B[i]);
    RSUB(&hs[i], &t, &C[i]);
    from_mont_r(&hs[i]);
  }
  free(abc);
  if (h_out) memcpy(h_out, hs, (size_t)n * 32);

  /* MSMs */
  g1_jac mA, mB1, mC, mH;
  g2_jac mB2;
  g1_msm(&mA, (const g1_aff*)s[5].p, wit, nVars);
  g1_msm(&mB1, (const g1_aff*)s[6].p, wit, nVars);
  g2_msm(&mB2, (const g2_aff*)s[7].p, wit, nVars);
  g1_msm(&mC, (const g1_aff*)s[8].p, wit + nPub + 1, nVars - nPub - 1);
  g1_msm(&mH, (const g1_aff*)s[9].p, hs, n);
  free(hs);
  if (msm_out) {
    g1_to_std_aff(msm_out, &mA);
    g1_to_std_aff(msm_out + 64, &mB1);
    g2_to_std_aff(msm_out + 128, &mB2);
    g1_to_std_aff(msm_out + 256, &mC);
    g1_to_std_aff(msm_out + 320, &mH);
  }

  /* assembly */
  fe r, sv;
  memcpy(r.v, rs, 32);
  memcpy(sv.v, rs + 32, 32);
  g1_jac alpha1, beta1, delta1, t1;
  g2_jac beta2, delta2, t2;
  g1_from_aff(&alpha1, (const g1_aff*)(pts));
  g1_from_aff(&beta1, (const g1_aff*)(pts + 64));
  g2_from_aff(&beta2, (const g2_aff*)(pts + 128));
  g1_from_aff(&delta1, (const g1_aff*)(pts + 384));
  g2_from_aff(&delta2, (const g2_aff*)(pts + 448));
  g1_jac pa, pb1, pc;
  g2_jac pb;
  g1_add(&pa, &mA, &alpha1);
  g1_mul_scalar(&t1, &delta1, &r);
  g1_add(&pa, &pa, &t1);
  /* pi_b = B2 + beta2 + s*delta2 (G2 scalar mul by double-and-add) */
  {
    g2_jac acc;
    memset(&acc, 0, sizeof acc);
    for (int i = 3; i >= 0; i--)
      for (int b = 63; b >= 0; b--) {
        g2_dbl(&acc, &acc);
        if ((sv.v[i] >> b) & 1) g2_add(&acc, &acc, &delta2);
      }
    t2 = acc;
  }
  g2_add(&pb, &mB2, &beta2);
  g2_add(&pb, &pb, &t2);
  g1_add(&pb1, &mB1, &beta1);
  g1_mul_scalar(&t1, &delta1, &sv);
  g1_add(&pb1, &pb1, &t1);
  g1_add(&pc, &mC, &mH);
  g1_mul_scalar(&t1, &pa, &sv);
  g1_add(&pc, &pc, &t1);
  g1_mul_scalar(&t1, &pb1, &r);
  g1_add(&pc, &pc, &t1);
  /* - r s delta1 */
  fe rm = r, sm = sv, rsv, z = {{0}};
  to_mont_r(&rm);
  to_mont_r(&sm);
  RMUL(&rsv, &rm, &sm);
  RSUB(&rsv, &z, &rsv);
  from_mont_r(&rsv);
  g1_mul_scalar(&t1, &delta1, &rsv);
  g1_add(&pc, &pc, &t1);
  g1_to_std_aff(proof, &pa);
  g2_to_std_aff(proof + 64, &pb);
  g1_to_std_aff(proof + 192, &pc);
  return 0;
}

int ref_prove(const uint8_t* zk, size_t zlen, const uint8_t* wt, size_t wlen, const uint8_t* rs, uint8_t* proof,
              int threads) {
  return ref_prove_ex(zk, zlen, wt, wlen, rs, proof, threads, NULL, NULL);
}

/* stand-alone MSM for cross-checks: bases mont affine, scalars std -> std affine out */
int ref_msm_g1(const uint8_t* bases, const uint8_t* scalars, size_t n, uint8_t* out, int threads) {
  init_consts();
  if (threads > 0) omp_set_num_threads(threads);
  g1_jac r;
  g1_msm(&r, (const g1_aff*)bases, (const fe*)scalars, n);
  g1_to_std_aff(out, &r);
  return 0;
}

/* fixed-base k*G (dev-ceremony backend for CPU tests): out = Montgomery affine, (0,0) = inf */
static void g1_to_mont_aff(uint8_t* out, const g1_jac* p) {
  if (g1_is_inf(p)) { memset(out, 0, 64); return; }
  fe zi, zi2, zi3, x, y;
  qinv(&zi, &p->Z);
  QMUL(&zi2, &zi, &zi);
  QMUL(&zi3, &zi2, &zi);
  QMUL(&x, &p->X, &zi2);
  QMUL(&y, &p->Y, &zi3);
  memcpy(out, x.v, 32);
  memcpy(out + 32, y.v, 32);
}

static void g2_to_mont_aff(uint8_t* out, const g2_jac* p) {
  if (g2_is_inf(p)) { memset(out, 0, 128); return; }
  fe2 zi, zi2, zi3, x, y;
  f2inv(&zi, &p->Z);
  f2mul(&zi2, &zi, &zi);
  f2mul(&zi3, &zi2, &zi);
  f2mul(&x, &p->X, &zi2);
  f2mul(&y, &p->Y, &zi3);
  memcpy(out, x.c0.v, 32); memcpy(out + 32, x.c1.v, 32);
  memcpy(out + 64, y.c0.v, 32); memcpy(out + 96, y.c1.v, 32);
}

static void q_to_mont(fe* x) { QMUL(x, x, &Q_R2); }

int ref_g1_gen_mul(const uint8_t* scalars, size_t n, uint8_t* out, int threads) {
  init_consts();
  if (threads > 0) omp_set_num_threads(threads);
  g1_jac G;
  memset(&G, 0, sizeof G);
  G.X.v[0] = 1; G.Y.v[0] = 2;
  q_to_mont(&G.X); q_to_mont(&G.Y);
  G.Z = Q_ONE;
#pragma omp parallel for schedule(dynamic, 16)
  for (size_t i = 0; i < n; i++) {
    g1_jac r;
    g1_mul_scalar(&r, &G, (const fe*)(scalars + 32 * i));
    g1_to_mont_aff(out + 64 * i, &r);
  }
  return 0;
}

int ref_g2_gen_mul(const uint8_t* scalars, size_t n, uint8_t* out, int threads) {
  init_consts();
  if (threads > 0) omp_set_num_threads(threads);
  static const uint64_t gx0[4] = {0x46debd5cd992f6edull, 0x674322d4f75edaddull, 0x426a00665e5c4479ull, 0x1800deef121f1e76ull};
  static const uint64_t gx1[4] = {0x97e485b7aef312c2ull, 0xf1aa493335a9e712ull, 0x7260bfb731fb5d25ull, 0x198e9393920d483aull};
  static const uint64_t gy0[4] = {0x4ce6cc0166fa7daaull, 0xe3d1e7690c43d37bull, 0x4aab71808dcb408full, 0x12c85ea5db8c6debull};
  static const uint64_t gy1[4] = {0x55acdadcd122975bull, 0xbc4b313370b38ef3ull, 0xec9e99ad690c3395ull, 0x090689d0585ff075ull};
  g2_jac G;
  memcpy(G.X.c0.v, gx0, 32); memcpy(G.X.c1.v, gx1, 32);
  memcpy(G.Y.c0.v, gy0, 32); memcpy(G.Y.c1.v, gy1, 32);
  q_to_mont(&G.X.c0); q_to_mont(&G.X.c1); q_to_mont(&G.Y.c0); q_to_mont(&G.Y.c1);
  G.Z.c0 = Q_ONE; memset(&G.Z.c1, 0, 32);
#pragma omp parallel for schedule(dynamic, 16)
  for (size_t i = 0; i < n; i++) {
    const fe* k = (const fe*)(scalars + 32 * i);
    g2_jac acc;
    memset(&acc, 0, sizeof acc);
    for (int w = 3; w >= 0; w--)
      for (int b = 63; b >= 0; b--) {
        g2_dbl(&acc, &acc);
        if ((k->v[w] >> b) & 1) g2_add(&acc, &acc, &G);
      }
    g2_to_mont_aff(out + 128 * i, &acc);
  }
  return 0;
}
