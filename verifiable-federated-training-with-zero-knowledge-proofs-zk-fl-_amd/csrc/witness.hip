// GPU witness generation: executes a compiled witness program (zkfl/wprog.py) for a batch of
// inputs.  Replaces circom's WASM witness calculator as the reference harness runs it
// (`node <c>_js/generate_witness.cjs <c>.wasm input.json out.wtns`,
// tests/full_system_simulation.mjs:758-767; `snarkjs wtns calculate`, tests/test_secureagg.cjs:108-118).
//
// Semantics per op (zkfl/r1cs.py Builder, circom --O2): LC  w[out] = <lc>;  MUL w[out] = <a><b>;
// INV w[out] = <x>^-1 (0 -> 0, circomlib IsZero hint);  BITS w[out+i] = bit i of <x> (Num2Bits
// hint);  POS: circomlib Poseidon permutation of [0, <in_0>, ...], writing (x^2, x^4, x^5) of
// every live S-box.  Then every assert constraint A*B = C is checked (circom aborts with
// "Assert Failed"; here ZKFL_E_CONSTRAINT).
//
// Schedule: ops are stored level by level (a level's ops only read wires of earlier levels);
// one launch per level, one lane per (witness, op); a final pass checks the asserts and writes
// the standard-form witness.  Independent of the circuit: the program image carries the linear
// combinations, the Poseidon templates and constants.
// Arithmetic: the 29-bit engine over Fr (fr29.h).  The wire vector, the coefficients and the
// Poseidon constants are kept as canonical x 2^261 (the image's 2^256 Montgomery coefficients
// and constants are converted once at load, k_wit_to_m261); a level of Poseidon permutations is
// a chain of ~4 dependent products per round on one wave per SIMD, so the product's latency is
// the witness engine's pace (config 5).
#include <hip/hip_runtime.h>
#include <string.h>

#include <cctype>
#include <cstdio>
#include <string>
#include <vector>

#include "common.h"
#include "field.h"
#include "fr29.h"
#include "host_parse.h"
#include "witness.h"
#include "wtrace.h"
#include "zkfl.h"

namespace zkfl {

namespace {

struct PosWidth {
  uint32_t rp;
  uint32_t c_off;  // index into consts (Fr) of the round constants
  uint32_t m_off;  // index of the MDS matrix
};

struct ProgView {  // device pointers, passed by value
  const uint4* ops;
  const uint32_t* lc_ptr;
  const uint32_t* term_wire;
  const Fr* term_coef;
  const uint32_t* asserts;
  const uint32_t* tmpl;  // 8 words per template
  const Fr* consts;
  PosWidth width[MAX_T + 1];
  uint32_t n_wires;
};

// term wire bit 31: coefficient one (no product)
ZK_DEV Fr29 lc_eval(const ProgView& P, const Fr* w, uint32_t lc) {
  Fr29 acc = f29_zero();
  const uint32_t e = P.lc_ptr[lc + 1];
  for (uint32_t t = P.lc_ptr[lc]; t < e; t++) {
    const uint32_t x = P.term_wire[t];
    Fr29 v = fr29_ld(w[x & 0x7FFFFFFFu]);
    if (!(x >> 31)) v = fr29_mul(v, fr29_ld(P.term_coef[t]));
    acc = fr29_add(acc, v);
  }
  return acc;
}

// the image's 2^256 Montgomery field elements (coefficients, Poseidon constants) -> x 2^261
__global__ __launch_bounds__(256) void k_wit_to_m261(Fr* a, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) a[i] = fr29_st(fr29_from_m256(a[i]));
}

// circomlib Poseidon permutation (zkfl/field.py::poseidon_perm_trace) of width T for one K_POS op
// per group of T lanes: lane i of a group holds state element i (9 VGPRs, no scratch), applies
// the ARK constant and, in full rounds or for i = 0, the S-box (writing x^2, x^4, x^5 when the
// template marks that S-box live), then computes MDS row i from the group's state read with
// cross-lane shuffles, 4 products per Montgomery reduction (pos_rounds).  The latency of a round is
// one row, not T rows (one lane per permutation), and nothing is spilled.  Every lane of the wave executes
// the shuffles; lanes without a job compute on zeros and store nothing.
// The rounds of one permutation for widths T <= 4 NC: the MDS row is NC independent 4-term sums
// (unrolled, so their shuffles, LDS reads and products overlap; a row's terms past T are zeros), the
// MDS matrix is read from LDS (staged once per block) and the next round's ARK constant is loaded
// while this round runs -- the round's latency is the S-box chain and one product, not a global
// load and T / 4 serial products.
struct PosCtx {
  const Fr* C;     // round constants of the width (global)
  const Fr* mrow;  // this lane's MDS row (LDS)
  Fr* w;
  uint4 op;
  uint32_t T, i, gb, rp;
  uint32_t lw[7], pre[7];  // live S-box bitmap of the op's template and its word prefix counts
};
template <int NC>
ZK_DEV void pos_rounds(const PosCtx& X, Fr29 st) {
  const uint32_t T = X.T, i = X.i, rp = X.rp, rounds = 8 + rp;
  Fr cn = X.C[i];
  for (uint32_t r = 0; r < rounds; r++) {
    const Fr cr = cn;
    if (r + 1 < rounds) cn = X.C[(r + 1) * T + i];  // in flight during this round
    st = fr29_add(st, fr29_ld(cr));
    const bool full = r < 4 || r >= 4 + rp;
    if (full || i == 0) {
      const uint32_t sb = r < 4 ? r * T + i : (r < 4 + rp ? 4 * T + (r - 4) : 4 * T + rp + (r - 4 - rp) * T + i);
      const Fr29 x2 = fr29_sqr(st), x4 = fr29_sqr(x2), x5 = fr29_mul(x4, st);
      const uint32_t q = sb >> 5, bit = sb & 31;
      uint32_t word = 0, rank = 0;
#pragma unroll
      for (int k = 0; k < 7; k++)
        if ((uint32_t)k == q) {
          word = X.lw[k];
          rank = X.pre[k];
        }
      if ((word >> bit) & 1u) {
        const uint32_t k = X.op.y + 3 * (rank + __popc(word & ((1u << bit) - 1u)));
        X.w[k] = fr29_st(x2);
        X.w[k + 1] = fr29_st(x4);
        X.w[k + 2] = fr29_st(x5);
      }
      st = x5;
    }
    Fr29 part[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) {
      Fr29 x[4], y[4];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint32_t j = 4 * c + k;
        const uint32_t src = X.gb + (j < T ? j : 0);
#pragma unroll
        for (int v = 0; v < 9; v++) x[k].v[v] = __shfl((int)st.v[v], (int)src);
        y[k] = j < T ? fr29_ld(X.mrow[j]) : f29_zero();
      }
      part[c] = fr29_mulsum<4>(x, y);
    }
    Fr29 acc = part[0];
#pragma unroll
    for (int c = 1; c < NC; c++) acc = fr29_add(acc, part[c]);
    st = acc;
  }
}

// (block bx of a K_POS segment: 64 / T permutations; every thread of the block calls it)
ZK_DEV void wit_pos_block(const ProgView& P, size_t n, uint32_t op0, uint32_t cnt, uint32_t T, Fr* W, size_t bx) {
  const uint32_t lane = threadIdx.x, G = 64 / T;
  const uint32_t g = lane / T, i = lane - g * T;
  const size_t job = bx * G + g;
  const bool active = g < G && job < n * cnt;
  const size_t jj = active ? job : 0;
  PosCtx X;
  X.op = P.ops[op0 + (uint32_t)(jj % cnt)];
  X.w = W + (jj / cnt) * P.n_wires;
  X.gb = (g < G ? g : 0) * T;  // the group's first lane
  X.T = T;
  X.i = i;
  const PosWidth pw = P.width[T];
  X.rp = pw.rp;
  X.C = P.consts + pw.c_off;
  __shared__ Fr mds[MAX_T * MAX_T];  // the width's MDS matrix, read every round
  const Fr* __restrict__ Mg = P.consts + pw.m_off;
  for (uint32_t e = lane; e < T * T; e += 64) mds[e] = Mg[e];
  __syncthreads();
  X.mrow = mds + (size_t)i * T;
  const uint32_t* live = P.tmpl + 8 * (X.op.w >> 8) + 1;
  uint32_t acc_live = 0;
#pragma unroll
  for (int q = 0; q < 7; q++) {
    X.lw[q] = active ? live[q] : 0u;
    X.pre[q] = acc_live;
    acc_live += __popc(X.lw[q]);
  }
  const Fr29 st = (active && i > 0) ? lc_eval(P, X.w, X.op.z + i - 1) : f29_zero();
  switch ((T + 3) / 4) {
    case 1: pos_rounds<1>(X, st); break;
    case 2: pos_rounds<2>(X, st); break;
    case 3: pos_rounds<3>(X, st); break;
    case 4: pos_rounds<4>(X, st); break;
    default: pos_rounds<5>(X, st); break;
  }
}

__global__ __launch_bounds__(64) void k_wit_inputs(size_t n, uint32_t nw, uint32_t in_first, uint32_t n_in,
                                                   const uint32_t* __restrict__ inputs, Fr* __restrict__ W) {
  size_t l = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= n * (n_in + 1)) return;
  const size_t j = l / (n_in + 1), i = l % (n_in + 1);
  Fr* w = W + j * nw;
  if (i == n_in) {
    w[0] = fr29_st(f29_const(R29::ONE));
    return;
  }
  Fr v;
#pragma unroll
  for (int q = 0; q < 8; q++) v.v[q] = inputs[(j * n_in + i) * 8 + q];
  w[in_first + i] = fr29_st(fr29_from_plain(v));
}

// lane l of a segment of LC / MUL / INV / BITS ops: op l % cnt of witness l / cnt
ZK_DEV void wit_op_lane(const ProgView& P, size_t n, uint32_t op0, uint32_t cnt, Fr* W, size_t l) {
  if (l >= n * cnt) return;
  const size_t j = l / cnt;
  const uint4 op = P.ops[op0 + (uint32_t)(l % cnt)];
  Fr* w = W + j * P.n_wires;
  switch (op.x) {
    case K_LC:
      w[op.y] = fr29_st(lc_eval(P, w, op.z));
      break;
    case K_MUL:
      w[op.y] = fr29_st(fr29_mul(lc_eval(P, w, op.z), lc_eval(P, w, op.z + 1)));
      break;
    case K_INV: {  // rare (IsZero hints): the 32-bit engine's inverse
      const Fr29 v = lc_eval(P, w, op.z);
      w[op.y] = fr29_is_zero(v) ? fr29_st(v) : fr29_st(fr29_from_m256(fp_inv(fr29_to_m256(v))));
      break;
    }
    case K_BITS: {
      Fr v = fr29_to_plain(lc_eval(P, w, op.z));
      const Fr one = fr29_st(f29_const(R29::ONE)), zero = fp_zero<FrP>();
#pragma unroll
      for (uint32_t q = 0; q < 8; q++) {  // constant limb index: v stays in registers
#pragma unroll 1
        for (uint32_t b = 0; b < 32 && q * 32 + b < op.w; b++) {
          const uint32_t bit = (v.v[q] >> b) & 1u;
          Fr o;
#pragma unroll
          for (int k = 0; k < 8; k++) o.v[k] = bit ? one.v[k] : zero.v[k];  // per-limb select, no stack copy
          w[op.y + q * 32 + b] = o;
        }
      }
      break;
    }
    default:  // K_POS ops run in lane groups (wit_pos_block: wprog_load groups them per level and width)
      break;
  }
}

// One level of the program in ONE launch: its segments (the LC / MUL / INV / BITS ops, then the
// Poseidon permutations of each width) side by side, blocks [blk0[s], blk0[s + 1]) for segment s.
// The ops of a level are independent, so a level's Poseidon widths no longer wait for each other:
// the config-5 training circuit's first level holds permutations of widths 3, 5 and 6, which ran
// as three dependent ~0.3-ms launches.
constexpr int WIT_MAX_SEGS = MAX_T + 1;
struct WitLevel {
  uint32_t n;  // segments
  uint32_t op0[WIT_MAX_SEGS], cnt[WIT_MAX_SEGS], t[WIT_MAX_SEGS];  // t = 0: LC / MUL / INV / BITS
  uint32_t blk0[WIT_MAX_SEGS + 1];
};
__global__ __launch_bounds__(64) void k_wit_lvl(ProgView P, size_t n, const WitLevel L, Fr* W) {
  ZK_WT(WT_WITNESS);
  uint32_t s = 0;
  while (s + 1 < L.n && blockIdx.x >= L.blk0[s + 1]) s++;
  const size_t bx = blockIdx.x - L.blk0[s];
  if (L.t[s] == 0)
    wit_op_lane(P, n, L.op0[s], L.cnt[s], W, bx * 64 + threadIdx.x);
  else
    wit_pos_block(P, n, L.op0[s], L.cnt[s], L.t[s], W, bx);
}

__global__ __launch_bounds__(64) void k_wit_asserts(ProgView P, size_t n, uint32_t na, const Fr* W, uint32_t* fail) {
  size_t l = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= n * na) return;
  const size_t j = l / na;
  const uint32_t a = (uint32_t)(l % na);
  const Fr* w = W + j * P.n_wires;
  const uint32_t lc0 = P.asserts[a];
  const Fr29 ab = fr29_mul(lc_eval(P, w, lc0), lc_eval(P, w, lc0 + 1));
  if (!fr29_eq(ab, lc_eval(P, w, lc0 + 2))) atomicMin(fail + j, a);
}

// x 2^261 -> standard form into each witness's output buffer
__global__ __launch_bounds__(256) void k_wit_out(size_t n, uint32_t nw, const Fr* W, Fr* const* outs) {
  size_t l = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= n * nw) return;
  const size_t j = l / nw, i = l % nw;
  outs[j][i] = fr29_to_plain(fr29_ld(W[l]));
}

int hip_err(hipError_t e, const char* where, std::string& err) {
  err = std::string(where) + ": " + hipGetErrorString(e);
  return e == hipErrorOutOfMemory ? ZKFL_E_OOM : ZKFL_E_DEVICE;
}

}  // namespace

struct WProg {
  std::vector<WSignal> signals;
  uint32_t n_wires = 0, n_pub_out = 0, n_pub_in = 0, n_prv_in = 0, in_first = 0;
  uint32_t n_ops = 0, n_levels = 0, n_asserts = 0;
  std::vector<uint32_t> level_ptr;
  struct Seg {
    uint32_t op0, cnt, t;  // t = 0: LC / MUL / INV / BITS ops; else K_POS ops of width t
  };
  std::vector<Seg> segs;            // level by level
  std::vector<uint32_t> seg_level;  // segs of level L: [seg_level[L], seg_level[L + 1]) -- one launch each
  ProgView view = {};
  std::vector<void*> allocs;
};

void wprog_free(WProg* p) {
  if (!p) return;
  for (void* a : p->allocs) (void)hipFree(a);
  delete p;
}

int wprog_inputs_json(const WProg* p, const char* json, std::vector<uint32_t>& out, std::string& err) {
  return inputs_from_json(p->signals, json, out, err);
}

int wprog_image_inputs_json(const uint8_t* img, size_t len, const char* json, std::vector<uint32_t>& out,
                            std::string& err) {
  std::vector<WSignal> sigs;  // the signal table alone, without touching the device
  int rc = wprog_signals(img, len, sigs, err);
  return rc ? rc : inputs_from_json(sigs, json, out, err);
}

void wprog_info(const WProg* p, uint32_t* nw, uint32_t* n_in, uint32_t* n_pub) {
  if (nw) *nw = p->n_wires;
  if (n_in) *n_in = p->n_pub_in + p->n_prv_in;
  if (n_pub) *n_pub = p->n_pub_out + p->n_pub_in;
}

int wprog_load(const uint8_t* img, size_t len, hipStream_t st, WProg** out, std::string& err) {
  WProgHost H;
  int rc = wprog_parse(img, len, H, err);  // csrc/host_parse.cc: every index validated
  if (rc) return rc;
  WProg* p = new WProg();
  p->n_wires = H.n_wires;
  p->n_pub_out = H.n_pub_out;
  p->n_pub_in = H.n_pub_in;
  p->n_prv_in = H.n_prv_in;
  p->in_first = H.in_first;
  p->n_ops = H.n_ops;
  p->n_levels = H.n_levels;
  p->n_asserts = H.n_asserts;
  p->level_ptr = std::move(H.level_ptr);
  p->signals = std::move(H.signals);
  for (int t = 0; t <= MAX_T; t++) p->view.width[t] = {H.width[t].rp, H.width[t].c_off, H.width[t].m_off};
  const uint32_t n_lcs = H.n_lcs, n_terms = H.n_terms, n_tmpl = H.n_tmpl;
  const uint8_t *lcp = H.lc_ptr, *tw = H.term_wire, *tc = H.term_coef, *as = H.asserts, *tm = H.tmpl;
  // Ops of a level are independent: regroup each level as [other ops][K_POS by width] so the
  // Poseidon permutations run in lane groups of their width (k_wit_lvl: one launch per level).
  std::vector<uint4> ops_v(p->n_ops);
  for (uint32_t L = 0; L < p->n_levels; L++) {
    p->seg_level.push_back((uint32_t)p->segs.size());
    const uint32_t a = p->level_ptr[L], b = p->level_ptr[L + 1];
    uint32_t o = a;
    for (uint32_t t = 0; t <= (uint32_t)MAX_T; t++) {
      const uint32_t first = o;
      for (uint32_t q = a; q < b; q++) {
        uint4 op;
        memcpy(&op, H.ops + 16ull * q, 16);
        const uint32_t opt = op.x == K_POS ? (op.w & 0xFFu) : 0u;
        if (opt == t) ops_v[o++] = op;
      }
      if (o > first) p->segs.push_back({first, o - first, t});
    }
  }
  p->seg_level.push_back((uint32_t)p->segs.size());
  const uint8_t* ops = reinterpret_cast<const uint8_t*>(ops_v.data());
  std::vector<uint8_t>& consts = H.consts;
  struct Up {
    const void* src;
    size_t bytes;
    void** dst;
  };
  void *d_ops, *d_lcp, *d_tw, *d_tc, *d_as, *d_tm, *d_c;
  Up ups[] = {{ops, 16ull * p->n_ops, &d_ops},       {lcp, 4ull * (n_lcs + 1), &d_lcp},
              {tw, 4ull * n_terms, &d_tw},            {tc, 32ull * n_terms, &d_tc},
              {as, 4ull * p->n_asserts, &d_as},      {tm, 32ull * n_tmpl, &d_tm},
              {consts.data(), consts.size(), &d_c}};
  hipError_t e = hipSuccess;
  for (auto& u : ups) {
    *u.dst = nullptr;
    if (e == hipSuccess) e = hipMalloc(u.dst, u.bytes + 16);
    if (e == hipSuccess) {
      p->allocs.push_back(*u.dst);
      if (u.bytes) e = hipMemcpyAsync(*u.dst, u.src, u.bytes, hipMemcpyHostToDevice, st);
    }
  }
  // the coefficients and constants into the witness engine's x 2^261 form
  const size_t n_c = consts.size() / 32;
  if (e == hipSuccess && n_terms)
    hipLaunchKernelGGL(k_wit_to_m261, dim3(zk_grid(n_terms, 256)), dim3(256), 0, st, (Fr*)d_tc, (size_t)n_terms);
  if (e == hipSuccess && n_c) hipLaunchKernelGGL(k_wit_to_m261, dim3(zk_grid(n_c, 256)), dim3(256), 0, st, (Fr*)d_c, n_c);
  if (e == hipSuccess) e = hipGetLastError();
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) {
    wprog_free(p);
    return hip_err(e, "witness program upload", err);
  }
  p->view.ops = (const uint4*)d_ops;
  p->view.lc_ptr = (const uint32_t*)d_lcp;
  p->view.term_wire = (const uint32_t*)d_tw;
  p->view.term_coef = (const Fr*)d_tc;
  p->view.asserts = (const uint32_t*)d_as;
  p->view.tmpl = (const uint32_t*)d_tm;
  p->view.consts = (const Fr*)d_c;
  p->view.n_wires = p->n_wires;
  *out = p;
  return ZKFL_OK;
}

bool wprog_inputs_ok(const WProg* p, size_t n, const uint8_t* inputs, std::string& err) {
  const uint32_t n_in = p->n_pub_in + p->n_prv_in;
  for (size_t i = 0; i < n * n_in; i++)
    if (!fr_lt_r(reinterpret_cast<const uint32_t*>(inputs + 32 * i))) {
      err = "witness input " + std::to_string(i % n_in) + " of witness " + std::to_string(i / n_in) + " is not < r";
      return false;
    }
  return true;
}

hipError_t wprog_enqueue(const WProg* p, size_t m, const uint32_t* d_in, Fr* W, Fr* const* d_outs, uint32_t* d_fail,
                         hipStream_t st) {
  const uint32_t n_in = p->n_pub_in + p->n_prv_in, nw = p->n_wires;
  hipError_t e = hipMemsetAsync(W, 0, m * (size_t)nw * 32, st);
  if (e == hipSuccess) e = hipMemsetAsync(d_fail, 0xFF, m * 4, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_wit_inputs, dim3(zk_grid(m * (n_in + 1), 64)), dim3(64), 0, st, m, nw, p->in_first, n_in, d_in,
                     W);
  for (size_t L = 0; L + 1 < p->seg_level.size(); L++) {
    WitLevel lv = {};
    uint32_t blocks = 0;
    for (uint32_t q = p->seg_level[L]; q < p->seg_level[L + 1]; q++) {
      const WProg::Seg& g = p->segs[q];
      lv.op0[lv.n] = g.op0;
      lv.cnt[lv.n] = g.cnt;
      lv.t[lv.n] = g.t;
      lv.blk0[lv.n] = blocks;
      blocks += g.t == 0 ? zk_grid(m * g.cnt, 64) : zk_grid(m * g.cnt, 64 / g.t);
      lv.n++;
    }
    lv.blk0[lv.n] = blocks;
    if (blocks) hipLaunchKernelGGL(k_wit_lvl, dim3(blocks), dim3(64), 0, st, p->view, m, lv, W);
  }
  if (p->n_asserts)
    hipLaunchKernelGGL(k_wit_asserts, dim3(zk_grid(m * p->n_asserts, 64)), dim3(64), 0, st, p->view, m, p->n_asserts,
                       (const Fr*)W, d_fail);
  hipLaunchKernelGGL(k_wit_out, dim3(zk_grid(m * nw, 256)), dim3(256), 0, st, m, nw, (const Fr*)W, d_outs);
  return hipGetLastError();
}

int wprog_run(const WProg* p, size_t n, const uint8_t* inputs, Fr* const* outs_host, hipStream_t st,
              std::string& err) {
  if (n == 0) return ZKFL_OK;
  if (!wprog_inputs_ok(p, n, inputs, err)) return ZKFL_E_ARG;
  const uint32_t n_in = p->n_pub_in + p->n_prv_in, nw = p->n_wires;
  // chunk so the Montgomery scratch stays bounded (M: 8.4 MB per witness)
  const size_t per = (size_t)nw * 32;
  size_t chunk = (size_t)(2048ull << 20) / (per ? per : 1);
  if (chunk < 1) chunk = 1;
  if (chunk > n) chunk = n;
  Fr* W = nullptr;
  uint32_t *d_in = nullptr, *d_fail = nullptr;
  Fr** d_outs = nullptr;
  hipError_t e = hipMalloc(&W, chunk * per);
  if (e == hipSuccess) e = hipMalloc(&d_in, chunk * n_in * 32 + 16);
  if (e == hipSuccess) e = hipMalloc(&d_fail, chunk * 4);
  if (e == hipSuccess) e = hipMalloc(&d_outs, chunk * sizeof(Fr*));
  std::vector<uint32_t> fails(chunk);
  int rc = ZKFL_OK;
  for (size_t off = 0; off < n && e == hipSuccess && rc == ZKFL_OK; off += chunk) {
    const size_t m = (n - off < chunk) ? n - off : chunk;
    if (n_in) e = hipMemcpyAsync(d_in, inputs + off * n_in * 32, m * n_in * 32, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipMemcpyAsync(d_outs, outs_host + off, m * sizeof(Fr*), hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = wprog_enqueue(p, m, d_in, W, (Fr* const*)d_outs, d_fail, st);
    if (e == hipSuccess) e = hipMemcpyAsync(fails.data(), d_fail, m * 4, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    for (size_t j = 0; e == hipSuccess && j < m; j++)
      if (fails[j] != 0xFFFFFFFFu) {
        err = "witness " + std::to_string(off + j) + ": assert constraint #" + std::to_string(fails[j]) +
              " failed (inputs do not satisfy the circuit)";
        rc = ZKFL_E_CONSTRAINT;
        break;
      }
  }
  if (rc == ZKFL_OK && e != hipSuccess) rc = hip_err(e, "witness compute", err);
  for (void* q : {(void*)W, (void*)d_in, (void*)d_fail, (void*)d_outs})
    if (q) (void)hipFree(q);
  return rc;
}

hipError_t zk_wtrace_bind_wit(const WtBuf& b) { return zk_wtrace_bind_tu(b); }

}  // namespace zkfl
