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
// one launch per level, one lane per (witness, op), values in Montgomery form; a final pass
// checks the asserts and writes the standard-form witness.  Independent of the circuit: the
// program image carries the linear combinations, the Poseidon templates and constants.
#include <hip/hip_runtime.h>
#include <string.h>

#include <cctype>
#include <cstdio>
#include <string>
#include <vector>

#include "common.h"
#include "field.h"
#include "witness.h"
#include "zkfl.h"

namespace zkfl {

namespace {

enum : uint32_t { K_LC = 0, K_MUL = 1, K_INV = 2, K_BITS = 3, K_POS = 4 };
constexpr int MAX_T = 17;

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

ZK_DEV Fr lc_eval(const ProgView& P, const Fr* w, uint32_t lc) {
  Fr acc = fp_zero<FrP>();
  const uint32_t e = P.lc_ptr[lc + 1];
  for (uint32_t t = P.lc_ptr[lc]; t < e; t++) {
    const uint32_t x = P.term_wire[t];
    Fr v = w[x & 0x7FFFFFFFu];
    if (!(x >> 31)) v = fp_mul(v, P.term_coef[t]);
    acc = fp_add(acc, v);
  }
  return acc;
}

// circomlib Poseidon permutation (zkfl/field.py::poseidon_perm_trace), width t, trace writes
__device__ __attribute__((noinline)) void pos_run(const ProgView& P, Fr* w, uint32_t out, uint32_t lc0, uint32_t t,
                                                   const uint32_t* live) {
  Fr st[MAX_T], ns[MAX_T];
  st[0] = fp_zero<FrP>();
  for (uint32_t i = 1; i < t; i++) st[i] = lc_eval(P, w, lc0 + i - 1);
  const PosWidth pw = P.width[t];
  const Fr* C = P.consts + pw.c_off;
  const Fr* M = P.consts + pw.m_off;
  const uint32_t rounds = 8 + pw.rp;
  uint32_t k = out, sb = 0;
  for (uint32_t r = 0; r < rounds; r++) {
    for (uint32_t i = 0; i < t; i++) st[i] = fp_add(st[i], C[r * t + i]);
    const uint32_t nl = (r < 4 || r >= 4 + pw.rp) ? t : 1;
    for (uint32_t i = 0; i < nl; i++, sb++) {
      Fr x2 = fp_sqr(st[i]);
      Fr x4 = fp_sqr(x2);
      Fr x5 = fp_mul(x4, st[i]);
      if ((live[sb >> 5] >> (sb & 31)) & 1u) {
        w[k] = x2;
        w[k + 1] = x4;
        w[k + 2] = x5;
        k += 3;
      }
      st[i] = x5;
    }
    for (uint32_t i = 0; i < t; i++) {
      Fr acc = fp_mul(M[i * t], st[0]);
      for (uint32_t j = 1; j < t; j++) acc = fp_add(acc, fp_mul(M[i * t + j], st[j]));
      ns[i] = acc;
    }
    for (uint32_t i = 0; i < t; i++) st[i] = ns[i];
  }
}

__global__ __launch_bounds__(64) void k_wit_inputs(size_t n, uint32_t nw, uint32_t in_first, uint32_t n_in,
                                                   const uint32_t* __restrict__ inputs, Fr* __restrict__ W) {
  size_t l = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= n * (n_in + 1)) return;
  const size_t j = l / (n_in + 1), i = l % (n_in + 1);
  Fr* w = W + j * nw;
  if (i == n_in) {
    w[0] = fp_one<FrP>();
    return;
  }
  Fr v;
#pragma unroll
  for (int q = 0; q < 8; q++) v.v[q] = inputs[(j * n_in + i) * 8 + q];
  w[in_first + i] = fp_to_mont(v);
}

__global__ __launch_bounds__(64) void k_wit_level(ProgView P, size_t n, uint32_t op0, uint32_t cnt, Fr* W) {
  size_t l = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= n * cnt) return;
  const size_t j = l / cnt;
  const uint4 op = P.ops[op0 + (uint32_t)(l % cnt)];
  Fr* w = W + j * P.n_wires;
  switch (op.x) {
    case K_LC:
      w[op.y] = lc_eval(P, w, op.z);
      break;
    case K_MUL:
      w[op.y] = fp_mul(lc_eval(P, w, op.z), lc_eval(P, w, op.z + 1));
      break;
    case K_INV: {
      Fr v = lc_eval(P, w, op.z);
      w[op.y] = fp_is_zero(v) ? v : fp_inv(v);
      break;
    }
    case K_BITS: {
      Fr v = fp_from_mont(lc_eval(P, w, op.z));
      const Fr one = fp_one<FrP>(), zero = fp_zero<FrP>();
      for (uint32_t i = 0; i < op.w; i++) w[op.y + i] = ((v.v[i >> 5] >> (i & 31)) & 1u) ? one : zero;
      break;
    }
    default:  // K_POS
      pos_run(P, w, op.y, op.z, op.w & 0xFFu, P.tmpl + 8 * (op.w >> 8) + 1);
      break;
  }
}

__global__ __launch_bounds__(64) void k_wit_asserts(ProgView P, size_t n, uint32_t na, const Fr* W, uint32_t* fail) {
  size_t l = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= n * na) return;
  const size_t j = l / na;
  const uint32_t a = (uint32_t)(l % na);
  const Fr* w = W + j * P.n_wires;
  const uint32_t lc0 = P.asserts[a];
  Fr ab = fp_mul(lc_eval(P, w, lc0), lc_eval(P, w, lc0 + 1));
  if (!fp_eq(ab, lc_eval(P, w, lc0 + 2))) atomicMin(fail + j, a);
}

// Montgomery -> standard form into each witness's output buffer
__global__ __launch_bounds__(256) void k_wit_out(size_t n, uint32_t nw, const Fr* W, Fr* const* outs) {
  size_t l = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= n * nw) return;
  const size_t j = l / nw, i = l % nw;
  outs[j][i] = fp_from_mont(W[l]);
}

int hip_err(hipError_t e, const char* where, std::string& err) {
  err = std::string(where) + ": " + hipGetErrorString(e);
  return e == hipErrorOutOfMemory ? ZKFL_E_OOM : ZKFL_E_DEVICE;
}

bool lt_r_host(const uint32_t* v) {
  static const uint32_t Rl[8] = {0xf0000001u, 0x43e1f593u, 0x79b97091u, 0x2833e848u,
                                 0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
  for (int i = 7; i >= 0; i--)
    if (v[i] != Rl[i]) return v[i] < Rl[i];
  return false;
}

struct Reader {
  const uint8_t* p;
  size_t left;
  bool ok = true;
  const uint8_t* take(size_t n) {
    if (!ok || n > left) {
      ok = false;
      return nullptr;
    }
    const uint8_t* r = p;
    p += n;
    left -= n;
    return r;
  }
  uint32_t u32() {
    const uint8_t* q = take(4);
    uint32_t v = 0;
    if (q) memcpy(&v, q, 4);
    return v;
  }
};


struct WSignal {  // one declared input signal (input.json key)
  std::string name;
  std::vector<uint32_t> dims;
  uint32_t first = 0;
  uint32_t pub = 0;
};

bool read_signals(Reader& R, std::vector<WSignal>& out) {
  const uint32_t n = R.u32();
  if (!R.ok || n > (1u << 20)) return false;
  for (uint32_t i = 0; i < n; i++) {
    WSignal sg;
    const uint32_t len = R.u32();
    if (!R.ok || len > 4096) return false;
    const uint8_t* nm = R.take((len + 3) & ~3u);
    if (!nm) return false;
    sg.name.assign(reinterpret_cast<const char*>(nm), len);
    const uint32_t nd = R.u32();
    if (!R.ok || nd > 16) return false;
    for (uint32_t d = 0; d < nd; d++) sg.dims.push_back(R.u32());
    sg.first = R.u32();
    sg.pub = R.u32();
    if (!R.ok) return false;
    out.push_back(std::move(sg));
  }
  return true;
}

// ---------------------------------------------------------------------------
// input.json -> flattened input signals (host).  The subset circom's witness calculator accepts
// for these circuits: one object mapping signal names to a number, a decimal (or 0x hex) string,
// or nested arrays of those; negatives are reduced mod r as circom does.  Extra keys are
// ignored (as zkfl/r1cs.py::flatten_inputs does).
// ---------------------------------------------------------------------------
struct JVal {
  enum Kind { SCALAR, ARRAY, OBJECT } kind = SCALAR;
  std::string text;  // scalar literal (string contents or number text)
  std::vector<JVal> items;
  std::vector<std::string> keys;
};

struct JParser {
  const char* s;
  const char* e;
  std::string err;
  void ws() {
    while (s < e && (*s == ' ' || *s == '\n' || *s == '\r' || *s == '\t')) s++;
  }
  bool fail(const char* m) {
    if (err.empty()) err = m;
    return false;
  }
  bool str(std::string& out) {
    if (s >= e || *s != '"') return fail("expected a string");
    s++;
    while (s < e && *s != '"') {
      if (*s == '\\') return fail("escapes are not supported in input strings");
      out.push_back(*s++);
    }
    if (s >= e) return fail("unterminated string");
    s++;
    return true;
  }
  bool value(JVal& v, int depth) {
    if (depth > 32) return fail("nesting too deep");
    ws();
    if (s >= e) return fail("unexpected end of input");
    if (*s == '{' || *s == '[') {
      const bool obj = *s == '{';
      const char close = obj ? '}' : ']';
      v.kind = obj ? JVal::OBJECT : JVal::ARRAY;
      s++;
      ws();
      if (s < e && *s == close) {
        s++;
        return true;
      }
      for (;;) {
        ws();
        std::string k;
        if (obj) {
          if (!str(k)) return false;
          ws();
          if (s >= e || *s != ':') return fail("expected ':'");
          s++;
        }
        JVal c;
        if (!value(c, depth + 1)) return false;
        if (obj) v.keys.push_back(k);
        v.items.push_back(std::move(c));
        ws();
        if (s < e && *s == ',') {
          s++;
          continue;
        }
        if (s < e && *s == close) {
          s++;
          return true;
        }
        return fail(obj ? "expected ',' or '}'" : "expected ',' or ']'");
      }
    }
    v.kind = JVal::SCALAR;
    if (*s == '"') return str(v.text);
    while (s < e && (isalnum((unsigned char)*s) || *s == '-' || *s == '+' || *s == '.')) v.text.push_back(*s++);
    if (v.text.empty()) return fail("unexpected character");
    return true;
  }
};

// decimal / 0x-hex integer literal (optional sign) -> std-form Fr limbs (mod r)
bool literal_to_fr(const std::string& t, uint32_t out[8]) {
  static const uint64_t RL[4] = {0x43e1f593f0000001ull, 0x2833e84879b97091ull, 0xb85045b68181585dull,
                                 0x30644e72e131a029ull};
  size_t i = 0;
  bool neg = false;
  if (i < t.size() && (t[i] == '-' || t[i] == '+')) neg = t[i++] == '-';
  unsigned base = 10;
  if (i + 1 < t.size() && t[i] == '0' && (t[i + 1] == 'x' || t[i + 1] == 'X')) {
    base = 16;
    i += 2;
  }
  if (i >= t.size()) return false;
  uint64_t acc[5] = {0, 0, 0, 0, 0};  // < 16 r + 15 < 2^259 before reduction
  for (; i < t.size(); i++) {
    const char ch = t[i];
    unsigned d;
    if (ch >= '0' && ch <= '9') d = ch - '0';
    else if (base == 16 && ch >= 'a' && ch <= 'f') d = ch - 'a' + 10;
    else if (base == 16 && ch >= 'A' && ch <= 'F') d = ch - 'A' + 10;
    else return false;  // fractions / exponents are not field elements
    unsigned __int128 c = d;
    for (int k = 0; k < 5; k++) {
      c += (unsigned __int128)acc[k] * base;
      acc[k] = (uint64_t)c;
      c >>= 64;
    }
    for (;;) {  // reduce below r
      bool ge = acc[4] != 0;
      if (!ge) {
        ge = true;
        for (int k = 3; k >= 0; k--)
          if (acc[k] != RL[k]) {
            ge = acc[k] > RL[k];
            break;
          }
      }
      if (!ge) break;
      uint64_t borrow = 0;
      for (int k = 0; k < 5; k++) {
        const unsigned __int128 sub = (unsigned __int128)(k < 4 ? RL[k] : 0) + borrow;
        borrow = (unsigned __int128)acc[k] < sub ? 1 : 0;
        acc[k] = (uint64_t)((unsigned __int128)acc[k] - sub);
      }
    }
  }
  const bool zero = !(acc[0] | acc[1] | acc[2] | acc[3]);
  if (neg && !zero) {  // r - v
    uint64_t borrow = 0;
    for (int k = 0; k < 4; k++) {
      const unsigned __int128 sub = (unsigned __int128)acc[k] + borrow;
      borrow = (unsigned __int128)RL[k] < sub ? 1 : 0;
      acc[k] = (uint64_t)((unsigned __int128)RL[k] - sub);
    }
  }
  for (int k = 0; k < 4; k++) {
    out[2 * k] = (uint32_t)acc[k];
    out[2 * k + 1] = (uint32_t)(acc[k] >> 32);
  }
  return true;
}

bool flatten(const JVal& v, const WSignal& sg, size_t dim, std::vector<uint32_t>& out, std::string& err) {
  if (dim == sg.dims.size()) {
    if (v.kind != JVal::SCALAR) {
      err = "input '" + sg.name + "' has too many dimensions";
      return false;
    }
    uint32_t fr[8];
    if (!literal_to_fr(v.text, fr)) {
      err = "input '" + sg.name + "': '" + v.text + "' is not an integer";
      return false;
    }
    out.insert(out.end(), fr, fr + 8);
    return true;
  }
  if (v.kind != JVal::ARRAY || v.items.size() != sg.dims[dim]) {
    std::string shape;
    for (uint32_t d : sg.dims) shape += (shape.empty() ? "" : ", ") + std::to_string(d);
    err = "input '" + sg.name + "' has wrong shape, expected (" + shape + ")";
    return false;
  }
  for (const JVal& c : v.items)
    if (!flatten(c, sg, dim + 1, out, err)) return false;
  return true;
}

int inputs_from_json(const std::vector<WSignal>& sigs, const char* json, std::vector<uint32_t>& out,
                     std::string& err) {
  if (!json) {
    err = "null input json";
    return ZKFL_E_ARG;
  }
  JParser P{json, json + strlen(json), ""};
  JVal root;
  if (!P.value(root, 0)) {
    err = "input json: " + P.err;
    return ZKFL_E_ARG;
  }
  P.ws();
  if (P.s != P.e || root.kind != JVal::OBJECT) {
    err = "input json: expected one object of signal names";
    return ZKFL_E_ARG;
  }
  for (const WSignal& sg : sigs) {
    size_t k = 0;
    while (k < root.keys.size() && root.keys[k] != sg.name) k++;
    if (k == root.keys.size()) {
      err = "missing input signal '" + sg.name + "'";
      return ZKFL_E_ARG;
    }
    if (!flatten(root.items[k], sg, 0, out, err)) return ZKFL_E_ARG;
  }
  return ZKFL_OK;
}

}  // namespace

struct WProg {
  std::vector<WSignal> signals;
  uint32_t n_wires = 0, n_pub_out = 0, n_pub_in = 0, n_prv_in = 0, in_first = 0;
  uint32_t n_ops = 0, n_levels = 0, n_asserts = 0;
  std::vector<uint32_t> level_ptr;
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
  // walk the image to its signal table without touching the device
  Reader R{img, len};
  const uint8_t* magic = R.take(4);
  if (!magic || memcmp(magic, "zkwp", 4) != 0 || R.u32() != 2) {
    err = "witness program: bad magic/version";
    return ZKFL_E_FORMAT;
  }
  uint32_t h[12];
  for (int i = 0; i < 12; i++) h[i] = R.u32();
  const uint32_t n_ops = h[5], n_levels = h[6], n_lcs = h[7], n_terms = h[8], n_asserts = h[9], n_tmpl = h[10],
                 n_widths = h[11];
  R.take(4ull * (n_levels + 1));
  R.take(16ull * n_ops);
  R.take(4ull * (n_lcs + 1));
  R.take(36ull * n_terms);
  R.take(4ull * n_asserts);
  R.take(32ull * n_tmpl);
  for (uint32_t k = 0; k < n_widths && R.ok; k++) {
    const uint32_t t = R.u32(), rp = R.u32();
    if (t > (uint32_t)MAX_T || rp > 128) R.ok = false;
    else R.take(32ull * ((8 + rp) * t + (size_t)t * t));
  }
  std::vector<WSignal> sigs;
  if (!R.ok || !read_signals(R, sigs)) {
    err = "witness program: truncated or inconsistent image";
    return ZKFL_E_FORMAT;
  }
  return inputs_from_json(sigs, json, out, err);
}

void wprog_info(const WProg* p, uint32_t* nw, uint32_t* n_in, uint32_t* n_pub) {
  if (nw) *nw = p->n_wires;
  if (n_in) *n_in = p->n_pub_in + p->n_prv_in;
  if (n_pub) *n_pub = p->n_pub_out + p->n_pub_in;
}

int wprog_load(const uint8_t* img, size_t len, hipStream_t st, WProg** out, std::string& err) {
  Reader R{img, len};
  const uint8_t* magic = R.take(4);
  if (!magic || memcmp(magic, "zkwp", 4) != 0 || R.u32() != 2) {
    err = "witness program: bad magic/version";
    return ZKFL_E_FORMAT;
  }
  WProg* p = new WProg();
  p->n_wires = R.u32();
  p->n_pub_out = R.u32();
  p->n_pub_in = R.u32();
  p->n_prv_in = R.u32();
  p->in_first = R.u32();
  p->n_ops = R.u32();
  p->n_levels = R.u32();
  const uint32_t n_lcs = R.u32(), n_terms = R.u32();
  p->n_asserts = R.u32();
  const uint32_t n_tmpl = R.u32(), n_widths = R.u32();
  const uint8_t* lp = R.take(4ull * (p->n_levels + 1));
  const uint8_t* ops = R.take(16ull * p->n_ops);
  const uint8_t* lcp = R.take(4ull * (n_lcs + 1));
  const uint8_t* tw = R.take(4ull * n_terms);
  const uint8_t* tc = R.take(32ull * n_terms);
  const uint8_t* as = R.take(4ull * p->n_asserts);
  const uint8_t* tm = R.take(32ull * n_tmpl);
  std::vector<uint8_t> consts;
  bool ok = R.ok && p->n_wires > 0 && p->in_first == 1 + p->n_pub_out &&
            (uint64_t)p->in_first + p->n_pub_in + p->n_prv_in <= p->n_wires;
  for (uint32_t k = 0; k < n_widths && ok; k++) {
    const uint32_t t = R.u32(), rp = R.u32();
    if (!R.ok || t < 2 || t > (uint32_t)MAX_T || rp > 128) {
      ok = false;
      break;
    }
    const size_t nc = (8 + rp) * t, nm = (size_t)t * t;
    const uint8_t* c = R.take(32 * (nc + nm));
    if (!c) {
      ok = false;
      break;
    }
    p->view.width[t] = {rp, (uint32_t)(consts.size() / 32), (uint32_t)(consts.size() / 32 + nc)};
    consts.insert(consts.end(), c, c + 32 * (nc + nm));
  }
  if (ok && !read_signals(R, p->signals)) ok = false;
  if (ok) {  // the signal table must tile the input range exactly, in declaration order
    uint64_t next = p->in_first;
    for (const WSignal& sg : p->signals) {
      uint64_t cnt = 1;
      for (uint32_t d : sg.dims) cnt *= d;
      ok = ok && sg.first == next;
      next += cnt;
    }
    ok = ok && next == (uint64_t)p->in_first + p->n_pub_in + p->n_prv_in && R.left == 0;
  }
  if (ok) {
    // structural validation (device code trusts these indices)
    p->level_ptr.resize(p->n_levels + 1);
    memcpy(p->level_ptr.data(), lp, 4ull * (p->n_levels + 1));
    std::vector<uint32_t> lcv(n_lcs + 1), twv(n_terms), asv(p->n_asserts), tmv(8ull * n_tmpl);
    memcpy(lcv.data(), lcp, lcv.size() * 4);
    memcpy(twv.data(), tw, twv.size() * 4);
    memcpy(asv.data(), as, asv.size() * 4);
    memcpy(tmv.data(), tm, tmv.size() * 4);
    ok = p->level_ptr[0] == 0 && p->level_ptr[p->n_levels] == p->n_ops && lcv[0] == 0 && lcv[n_lcs] == n_terms;
    for (uint32_t i = 0; ok && i < p->n_levels; i++) ok = p->level_ptr[i] <= p->level_ptr[i + 1];
    for (uint32_t i = 0; ok && i < n_lcs; i++) ok = lcv[i] <= lcv[i + 1];
    for (uint32_t i = 0; ok && i < n_terms; i++) ok = (twv[i] & 0x7FFFFFFFu) < p->n_wires;
    for (uint32_t i = 0; ok && i < p->n_asserts; i++) ok = (uint64_t)asv[i] + 3 <= n_lcs;
    for (uint32_t i = 0; ok && i < p->n_ops; i++) {
      uint32_t o[4];
      memcpy(o, ops + 16ull * i, 16);
      const uint32_t kind = o[0], outw = o[1], lc0 = o[2], aux = o[3];
      uint64_t nout = 1, nlc = 1;
      if (kind == K_MUL) nlc = 2;
      else if (kind == K_BITS) nout = aux, ok = aux >= 1 && aux <= 254;
      else if (kind == K_POS) {
        const uint32_t t = aux & 0xFF, tid = aux >> 8;
        ok = t >= 2 && t <= (uint32_t)MAX_T && tid < n_tmpl && p->view.width[t].rp != 0 &&
             tmv[8ull * tid] == 8 * t + p->view.width[t].rp;  // n_sbox = R_F t + R_P
        if (ok) {
          uint32_t live = 0;
          for (int q = 1; q < 8; q++) live += __builtin_popcount(tmv[8ull * tid + q]);
          nout = 3ull * live;
          nlc = t - 1;
        }
      } else ok = ok && (kind == K_LC || kind == K_INV);
      // outputs: never the constant wire, never an input signal
      const uint64_t in_end = (uint64_t)p->in_first + p->n_pub_in + p->n_prv_in;
      ok = ok && (uint64_t)lc0 + nlc <= n_lcs && (uint64_t)outw + nout <= p->n_wires && outw >= 1 &&
           ((uint64_t)outw + nout <= p->in_first || outw >= in_end);
    }
  }
  if (!ok) {
    wprog_free(p);
    err = "witness program: truncated or inconsistent image";
    return ZKFL_E_FORMAT;
  }
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
    if (!lt_r_host(reinterpret_cast<const uint32_t*>(inputs + 32 * i))) {
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
  for (uint32_t L = 0; L < p->n_levels; L++) {
    const uint32_t op0 = p->level_ptr[L], cnt = p->level_ptr[L + 1] - op0;
    if (cnt) hipLaunchKernelGGL(k_wit_level, dim3(zk_grid(m * cnt, 64)), dim3(64), 0, st, p->view, m, op0, cnt, W);
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

}  // namespace zkfl
