// Host-side parsers (see host_parse.h).  Formats: SURVEY.md Appendix A (iden3 binfile, snarkjs .wtns
// v2 and groth16 .zkey, as `snarkjs groth16 prove` reads them, tests/full_system_simulation.mjs:773-776),
// zkfl/wprog.py's witness-program image, and circom's input.json (generate_witness.cjs, :758-767).
#include "host_parse.h"

#include <stdlib.h>
#include <string.h>

#include <cctype>
#include <algorithm>
#include <thread>

#include "zkfl.h"

namespace zkfl {

namespace {

const uint32_t R_LIMBS[8] = {0xf0000001u, 0x43e1f593u, 0x79b97091u, 0x2833e848u,
                             0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
const uint32_t Q_LIMBS[8] = {0xd87cfd47u, 0x3c208c16u, 0x6871ca8du, 0x97816a91u,
                             0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};

int bad(std::string& err, int code, const std::string& msg) {
  err = msg;
  return code;
}

uint32_t rd32(const uint8_t* p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}

// bounded sequential reader over an image
struct Reader {
  const uint8_t* p;
  size_t left;
  bool ok = true;
  const uint8_t* take(uint64_t n) {
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
    return q ? rd32(q) : 0;
  }
};

bool read_signals(Reader& R, uint32_t n_wires, std::vector<WSignal>& out) {
  const uint32_t n = R.u32();
  if (!R.ok || n > (1u << 20)) return false;
  for (uint32_t i = 0; i < n; i++) {
    WSignal sg;
    const uint32_t len = R.u32();
    if (!R.ok || len > 4096) return false;
    const uint8_t* nm = R.take((len + 3ull) & ~3ull);
    if (!nm) return false;
    sg.name.assign(reinterpret_cast<const char*>(nm), len);
    const uint32_t nd = R.u32();
    if (!R.ok || nd > 16) return false;
    uint64_t cnt = 1;
    for (uint32_t d = 0; d < nd; d++) {
      const uint32_t dim = R.u32();
      // a signal never has more elements than the program has wires (no overflow of cnt)
      if (dim == 0 || dim > n_wires || cnt * dim > n_wires) return false;
      cnt *= dim;
      sg.dims.push_back(dim);
    }
    sg.first = R.u32();
    sg.pub = R.u32();
    if (!R.ok) return false;
    out.push_back(std::move(sg));
  }
  return true;
}

// ---------------------------------------------------------------------------
// input.json.  The subset circom's witness calculator accepts for these circuits: one object
// mapping signal names to a number, a decimal (or 0x hex) string, or nested arrays of those;
// negatives are reduced mod r as circom does.  Extra keys are ignored (as zkfl/r1cs.py does).
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

// decimal / 0x-hex integer literal (optional sign) -> std-form Fr limbs (mod r).  Digits are
// consumed in chunks of 18 (decimal) / 15 (hex) into a value kept below r: acc = acc * base^len +
// chunk (< r * 2^60 < 2^314), then reduced with a quotient estimated from its top 128 bits over
// r's top word plus one (never above the true quotient, at most 2 short), and <= 3 subtractions.
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
  const size_t per = base == 10 ? 18 : 15;  // base^per <= 2^60
  uint64_t acc[5] = {0, 0, 0, 0, 0};
  auto ge_r = [&]() {
    if (acc[4]) return true;
    for (int k = 3; k >= 0; k--)
      if (acc[k] != RL[k]) return acc[k] > RL[k];
    return true;
  };
  auto sub_qr = [&](uint64_t q) {  // acc -= q * r
    unsigned __int128 prod = 0;
    uint64_t borrow = 0;
    for (int k = 0; k < 5; k++) {
      prod += (unsigned __int128)(k < 4 ? RL[k] : 0) * q;
      const uint64_t p = (uint64_t)prod;
      prod >>= 64;
      const unsigned __int128 sub = (unsigned __int128)p + borrow;
      borrow = (unsigned __int128)acc[k] < sub ? 1 : 0;
      acc[k] = (uint64_t)((unsigned __int128)acc[k] - sub);
    }
  };
  while (i < t.size()) {
    const size_t take = t.size() - i < per ? t.size() - i : per;
    uint64_t v = 0, m = 1;
    for (size_t j = 0; j < take; j++, i++) {
      const char ch = t[i];
      unsigned d;
      if (ch >= '0' && ch <= '9') d = ch - '0';
      else if (base == 16 && ch >= 'a' && ch <= 'f') d = ch - 'a' + 10;
      else if (base == 16 && ch >= 'A' && ch <= 'F') d = ch - 'A' + 10;
      else return false;  // fractions / exponents are not field elements
      v = v * base + d;
      m *= base;
    }
    unsigned __int128 c = v;  // acc < r before: acc * m + v < 2^314
    for (int k = 0; k < 5; k++) {
      c += (unsigned __int128)acc[k] * m;
      acc[k] = (uint64_t)c;
      c >>= 64;
    }
    const unsigned __int128 top = ((unsigned __int128)acc[4] << 64) | acc[3];
    const uint64_t q = (uint64_t)(top / ((unsigned __int128)RL[3] + 1));
    if (q) sub_qr(q);
    while (ge_r()) sub_qr(1);
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

// the header of a "zkwp" v2 image, then its section views (shared by the two image readers)
struct WHeader {
  uint32_t h[12];
};

bool wprog_header(Reader& R, WHeader& H) {
  const uint8_t* magic = R.take(4);
  if (!magic || memcmp(magic, "zkwp", 4) != 0 || R.u32() != 2) return false;
  for (int i = 0; i < 12; i++) H.h[i] = R.u32();
  return R.ok;
}

}  // namespace

bool fr_lt_r(const uint32_t v[8]) {
  for (int i = 7; i >= 0; i--)
    if (v[i] != R_LIMBS[i]) return v[i] < R_LIMBS[i];
  return false;
}

int binfile_sections(const uint8_t* buf, size_t len, const char magic[4], std::vector<Section>& secs,
                     std::string& err) {
  if (!buf || len < 12) return bad(err, ZKFL_E_FORMAT, "file too short");
  if (memcmp(buf, magic, 4) != 0) return bad(err, ZKFL_E_FORMAT, std::string("bad magic, expected ") + magic);
  const uint32_t nsec = rd32(buf + 8);
  size_t off = 12;
  secs.assign(16, Section());
  for (uint32_t i = 0; i < nsec; i++) {
    if (12 > len - off) return bad(err, ZKFL_E_FORMAT, "truncated section header");
    const uint32_t typ = rd32(buf + off);
    uint64_t size;
    memcpy(&size, buf + off + 4, 8);
    off += 12;
    if (size > len - off) return bad(err, ZKFL_E_FORMAT, "truncated section");  // len >= off here
    if (typ < secs.size() && !secs[typ].present) {
      secs[typ].off = off;
      secs[typ].size = (size_t)size;
      secs[typ].present = true;
    }
    off += (size_t)size;
  }
  return ZKFL_OK;
}

int wtns_parse(const uint8_t* buf, size_t len, WtnsView& out, std::string& err) {
  std::vector<Section> s;
  int rc = binfile_sections(buf, len, "wtns", s, err);
  if (rc) return rc;
  if (!s[1].present || !s[2].present) return bad(err, ZKFL_E_FORMAT, "wtns: missing section");
  if (s[1].size < 4 + 32 + 4) return bad(err, ZKFL_E_FORMAT, "wtns: header section too short");
  const uint8_t* h = buf + s[1].off;
  if (rd32(h) != 32) return bad(err, ZKFL_E_FORMAT, "wtns: n8 != 32");
  if (memcmp(h + 4, R_LIMBS, 32) != 0) return bad(err, ZKFL_E_PRIME, "wtns: prime is not bn128 r");
  out.n = rd32(h + 36);
  if (s[2].size != (size_t)out.n * 32) return bad(err, ZKFL_E_FORMAT, "wtns: section 2 size");
  out.data = buf + s[2].off;
  return ZKFL_OK;
}

// Coefficient dictionary: open addressing over the 32-byte values (a circuit's coefficients take
// few distinct values -- 1971 over the metric circuit's 7.0 M terms).
struct CoefDict {
  std::vector<uint32_t> slot;  // id + 1, 0 = empty
  std::vector<uint32_t> vals;  // 8 u32 per id
  uint32_t mask = 0;
  CoefDict() { rehash(1024); }
  uint32_t size() const { return (uint32_t)(vals.size() / 8); }
  static uint32_t hash(const uint32_t* v) {
    uint64_t h = 0x9E3779B97F4A7C15ull;
    for (int i = 0; i < 8; i++) h = (h ^ v[i]) * 0x100000001B3ull;
    return (uint32_t)(h ^ (h >> 31));
  }
  void rehash(uint32_t cap) {
    slot.assign(cap, 0);
    mask = cap - 1;
    for (uint32_t id = 0; id < size(); id++) {
      uint32_t i = hash(&vals[(size_t)id * 8]) & mask;
      while (slot[i]) i = (i + 1) & mask;
      slot[i] = id + 1;
    }
  }
  uint32_t intern(const uint8_t* p) {
    uint32_t v[8];
    memcpy(v, p, 32);
    uint32_t i = hash(v) & mask;
    for (;; i = (i + 1) & mask) {
      const uint32_t e = slot[i];
      if (!e) break;
      if (memcmp(&vals[(size_t)(e - 1) * 8], v, 32) == 0) return e - 1;
    }
    const uint32_t id = size();
    vals.insert(vals.end(), v, v + 8);
    slot[i] = id + 1;
    if (2 * (size_t)size() > slot.size()) rehash((uint32_t)slot.size() * 2);
    return id;
  }
};

// Section 4 (ncoef x {matrix, constraint, signal, value}) -> CSR rows (A rows, then B rows over one
// term array), terms in file order within each row.  Contiguous ranges of the entries go to
// threads: each validates its range, counts its terms per row and interns the values in its own
// dictionary; the dictionaries merge in range order, thread t's terms of row j start after the
// earlier ranges' terms of row j, and the scatter runs in parallel again.  Terms pack col | value
// id << cshift when both fit a u32 (otherwise every term keeps its 32-byte value: cshift = 0).
int coef_csr(const uint8_t* ent, uint32_t ncoef, ZkeyHost& z, std::string& err) {
  const size_t dom = z.dom, rows = 2 * (dom + 1);
  uint32_t colbits = 1;
  while (colbits < 32 && (1ull << colbits) < z.nVars) colbits++;
#ifndef ZK_COEF_DICT_MAX
#define ZK_COEF_DICT_MAX 0xFFFFFFFFull  // tests build a smaller cap to reach the wide path
#endif
  const uint64_t id_limit = colbits < 32 ? std::min<uint64_t>(1ull << (32 - colbits), ZK_COEF_DICT_MAX) : 0;
  unsigned T = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
  T = (unsigned)std::min<size_t>(T, std::max<size_t>(1, ncoef / 65536));
  if (const char* e = getenv("ZKFL_PARSE_THREADS")) T = (unsigned)std::max(1, std::min(64, atoi(e)));
  T = (unsigned)std::min<size_t>(T, std::max<size_t>(1, ((size_t)256 << 20) / (rows * 4)));  // histograms
  std::vector<std::vector<uint32_t>> hist(T);
  std::vector<CoefDict> dicts(T);
  std::vector<uint32_t> lid(ncoef);
  std::vector<int> badr(T, 0);
  auto range = [&](unsigned t, size_t& a, size_t& b) {
    a = (size_t)ncoef * t / T;
    b = (size_t)ncoef * (t + 1) / T;
  };
  auto par = [&](auto&& fn) {
    std::vector<std::thread> th;
    for (unsigned t = 1; t < T; t++) th.emplace_back(fn, t);
    fn(0u);
    for (auto& x : th) x.join();
  };
  par([&](unsigned t) {
    size_t a, b;
    range(t, a, b);
    std::vector<uint32_t>& h = hist[t];
    h.assign(rows, 0);
    CoefDict& d = dicts[t];
    for (size_t i = a; i < b; i++) {
      const uint8_t* e = ent + i * 44;
      uint32_t mcs[3];
      memcpy(mcs, e, 12);
      if (mcs[0] > 1 || mcs[1] >= dom || mcs[2] >= z.nVars) {
        badr[t] = 1;
        return;
      }
      h[mcs[0] * (dom + 1) + mcs[1]]++;
      if (id_limit) lid[i] = d.intern(e + 12);
    }
  });
  for (int x : badr)
    if (x) return bad(err, ZKFL_E_FORMAT, "zkey: coefficient out of range");
  // merged dictionary (range order) and each range's local -> merged id map
  CoefDict g;
  std::vector<std::vector<uint32_t>> gmap(T);
  bool packed = id_limit != 0 && ncoef != 0;
  for (unsigned t = 0; t < T && packed; t++) {
    const CoefDict& d = dicts[t];
    gmap[t].resize(d.size());
    for (uint32_t j = 0; j < d.size() && packed; j++) {
      gmap[t][j] = g.intern(reinterpret_cast<const uint8_t*>(&d.vals[(size_t)j * 8]));
      packed = g.size() <= id_limit;
    }
  }
  // row pointers: per row, the ranges' counts in order; hist[t][row] becomes range t's first slot
  std::vector<uint32_t>& rowptr = z.rowptr;
  rowptr.assign(rows, 0);
  size_t run = 0;
  for (size_t m = 0; m < 2; m++)
    for (size_t j = 0; j < dom; j++) {
      const size_t r = m * (dom + 1) + j;
      rowptr[r] = (uint32_t)run;
      for (unsigned t = 0; t < T; t++) {
        const uint32_t c = hist[t][r];
        hist[t][r] = (uint32_t)run;
        run += c;
      }
      if (j + 1 == dom) rowptr[r + 1] = (uint32_t)run;
    }
  // rowptr[m (dom + 1) + j] = first term of row j of matrix m; rowptr[dom] = nA = rowptr[dom + 1]
  std::vector<uint32_t> cols(ncoef);
  std::vector<uint32_t> coefs(packed ? 0 : (size_t)ncoef * 8);
  par([&](unsigned t) {
    size_t a, b;
    range(t, a, b);
    std::vector<uint32_t>& h = hist[t];
    const uint32_t* gm = packed ? gmap[t].data() : nullptr;
    for (size_t i = a; i < b; i++) {
      const uint8_t* e = ent + i * 44;
      uint32_t mcs[3];
      memcpy(mcs, e, 12);
      const uint32_t pos = h[mcs[0] * (dom + 1) + mcs[1]]++;
      if (packed) {
        cols[pos] = mcs[2] | (gm[lid[i]] << colbits);
      } else {
        cols[pos] = mcs[2];
        memcpy(&coefs[(size_t)pos * 8], e + 12, 32);
      }
    }
  });
  z.cshift = packed ? colbits : 0;
  z.cols.swap(cols);
  if (packed)
    z.coefs.swap(g.vals);
  else
    z.coefs.swap(coefs);
  return ZKFL_OK;
}

int zkey_parse(const uint8_t* buf, size_t len, ZkeyHost& z, std::string& err) {
  std::vector<Section> s;
  int rc = binfile_sections(buf, len, "zkey", s, err);
  if (rc) return rc;
  for (int i = 1; i <= 9; i++)
    if (!s[i].present) return bad(err, ZKFL_E_FORMAT, "zkey: missing section " + std::to_string(i));
  if (s[1].size < 4 || rd32(buf + s[1].off) != 1) return bad(err, ZKFL_E_FORMAT, "zkey: not a groth16 key");
  constexpr size_t HDR = 84 + 64 * 3 + 128 * 3;  // n8q q n8r r nVars nPub dom | 6 points
  if (s[2].size < HDR) return bad(err, ZKFL_E_FORMAT, "zkey: header size");
  const uint8_t* h = buf + s[2].off;
  if (rd32(h) != 32 || memcmp(h + 4, Q_LIMBS, 32) != 0) return bad(err, ZKFL_E_PRIME, "zkey: q is not bn128");
  if (rd32(h + 36) != 32 || memcmp(h + 40, R_LIMBS, 32) != 0) return bad(err, ZKFL_E_PRIME, "zkey: r is not bn128");
  z.nVars = rd32(h + 72);
  z.nPub = rd32(h + 76);
  z.dom = rd32(h + 80);
  z.pts = h + 84;
  int logn = 0;
  while (logn < 31 && (1ull << logn) < z.dom) logn++;
  if ((1ull << logn) != z.dom || logn > 28 || z.dom < 2) return bad(err, ZKFL_E_FORMAT, "zkey: domain size");
  z.logn = logn;
  if ((uint64_t)z.nVars < (uint64_t)z.nPub + 1) return bad(err, ZKFL_E_FORMAT, "zkey: nVars < nPublic+1");
  z.nC = (size_t)z.nVars - z.nPub - 1;
  if (s[3].size != ((size_t)z.nPub + 1) * 64 || s[5].size != (size_t)z.nVars * 64 ||
      s[6].size != (size_t)z.nVars * 64 || s[7].size != (size_t)z.nVars * 128 || s[8].size != z.nC * 64 ||
      s[9].size != (size_t)z.dom * 64)
    return bad(err, ZKFL_E_MISMATCH, "zkey: section sizes do not match header");
  z.secA = buf + s[5].off;
  z.secB1 = buf + s[6].off;
  z.secB2 = buf + s[7].off;
  z.secC = buf + s[8].off;
  z.secH = buf + s[9].off;
  // coefficients -> CSR (sizes above bound every allocation by the input length)
  if (s[4].size < 4) return bad(err, ZKFL_E_FORMAT, "zkey: coefficient section size");
  const uint8_t* cs = buf + s[4].off;
  const uint32_t ncoef = rd32(cs);
  if (s[4].size != 4 + (size_t)ncoef * 44) return bad(err, ZKFL_E_FORMAT, "zkey: coefficient section size");
  z.ncoef = ncoef;
  return coef_csr(cs + 4, ncoef, z, err);
}

int wprog_signals(const uint8_t* img, size_t len, std::vector<WSignal>& sigs, std::string& err) {
  Reader R{img, len};
  WHeader H;
  if (!img || !wprog_header(R, H)) return bad(err, ZKFL_E_FORMAT, "witness program: bad magic/version");
  const uint32_t n_wires = H.h[0], n_ops = H.h[5], n_levels = H.h[6], n_lcs = H.h[7], n_terms = H.h[8],
                 n_asserts = H.h[9], n_tmpl = H.h[10], n_widths = H.h[11];
  R.take(4ull * (n_levels + 1ull));
  R.take(16ull * n_ops);
  R.take(4ull * (n_lcs + 1ull));
  R.take(36ull * n_terms);
  R.take(4ull * n_asserts);
  R.take(32ull * n_tmpl);
  for (uint32_t k = 0; k < n_widths && R.ok; k++) {
    const uint32_t t = R.u32(), rp = R.u32();
    if (t > (uint32_t)MAX_T || rp > 128) R.ok = false;
    else R.take(32ull * ((8ull + rp) * t + (uint64_t)t * t));
  }
  if (!R.ok || !read_signals(R, n_wires, sigs))
    return bad(err, ZKFL_E_FORMAT, "witness program: truncated or inconsistent image");
  return ZKFL_OK;
}

int wprog_parse(const uint8_t* img, size_t len, WProgHost& p, std::string& err) {
  Reader R{img, len};
  WHeader H;
  if (!img || !wprog_header(R, H)) return bad(err, ZKFL_E_FORMAT, "witness program: bad magic/version");
  p.n_wires = H.h[0];
  p.n_pub_out = H.h[1];
  p.n_pub_in = H.h[2];
  p.n_prv_in = H.h[3];
  p.in_first = H.h[4];
  p.n_ops = H.h[5];
  p.n_levels = H.h[6];
  p.n_lcs = H.h[7];
  p.n_terms = H.h[8];
  p.n_asserts = H.h[9];
  p.n_tmpl = H.h[10];
  const uint32_t n_widths = H.h[11];
  const uint8_t* lp = R.take(4ull * (p.n_levels + 1ull));
  p.ops = R.take(16ull * p.n_ops);
  p.lc_ptr = R.take(4ull * (p.n_lcs + 1ull));
  p.term_wire = R.take(4ull * p.n_terms);
  p.term_coef = R.take(32ull * p.n_terms);
  p.asserts = R.take(4ull * p.n_asserts);
  p.tmpl = R.take(32ull * p.n_tmpl);
  const uint64_t in_end = (uint64_t)p.in_first + p.n_pub_in + p.n_prv_in;
  bool ok = R.ok && p.n_wires > 0 && (uint64_t)p.in_first == 1ull + p.n_pub_out && in_end <= p.n_wires;
  for (uint32_t k = 0; k < n_widths && ok; k++) {
    const uint32_t t = R.u32(), rp = R.u32();
    if (!R.ok || t < 2 || t > (uint32_t)MAX_T || rp > 128) {
      ok = false;
      break;
    }
    const size_t nc = (8 + rp) * t, nm = (size_t)t * t;
    const uint8_t* c = R.take(32ull * (nc + nm));
    if (!c) {
      ok = false;
      break;
    }
    p.width[t] = {rp, (uint32_t)(p.consts.size() / 32), (uint32_t)(p.consts.size() / 32 + nc)};
    p.consts.insert(p.consts.end(), c, c + 32 * (nc + nm));
  }
  if (ok && !read_signals(R, p.n_wires, p.signals)) ok = false;
  if (ok) {  // the signal table must tile the input range exactly, in declaration order
    uint64_t next = p.in_first;
    for (const WSignal& sg : p.signals) {
      uint64_t cnt = 1;
      for (uint32_t d : sg.dims) cnt *= d;  // <= n_wires (read_signals)
      ok = ok && sg.first == next;
      next += cnt;
    }
    ok = ok && next == in_end && R.left == 0;
  }
  if (ok) {
    // structural validation (device code trusts these indices)
    p.level_ptr.resize(p.n_levels + 1ull);
    memcpy(p.level_ptr.data(), lp, 4ull * (p.n_levels + 1ull));
    std::vector<uint32_t> lcv(p.n_lcs + 1ull), twv(p.n_terms), asv(p.n_asserts), tmv(8ull * p.n_tmpl);
    memcpy(lcv.data(), p.lc_ptr, lcv.size() * 4);
    memcpy(twv.data(), p.term_wire, twv.size() * 4);
    memcpy(asv.data(), p.asserts, asv.size() * 4);
    memcpy(tmv.data(), p.tmpl, tmv.size() * 4);
    ok = p.level_ptr[0] == 0 && p.level_ptr[p.n_levels] == p.n_ops && lcv[0] == 0 && lcv[p.n_lcs] == p.n_terms;
    for (uint32_t i = 0; ok && i < p.n_levels; i++) ok = p.level_ptr[i] <= p.level_ptr[i + 1];
    for (uint32_t i = 0; ok && i < p.n_lcs; i++) ok = lcv[i] <= lcv[i + 1];
    for (uint32_t i = 0; ok && i < p.n_terms; i++) ok = (twv[i] & 0x7FFFFFFFu) < p.n_wires;
    for (uint32_t i = 0; ok && i < p.n_asserts; i++) ok = (uint64_t)asv[i] + 3 <= p.n_lcs;
    for (uint32_t i = 0; ok && i < p.n_ops; i++) {
      uint32_t o[4];
      memcpy(o, p.ops + 16ull * i, 16);
      const uint32_t kind = o[0], outw = o[1], lc0 = o[2], aux = o[3];
      uint64_t nout = 1, nlc = 1;
      if (kind == K_MUL) nlc = 2;
      else if (kind == K_BITS) nout = aux, ok = aux >= 1 && aux <= 254;
      else if (kind == K_POS) {
        const uint32_t t = aux & 0xFF, tid = aux >> 8;
        ok = t >= 2 && t <= (uint32_t)MAX_T && tid < p.n_tmpl && p.width[t].rp != 0 &&
             tmv[8ull * tid] == 8 * t + p.width[t].rp;  // n_sbox = R_F t + R_P
        if (ok) {
          uint32_t live = 0;
          for (int q = 1; q < 8; q++) live += __builtin_popcount(tmv[8ull * tid + q]);
          nout = 3ull * live;
          nlc = t - 1;
        }
      } else ok = ok && (kind == K_LC || kind == K_INV);
      // outputs: never the constant wire, never an input signal
      ok = ok && (uint64_t)lc0 + nlc <= p.n_lcs && (uint64_t)outw + nout <= p.n_wires && outw >= 1 &&
           ((uint64_t)outw + nout <= p.in_first || outw >= in_end);
    }
  }
  if (!ok) return bad(err, ZKFL_E_FORMAT, "witness program: truncated or inconsistent image");
  return ZKFL_OK;
}

int inputs_from_json(const std::vector<WSignal>& sigs, const char* json, std::vector<uint32_t>& out,
                     std::string& err) {
  if (!json) return bad(err, ZKFL_E_ARG, "null input json");
  JParser P{json, json + strlen(json), ""};
  JVal root;
  if (!P.value(root, 0)) return bad(err, ZKFL_E_ARG, "input json: " + P.err);
  P.ws();
  if (P.s != P.e || root.kind != JVal::OBJECT)
    return bad(err, ZKFL_E_ARG, "input json: expected one object of signal names");
  for (const WSignal& sg : sigs) {
    size_t k = 0;
    while (k < root.keys.size() && root.keys[k] != sg.name) k++;
    if (k == root.keys.size()) return bad(err, ZKFL_E_ARG, "missing input signal '" + sg.name + "'");
    if (!flatten(root.items[k], sg, 0, out, err)) return ZKFL_E_ARG;
  }
  return ZKFL_OK;
}

}  // namespace zkfl
