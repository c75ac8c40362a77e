// Host-side parsers of everything the C ABI accepts as bytes or text: the iden3 binfile container,
// snarkjs .wtns and groth16 .zkey, the witness-program image written by
// zkfl/wprog.py, and circom's input.json.  Pure C++ (no HIP): libzkfl links it, and
// tools/parse_fuzz.cc links the same file under AddressSanitizer/UBSan for the corpus test
// (tests/test_parse_fuzz.py).
//
// Every reader checks a length before it reads: offsets are compared as `need > len - off` (never
// `off + need > len`, which wraps for a crafted 64-bit size), counts taken from a file are bounded
// before they size an allocation, and a failed check returns ZKFL_E_FORMAT / ZKFL_E_PRIME /
// ZKFL_E_MISMATCH / ZKFL_E_ARG with a message, leaving the outputs unspecified.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

namespace zkfl {

// ---------------------------------------------------------------------------
// iden3 binfile: magic (4) | version u32 | nSections u32 | {type u32, size u64, data}*
// ---------------------------------------------------------------------------
struct Section {
  size_t off = 0, size = 0;
  bool present = false;
};
int binfile_sections(const uint8_t* buf, size_t len, const char magic[4], std::vector<Section>& secs,
                     std::string& err);

// .wtns v2: section 1 = n8 u32 | prime (n8 B) | nWitness u32; section 2 = nWitness x 32 B std
struct WtnsView {
  const uint8_t* data = nullptr;
  uint32_t n = 0;
};
int wtns_parse(const uint8_t* buf, size_t len, WtnsView& out, std::string& err);

// groth16 .zkey -> header, point sections, and the QAP coefficients as CSR rows (A rows then B
// rows over one term array) with the packed-dictionary encoding of csrc/zkfl.hip::k_abc_chunks.
struct ZkeyHost {
  uint32_t nVars = 0, nPub = 0, dom = 0;
  int logn = 0;
  size_t nC = 0;  // C query length nVars - nPub - 1
  const uint8_t* pts = nullptr;  // alpha1 64 | beta1 64 | beta2 128 | gamma2 128 | delta1 64 | delta2 128
  const uint8_t *secA = nullptr, *secB1 = nullptr, *secB2 = nullptr, *secC = nullptr, *secH = nullptr;
  size_t ncoef = 0;
  std::vector<uint32_t> rowptr;  // [2 (dom + 1)]: A row pointers, then B row pointers offset by nnz(A)
  std::vector<uint32_t> cols;    // packed terms (col | dict index << cshift) or plain columns
  std::vector<uint32_t> coefs;   // dictionary (packed) or one coefficient per term, 8 u32 each
  uint32_t cshift = 0;           // 0 = wide terms
};
int zkey_parse(const uint8_t* buf, size_t len, ZkeyHost& out, std::string& err);

// ---------------------------------------------------------------------------
// Witness-program image (zkfl/wprog.py, "zkwp" v2)
// ---------------------------------------------------------------------------
enum : uint32_t { K_LC = 0, K_MUL = 1, K_INV = 2, K_BITS = 3, K_POS = 4 };
constexpr int MAX_T = 17;

struct WSignal {  // one declared input signal (input.json key)
  std::string name;
  std::vector<uint32_t> dims;
  uint32_t first = 0;
  uint32_t pub = 0;
};

struct PosWidthHost {
  uint32_t rp = 0, c_off = 0, m_off = 0;  // in Fr units within `consts`
};

// A validated image: the device code may trust every index in it.
struct WProgHost {
  uint32_t n_wires = 0, n_pub_out = 0, n_pub_in = 0, n_prv_in = 0, in_first = 0;
  uint32_t n_ops = 0, n_levels = 0, n_lcs = 0, n_terms = 0, n_asserts = 0, n_tmpl = 0;
  std::vector<uint32_t> level_ptr;
  const uint8_t *ops = nullptr, *lc_ptr = nullptr, *term_wire = nullptr, *term_coef = nullptr,
                *asserts = nullptr, *tmpl = nullptr;  // views into the image
  std::vector<uint8_t> consts;                         // Poseidon constants of every width used
  PosWidthHost width[MAX_T + 1];
  std::vector<WSignal> signals;
};
int wprog_parse(const uint8_t* img, size_t len, WProgHost& out, std::string& err);
// The signal table alone (zkfl_wprog_parse_inputs: no structural validation of the ops).
int wprog_signals(const uint8_t* img, size_t len, std::vector<WSignal>& out, std::string& err);

// circom's input.json -> flattened input signals (n_inputs x 8 u32 std form, reduced mod r).
int inputs_from_json(const std::vector<WSignal>& sigs, const char* json, std::vector<uint32_t>& out,
                     std::string& err);

bool fr_lt_r(const uint32_t v[8]);

}  // namespace zkfl
