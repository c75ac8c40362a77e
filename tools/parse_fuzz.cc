// Corpus + mutation driver for the host parsers of libzkfl (csrc/host_parse.cc), built for the CPU
// under AddressSanitizer + UBSan by tests/test_parse_fuzz.py:
//   g++ -std=c++17 -g -O1 -fsanitize=address,undefined -fno-sanitize-recover=all \
//       -I include -I <pkg>/csrc tools/parse_fuzz.cc <pkg>/csrc/host_parse.cc -o parse_fuzz
//   parse_fuzz <zkey> <wtns> <wprog image> <input.json>
// Each well-formed file must parse; then every parser meets every prefix of its file (all of them
// for short files, a strided set plus the header region for long ones), byte flips over the header
// region, every 32/64-bit field of the binfile section table overwritten with hostile sizes
// (0, len, 2^32-1, 2^63, 2^64-16, ...), and hostile input.json texts (deep nesting, huge numbers,
// unterminated strings, wrong shapes).  The sanitizers abort on any out-of-bounds read, overflow or
// undefined behaviour; a clean run prints the number of cases and exits 0.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "host_parse.h"

using namespace zkfl;

static std::vector<uint8_t> slurp(const char* path) {
  std::vector<uint8_t> v;
  FILE* f = fopen(path, "rb");
  if (!f) return v;
  uint8_t buf[1 << 16];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) v.insert(v.end(), buf, buf + n);
  fclose(f);
  return v;
}

static size_t g_cases = 0;

// run `fn` over a private heap copy of exactly `len` bytes (so ASan sees every overread)
template <class F>
static int run_on(const std::vector<uint8_t>& src, size_t len, F fn) {
  std::vector<uint8_t> copy(src.begin(), src.begin() + (ptrdiff_t)len);
  copy.shrink_to_fit();
  g_cases++;
  return fn(copy.empty() ? nullptr : copy.data(), copy.size());
}

template <class F>
static void mutate_binary(const std::vector<uint8_t>& file, bool binfile, F fn) {
  const size_t n = file.size();
  // prefixes
  const size_t stride = n <= 4096 ? 1 : n / 2048;
  for (size_t k = 0; k < n; k += stride) run_on(file, k, fn);
  for (size_t k = 0; k < n && k < 1024; k++) run_on(file, k, fn);
  // byte flips over the header region
  for (size_t i = 0; i < n && i < 512; i++)
    for (uint8_t x : {0x01, 0x80, 0xFF}) {
      std::vector<uint8_t> m = file;
      m[i] ^= x;
      run_on(m, m.size(), fn);
    }
  if (!binfile) return;
  // hostile values in every section-table field (type u32 at off, size u64 at off + 4)
  const uint64_t sizes[] = {0, 1, 11, 12, (uint64_t)n, (uint64_t)n - 12, 0xFFFFFFFFull, 0x100000000ull,
                            1ull << 63, ~0ull - 15, ~0ull};
  uint32_t nsec = 0;
  memcpy(&nsec, file.data() + 8, 4);
  size_t off = 12;
  for (uint32_t s = 0; s < nsec && off + 12 <= n; s++) {
    uint64_t size;
    memcpy(&size, file.data() + off + 4, 8);
    for (uint64_t v : sizes) {
      std::vector<uint8_t> m = file;
      memcpy(m.data() + off + 4, &v, 8);
      run_on(m, m.size(), fn);
    }
    for (uint32_t t : {0u, 1u, 2u, 4u, 9u, 15u, 16u, 0xFFFFFFFFu}) {
      std::vector<uint8_t> m = file;
      memcpy(m.data() + off, &t, 4);
      run_on(m, m.size(), fn);
    }
    // every 32-bit word of the section's first 96 bytes (counts, sizes, n8) set to hostile values
    for (size_t w = 0; w < 96 && off + 12 + w + 4 <= n && w + 4 <= size; w += 4)
      for (uint32_t v : {0u, 1u, 31u, 33u, 0x7FFFFFFFu, 0xFFFFFFFFu}) {
        std::vector<uint8_t> m = file;
        memcpy(m.data() + off + 12 + w, &v, 4);
        run_on(m, m.size(), fn);
      }
    if (size > n - off - 12) break;
    off += 12 + size;
  }
  for (uint32_t v : {0u, 1u, 100u, 0xFFFFFFFFu}) {  // section count
    std::vector<uint8_t> m = file;
    memcpy(m.data() + 8, &v, 4);
    run_on(m, m.size(), fn);
  }
}

int main(int argc, char** argv) {
  if (argc != 5) {
    fprintf(stderr, "usage: %s <zkey> <wtns> <wprog image> <input.json>\n", argv[0]);
    return 2;
  }
  const std::vector<uint8_t> zk = slurp(argv[1]), wt = slurp(argv[2]), wp = slurp(argv[3]), js = slurp(argv[4]);
  if (zk.empty() || wt.empty() || wp.empty() || js.empty()) {
    fprintf(stderr, "unreadable corpus file\n");
    return 2;
  }
  auto zkey = [](const uint8_t* b, size_t l) {
    ZkeyHost z;
    std::string e;
    return zkey_parse(b, l, z, e);
  };
  auto wtns = [](const uint8_t* b, size_t l) {
    WtnsView v;
    std::string e;
    return wtns_parse(b, l, v, e);
  };
  auto wprog = [](const uint8_t* b, size_t l) {
    WProgHost p;
    std::string e;
    int rc = wprog_parse(b, l, p, e);
    std::vector<WSignal> s;
    wprog_signals(b, l, s, e);
    return rc;
  };
  // the well-formed corpus must parse
  if (run_on(zk, zk.size(), zkey) || run_on(wt, wt.size(), wtns) || run_on(wp, wp.size(), wprog)) {
    fprintf(stderr, "corpus file rejected\n");
    return 3;
  }
  std::vector<WSignal> sigs;
  std::string err;
  if (wprog_signals(wp.data(), wp.size(), sigs, err)) return 3;
  std::string text(js.begin(), js.end());
  std::vector<uint32_t> vals;
  if (inputs_from_json(sigs, text.c_str(), vals, err)) {
    fprintf(stderr, "corpus input.json rejected: %s\n", err.c_str());
    return 3;
  }
  mutate_binary(zk, true, zkey);
  mutate_binary(wt, true, wtns);
  mutate_binary(wp, false, wprog);
  // input.json: prefixes, byte flips, hostile documents
  auto json = [&](const std::string& t) {
    std::vector<uint32_t> out;
    std::string e;
    g_cases++;
    return inputs_from_json(sigs, t.c_str(), out, e);
  };
  for (size_t k = 0; k <= text.size(); k += (text.size() > 4096 ? text.size() / 1024 : 1)) json(text.substr(0, k));
  for (size_t i = 0; i < text.size() && i < 2048; i++)
    for (char c : {'"', '[', ']', '{', '}', ',', ':', '-', 'x', '\\', '\0'}) {
      std::string m = text;
      m[i] = c;
      json(m);
    }
  json(std::string(100000, '['));
  json(std::string(100000, '{'));
  json("{\"a\":" + std::string(5000, '9') + "}");
  json("{\"" + std::string(10000, 'k'));
  json("[1,2,3]");
  json("{}");
  json("");
  printf("parse_fuzz: %zu cases, no sanitizer findings\n", g_cases);
  return 0;
}
