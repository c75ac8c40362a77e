// Dump of the zkey coefficient CSR that csrc/host_parse.cc builds (tests/test_zkey_csr.py):
//   zkey_csr_dump <zkey> <out>
// out: u32 cshift, u32 ncoef, u32 dom | rowptr [2 (dom + 1)] u32 | per term: col u32, value 8 u32
// (the dictionary resolved, so packed and wide parses dump the same bytes).
#include <stdio.h>

#include <string>
#include <vector>

#include "host_parse.h"

int main(int argc, char** argv) {
  if (argc != 3) return 2;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  std::vector<uint8_t> buf;
  uint8_t tmp[1 << 16];
  size_t got;
  while ((got = fread(tmp, 1, sizeof(tmp), f)) > 0) buf.insert(buf.end(), tmp, tmp + got);
  fclose(f);
  zkfl::ZkeyHost z;
  std::string err;
  if (int rc = zkfl::zkey_parse(buf.data(), buf.size(), z, err)) {
    fprintf(stderr, "parse: %d %s\n", rc, err.c_str());
    return 1;
  }
  FILE* o = fopen(argv[2], "wb");
  if (!o) return 2;
  const uint32_t hdr[3] = {z.cshift, (uint32_t)z.ncoef, z.dom};
  fwrite(hdr, 4, 3, o);
  fwrite(z.rowptr.data(), 4, z.rowptr.size(), o);
  const uint32_t mask = z.cshift ? (1u << z.cshift) - 1 : 0xFFFFFFFFu;
  for (size_t p = 0; p < z.ncoef; p++) {
    const uint32_t col = z.cols[p] & mask;
    const size_t id = z.cshift ? (z.cols[p] >> z.cshift) : p;
    fwrite(&col, 4, 1, o);
    fwrite(&z.coefs[id * 8], 4, 8, o);
  }
  fclose(o);
  printf("cshift %u ncoef %zu\n", z.cshift, z.ncoef);
  return 0;
}
