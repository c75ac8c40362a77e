// GPU Poseidon batches, vectorHash and Poseidon Merkle trees (the reference's data/server side).
//
// Reference behaviour (tests/full_system_simulation.mjs): vectorHash :139-156 (Poseidon of <= 16
// values, else Poseidon of the 16-value chunk hashes), the commitments :158-181, buildMerkleTree
// :198-223 (leaves padded to 2^DEPTH with Poseidon([0]), pairs hashed bottom-up with Poseidon(2)),
// getMerkleProof :225-238, computeDatasetCommitment :309-335 (leaf i = vectorHash(features[i] ||
// label[i])).  Same values as oracle/poseidon.py and zkfl/clients.py (pinned by the reference
// fixture data/test_input_v5.json: leaves, root_D, root_G).
//
// Layout and schedule (MI355X): one lane per hash, state in VGPRs, constants in SGPRs
// (csrc/poseidon.h).  A tree is built level by level, one launch per level while a level has more
// than 512 live nodes (one lane per parent, the whole chip busy), then ONE workgroup finishes the
// remaining levels through LDS (the top ~9 levels would otherwise be 9 nearly empty launches).  Only
// nodes above real leaves are hashed: every other node of level l is the zero-subtree hash z_l
// (z_0 = Poseidon([0]), z_{l+1} = Poseidon([z_l, z_l])), which is what the reference's padded tree
// holds there; the padded levels are materialised only when the tree is written out.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "common.h"
#include "merkle.h"
#include "poseidon.h"
#include "zkfl.h"

namespace zkfl {

namespace {

// ---------------------------------------------------------------------------
// Host: circomlib parameter generation (Grain LFSR), restating zkfl/field.py::poseidon_params
// ---------------------------------------------------------------------------
const uint32_t RP_TABLE[16] = {56, 57, 56, 60, 60, 63, 64, 63, 60, 66, 60, 65, 70, 60, 64, 68};  // t = 2..17
const uint64_t R64[4] = {0x43e1f593f0000001ull, 0x2833e84879b97091ull, 0xb85045b68181585dull,
                         0x30644e72e131a029ull};

struct U256 {
  uint64_t w[4] = {0, 0, 0, 0};  // little-endian
};

bool u256_ge(const U256& a, const uint64_t b[4]) {
  for (int i = 3; i >= 0; i--)
    if (a.w[i] != b[i]) return a.w[i] > b[i];
  return true;
}

void u256_sub(U256& a, const uint64_t b[4]) {
  unsigned __int128 borrow = 0;
  for (int i = 0; i < 4; i++) {
    const unsigned __int128 d = (unsigned __int128)a.w[i] - b[i] - borrow;
    a.w[i] = (uint64_t)d;
    borrow = (d >> 64) ? 1 : 0;
  }
}

bool u256_eq(const U256& a, const U256& b) { return !memcmp(a.w, b.w, 32); }

// (a + b) mod r == 0 for a, b < r
bool u256_sum_is_r(const U256& a, const U256& b) {
  unsigned __int128 c = 0;
  uint64_t s[4];
  for (int i = 0; i < 4; i++) {
    c += (unsigned __int128)a.w[i] + b.w[i];
    s[i] = (uint64_t)c;
    c >>= 64;
  }
  const bool zero = !(a.w[0] | a.w[1] | a.w[2] | a.w[3] | b.w[0] | b.w[1] | b.w[2] | b.w[3]);
  return zero || (c == 0 && !memcmp(s, R64, 32));
}

struct Grain {
  unsigned __int128 reg;
  Grain(uint32_t t, uint32_t rp) {
    // field = 1 (2 bits), sbox = 0 (4), n = 254 (12), t (12), R_F = 8 (10), R_P (10), then 30 ones;
    // bit 79 is the oldest.
    unsigned __int128 s = 0;
    const uint32_t vals[6] = {1, 0, 254, t, 8, rp};
    const int widths[6] = {2, 4, 12, 12, 10, 10};
    for (int i = 0; i < 6; i++) s = (s << widths[i]) | vals[i];
    s = (s << 30) | ((1u << 30) - 1);
    reg = s;
    for (int i = 0; i < 160; i++) clock();
  }
  int clock() {
    const int b = (int)(((reg >> 79) ^ (reg >> 66) ^ (reg >> 56) ^ (reg >> 41) ^ (reg >> 28) ^ (reg >> 17)) & 1);
    const unsigned __int128 mask = (((unsigned __int128)1) << 80) - 1;
    reg = ((reg << 1) & mask) | (unsigned __int128)b;
    return b;
  }
  int bit() {  // self-shrinking: emit the second bit of a pair whose first bit is 1
    for (;;) {
      const int first = clock();
      const int second = clock();
      if (first) return second;
    }
  }
  U256 draw() {  // 254 bits, most significant first
    U256 v;
    for (int k = 0; k < 254; k++) {
      v.w[3] = (v.w[3] << 1) | (v.w[2] >> 63);
      v.w[2] = (v.w[2] << 1) | (v.w[1] >> 63);
      v.w[1] = (v.w[1] << 1) | (v.w[0] >> 63);
      v.w[0] = (v.w[0] << 1) | (uint64_t)bit();
    }
    return v;
  }
};

// ---------------------------------------------------------------------------
// Device
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_to_mont(const Fr* in, size_t n, Fr* out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = fp_to_mont(in[i]);
}

// M[i][j] = 1 / (x_i + y_j), Montgomery form; xy raw std (x[t] then y[t])
__global__ __launch_bounds__(64) void k_pos_mds(const Fr* xy, uint32_t t, Fr* M) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= t * t) return;
  const uint32_t i = g / t, j = g % t;
  M[g] = fp_inv(fp_add(fp_to_mont(xy[i]), fp_to_mont(xy[t + j])));
}

// zero-subtree hashes z_0 = Poseidon([0]), z_{l+1} = Poseidon([z_l, z_l]) (Montgomery)
__global__ __launch_bounds__(64) void k_pos_zeros(PosConsts K2, PosConsts K3, Fr* zeros, uint32_t levels) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  Fr s2[2] = {fp_zero<FrP>(), fp_zero<FrP>()};
  Fr z = poseidon_perm0<2>(s2, K2);
  zeros[0] = z;
  for (uint32_t l = 1; l < levels; l++) {
    Fr s3[3] = {fp_zero<FrP>(), z, z};
    z = poseidon_perm0<3>(s3, K3);
    zeros[l] = z;
  }
}

// out[i * out_stride] = Poseidon(in[i * in_stride + 0 .. T-2]); in/out Montgomery or std
template <int T>
__global__ __launch_bounds__(256) void k_poseidon_rows(PosConsts K, size_t n, const Fr* __restrict__ in,
                                                       size_t in_stride, uint32_t in_mont, Fr* __restrict__ out,
                                                       size_t out_stride, uint32_t out_mont) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Fr st[T];
  st[0] = fp_zero<FrP>();
  const Fr* row = in + i * in_stride;
#pragma unroll
  for (int k = 1; k < T; k++) st[k] = in_mont ? row[k - 1] : fp_to_mont(row[k - 1]);
  const Fr h = poseidon_perm0<T>(st, K);
  out[i * out_stride] = out_mont ? h : fp_from_mont(h);
}

// one level of the tree: up[j] = Poseidon(lvl[2j], lvl[2j+1] or z_l)  (Montgomery)
__global__ __launch_bounds__(256) void k_merkle_level(PosConsts K, const Fr* __restrict__ lvl, size_t live,
                                                      const Fr* __restrict__ zero_l, Fr* __restrict__ up,
                                                      size_t up_live) {
  const size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= up_live) return;
  Fr st[3];
  st[0] = fp_zero<FrP>();
  st[1] = lvl[2 * j];
  st[2] = (2 * j + 1 < live) ? lvl[2 * j + 1] : *zero_l;
  up[j] = poseidon_perm0<3>(st, K);
}

struct LevelMap {
  uint64_t off[33];   // compact level offsets in the work buffer
  uint64_t live[33];  // live (non-padding) node count per level
};

constexpr uint32_t TOP_LANES = 256;  // the fused top: <= 2 * 256 live nodes on entry

// levels l0 .. depth-1 -> l0+1 .. depth in one workgroup, the level in flight kept in LDS
__global__ __launch_bounds__(TOP_LANES) void k_merkle_top(PosConsts K, Fr* work, LevelMap map, uint32_t l0,
                                                          uint32_t depth, const Fr* __restrict__ zeros) {
  __shared__ Fr buf[2][2 * TOP_LANES];
  const uint32_t j = threadIdx.x;
  uint32_t live = (uint32_t)map.live[l0];
  for (uint32_t q = j; q < live; q += TOP_LANES) buf[0][q] = work[map.off[l0] + q];
  __syncthreads();
  int cur = 0;
  for (uint32_t l = l0; l < depth; l++) {
    const uint32_t up = (uint32_t)map.live[l + 1];
    if (j < up) {
      Fr st[3];
      st[0] = fp_zero<FrP>();
      st[1] = buf[cur][2 * j];
      st[2] = (2 * j + 1 < live) ? buf[cur][2 * j + 1] : zeros[l];
      const Fr h = poseidon_perm0<3>(st, K);
      buf[cur ^ 1][j] = h;
      work[map.off[l + 1] + j] = h;
    }
    __syncthreads();
    cur ^= 1;
    live = up;
  }
}

// full padded levels, standard form: node g of the output -> (level, index) -> live node or z_l
__global__ __launch_bounds__(256) void k_tree_out(const Fr* __restrict__ work, LevelMap map, uint32_t depth,
                                                  const Fr* __restrict__ zeros, Fr* __restrict__ out) {
  const uint64_t total = (2ull << depth) - 1;
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= total) return;
  uint32_t l = 0;
  uint64_t base = 0, width = 1ull << depth;
  while (g >= base + width) {
    base += width;
    width >>= 1;
    l++;
  }
  const uint64_t idx = g - base;
  const Fr v = idx < map.live[l] ? work[map.off[l] + idx] : zeros[l];
  out[g] = fp_from_mont(v);
}

template <int T>
hipError_t launch_rows(const PosConsts& K, size_t n, const Fr* in, size_t in_stride, bool in_mont, Fr* out,
                       size_t out_stride, bool out_mont, hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_poseidon_rows<T>, dim3(zk_grid(n, 256)), dim3(256), 0, st, K, n, in, in_stride,
                     (uint32_t)in_mont, out, out_stride, (uint32_t)out_mont);
  return hipGetLastError();
}

hipError_t rows_any(const PosConsts* W, uint32_t arity, size_t n, const Fr* in, size_t in_stride, bool in_mont,
                    Fr* out, size_t out_stride, bool out_mont, hipStream_t st) {
  const PosConsts& K = W[arity + 1];
  switch (arity + 1) {
#define ZK_ROWS(T) \
  case T:          \
    return launch_rows<T>(K, n, in, in_stride, in_mont, out, out_stride, out_mont, st);
    ZK_ROWS(2) ZK_ROWS(3) ZK_ROWS(4) ZK_ROWS(5) ZK_ROWS(6) ZK_ROWS(7) ZK_ROWS(8) ZK_ROWS(9)
    ZK_ROWS(10) ZK_ROWS(11) ZK_ROWS(12) ZK_ROWS(13) ZK_ROWS(14) ZK_ROWS(15) ZK_ROWS(16) ZK_ROWS(17)
#undef ZK_ROWS
    default:
      return hipErrorInvalidValue;
  }
}

LevelMap level_map(size_t n, uint32_t depth, size_t* total) {
  LevelMap m = {};
  size_t off = 0, live = n;
  for (uint32_t l = 0; l <= depth; l++) {
    m.off[l] = off;
    m.live[l] = live;
    off += live;
    live = (live + 1) / 2;
  }
  *total = off;
  return m;
}

}  // namespace

constexpr uint32_t ZERO_LEVELS = 33;

struct PosTables {
  Fr* buf = nullptr;      // all widths: C then M per width, Montgomery
  Fr* zeros = nullptr;    // [ZERO_LEVELS] zero-subtree hashes, Montgomery
  PosConsts w[18] = {};   // by width t
};

uint32_t pos_rp(uint32_t t) { return (t >= 2 && t <= 17) ? RP_TABLE[t - 2] : 0; }

void pos_params_raw(uint32_t t, uint8_t* consts_out, uint8_t* xy_out) {
  const uint32_t rp = pos_rp(t);
  Grain g(t, rp);
  const size_t nc = (size_t)(8 + rp) * t;
  for (size_t k = 0; k < nc;) {
    const U256 v = g.draw();
    if (u256_ge(v, R64)) continue;  // rejection sampling below r
    if (consts_out) memcpy(consts_out + 32 * k, v.w, 32);
    k++;
  }
  for (;;) {
    std::vector<U256> xy(2 * t);
    for (auto& v : xy) {
      v = g.draw();
      if (u256_ge(v, R64)) u256_sub(v, R64);  // draw() % r (2^254 < 2r)
    }
    bool ok = true;
    for (uint32_t a = 0; a < 2 * t && ok; a++)
      for (uint32_t b = a + 1; b < 2 * t && ok; b++) ok = !u256_eq(xy[a], xy[b]);
    for (uint32_t a = 0; a < t && ok; a++)
      for (uint32_t b = 0; b < t && ok; b++) ok = !u256_sum_is_r(xy[a], xy[t + b]);
    if (!ok) continue;
    if (xy_out)
      for (uint32_t k = 0; k < 2 * t; k++) memcpy(xy_out + 32 * k, xy[k].w, 32);
    return;
  }
}

void pos_tables_free(PosTables* p) {
  if (!p) return;
  if (p->buf) (void)hipFree(p->buf);
  if (p->zeros) (void)hipFree(p->zeros);
  delete p;
}

int pos_tables_create(PosTables** out, hipStream_t st, std::string& err) {
  // host: raw constants of every width; device: Montgomery form, MDS inverses, zero hashes
  size_t total = 0, off[18] = {}, nc[18] = {};
  for (uint32_t t = 2; t <= 17; t++) {
    off[t] = total;
    nc[t] = (size_t)(8 + pos_rp(t)) * t;
    total += nc[t] + (size_t)t * t;
  }
  std::vector<uint8_t> raw(total * 32, 0);
  PosTables* p = new PosTables();
  Fr* d_raw = nullptr;
  Fr* d_xy = nullptr;
  hipError_t e = hipMalloc(&p->buf, total * 32);
  if (e == hipSuccess) e = hipMalloc(&p->zeros, ZERO_LEVELS * 32);
  if (e == hipSuccess) e = hipMalloc(&d_raw, total * 32);
  if (e == hipSuccess) e = hipMalloc(&d_xy, 16 * 2 * 17 * 32);
  std::vector<uint8_t> xy_all(16 * 2 * 17 * 32, 0);
  for (uint32_t t = 2; t <= 17; t++) {
    pos_params_raw(t, raw.data() + 32 * off[t], xy_all.data() + (size_t)(t - 2) * 2 * 17 * 32);
    p->w[t] = {p->buf + off[t], p->buf + off[t] + nc[t], pos_rp(t)};
  }
  if (e == hipSuccess) e = hipMemcpyAsync(d_raw, raw.data(), raw.size(), hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(d_xy, xy_all.data(), xy_all.size(), hipMemcpyHostToDevice, st);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_to_mont, dim3(zk_grid(total, 256)), dim3(256), 0, st, d_raw, total, p->buf);
    for (uint32_t t = 2; t <= 17; t++)
      hipLaunchKernelGGL(k_pos_mds, dim3(zk_grid(t * t, 64)), dim3(64), 0, st, d_xy + (size_t)(t - 2) * 2 * 17, t,
                         p->buf + off[t] + nc[t]);
    hipLaunchKernelGGL(k_pos_zeros, dim3(1), dim3(64), 0, st, p->w[2], p->w[3], p->zeros, ZERO_LEVELS);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (d_raw) (void)hipFree(d_raw);
  if (d_xy) (void)hipFree(d_xy);
  if (e != hipSuccess) {
    pos_tables_free(p);
    err = std::string("poseidon tables: ") + hipGetErrorString(e);
    return e == hipErrorOutOfMemory ? ZKFL_E_OOM : ZKFL_E_DEVICE;
  }
  *out = p;
  return ZKFL_OK;
}

hipError_t fr_to_mont_batch(const Fr* in, size_t n, Fr* out, hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_to_mont, dim3(zk_grid(n, 256)), dim3(256), 0, st, in, n, out);
  return hipGetLastError();
}

hipError_t poseidon_batch(const PosTables* P, uint32_t arity, size_t n, const Fr* in, Fr* out, hipStream_t st) {
  if (arity < 1 || arity > POS_MAX_ARITY) return hipErrorInvalidValue;
  return rows_any(P->w, arity, n, in, arity, false, out, 1, false, st);
}

hipError_t vector_hash_batch(const PosTables* P, uint32_t len, size_t n, const Fr* in, Fr* out, bool out_mont,
                             Fr* scratch, hipStream_t st) {
  if (len < 1 || len > VHASH_CHUNK * VHASH_CHUNK) return hipErrorInvalidValue;
  if (len <= VHASH_CHUNK) return rows_any(P->w, len, n, in, len, false, out, 1, out_mont, st);
  const uint32_t nch = (len + VHASH_CHUNK - 1) / VHASH_CHUNK;
  for (uint32_t c = 0; c < nch; c++) {
    const uint32_t cl = std::min(VHASH_CHUNK, len - c * VHASH_CHUNK);
    ZK_CHECK(rows_any(P->w, cl, n, in + (size_t)c * VHASH_CHUNK, len, false, scratch + c, nch, true, st));
  }
  return rows_any(P->w, nch, n, scratch, nch, true, out, 1, out_mont, st);
}

size_t merkle_work_size(size_t n, uint32_t depth) {
  size_t total = 0;
  (void)level_map(n, depth, &total);
  return total ? total : 1;
}

hipError_t merkle_build(const PosTables* P, const Fr* leaves_mont, size_t n, uint32_t depth, Fr* tree_std, Fr* work,
                        hipStream_t st) {
  if (depth > 32 || (depth < 64 && n > (1ull << depth))) return hipErrorInvalidValue;
  size_t total = 0;
  const LevelMap map = level_map(n, depth, &total);
  if (n) ZK_CHECK(hipMemcpyAsync(work, leaves_mont, n * 32, hipMemcpyDeviceToDevice, st));
  uint32_t l = 0;
  for (; l < depth && map.live[l] > 2 * TOP_LANES; l++)
    hipLaunchKernelGGL(k_merkle_level, dim3(zk_grid(map.live[l + 1], 256)), dim3(256), 0, st, P->w[3],
                       work + map.off[l], (size_t)map.live[l], P->zeros + l, work + map.off[l + 1],
                       (size_t)map.live[l + 1]);
  if (l < depth && map.live[l] > 0)
    hipLaunchKernelGGL(k_merkle_top, dim3(1), dim3(TOP_LANES), 0, st, P->w[3], work, map, l, depth, P->zeros);
  const uint64_t nodes = (2ull << depth) - 1;
  hipLaunchKernelGGL(k_tree_out, dim3(zk_grid(nodes, 256)), dim3(256), 0, st, work, map, depth, P->zeros, tree_std);
  return hipGetLastError();
}

}  // namespace zkfl
