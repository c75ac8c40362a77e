// NTT kernels (see ntt.h for the algorithm and the reference behaviour it replaces).
#include "ntt.h"
#include "fr_consts.h"
#include "wtrace.h"

namespace zkfl {

#ifndef NTT_LDS_LOG_BITS
#define NTT_LDS_LOG_BITS 10
#endif
constexpr int NTT_LDS_LOG = NTT_LDS_LOG_BITS;
constexpr int NTT_LDS_N = 1 << NTT_LDS_LOG;

// tw[i] = root^i (Montgomery) for i < n/2
__global__ void k_ntt_twiddles(Fr* __restrict__ tw, size_t half, Fr root_mont) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= half) return;
  // root^i by square-and-multiply over the bits of i
  Fr acc = fp_one<FrP>();
  Fr base = root_mont;
  size_t e = i;
  while (e) {
    if (e & 1) acc = fp_mul(acc, base);
    base = fp_sqr(base);
    e >>= 1;
  }
  tw[i] = acc;
}

// coset[p] = inc^{bitrev(p)} / n (Montgomery), p < n
__global__ void k_ntt_coset_table(Fr* __restrict__ tab, size_t n, int logn, Fr inc_mont, Fr ninv_mont) {
  size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  size_t i = __brevll((unsigned long long)p) >> (64 - logn);
  Fr acc = ninv_mont;
  Fr base = inc_mont;
  size_t e = i;
  while (e) {
    if (e & 1) acc = fp_mul(acc, base);
    base = fp_sqr(base);
    e >>= 1;
  }
  tab[p] = acc;
}

// One global DIF stage (span `half`, len = 2*half); tw stride = n / len.
__global__ void k_ntt_dif_stage(Fr* __restrict__ a, size_t n, size_t half, const Fr* __restrict__ tw,
                                size_t twstride, int nvec, size_t vstride) {
  size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t nb = n >> 1;
  if (t >= nb * nvec) return;
  size_t v = t / nb;
  t -= v * nb;
  Fr* x = a + v * vstride;
  size_t j = t & (half - 1);
  size_t i0 = ((t - j) << 1) + j;
  size_t i1 = i0 + half;
  Fr u = x[i0], w = x[i1];
  x[i0] = fp_add(u, w);
  x[i1] = fp_mul(fp_sub(u, w), tw[j * twstride]);
}

__global__ void k_ntt_dit_stage(Fr* __restrict__ a, size_t n, size_t half, const Fr* __restrict__ tw,
                                size_t twstride, int nvec, size_t vstride) {
  size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t nb = n >> 1;
  if (t >= nb * nvec) return;
  size_t v = t / nb;
  t -= v * nb;
  Fr* x = a + v * vstride;
  size_t j = t & (half - 1);
  size_t i0 = ((t - j) << 1) + j;
  size_t i1 = i0 + half;
  Fr u = x[i0];
  Fr w = fp_mul(x[i1], tw[j * twstride]);
  x[i0] = fp_add(u, w);
  x[i1] = fp_sub(u, w);
}

// Fused small-span stages inside one LDS tile of T = min(n, 1024) elements.
//   DIF: spans T/2 .. 1 (the last log2 T stages of the inverse transform)
//   DIT: spans 1 .. T/2 (the first log2 T stages of the forward transform)
template <bool DIF>
__global__ void __launch_bounds__(512) k_ntt_lds(Fr* __restrict__ a, size_t n, int logt,
                                                 const Fr* __restrict__ tw, int nvec, size_t vstride,
                                                 const Fr* __restrict__ scale) {
  __shared__ Fr tile[NTT_LDS_N];
  const size_t T = (size_t)1 << logt;
  const size_t tiles_per_vec = n >> logt;
  const size_t tile_id = blockIdx.x;
  const size_t v = tile_id / tiles_per_vec;
  if (v >= (size_t)nvec) return;
  Fr* x = a + v * vstride + (tile_id - v * tiles_per_vec) * T;
  for (size_t i = threadIdx.x; i < T; i += blockDim.x) tile[i] = x[i];
  __syncthreads();
  const size_t nbf = T >> 1;
  for (int s = 0; s < logt; s++) {
    const size_t half = DIF ? (T >> (s + 1)) : ((size_t)1 << s);
    const size_t len = half << 1;
    const size_t twstride = n / len;
    for (size_t t = threadIdx.x; t < nbf; t += blockDim.x) {
      size_t j = t & (half - 1);
      size_t i0 = ((t - j) << 1) + j;
      size_t i1 = i0 + half;
      Fr u = tile[i0], w = tile[i1];
      Fr tws = tw[j * twstride];
      if (DIF) {
        tile[i0] = fp_add(u, w);
        tile[i1] = fp_mul(fp_sub(u, w), tws);
      } else {
        w = fp_mul(w, tws);
        tile[i0] = fp_add(u, w);
        tile[i1] = fp_sub(u, w);
      }
    }
    __syncthreads();
  }
  const size_t base = (tile_id - v * tiles_per_vec) * T;
  if (scale)  // fused coset scale (inverse pass): x[p] *= inc^bitrev(p) / n
    for (size_t i = threadIdx.x; i < T; i += blockDim.x) x[i] = fp_mul(tile[i], scale[base + i]);
  else
    for (size_t i = threadIdx.x; i < T; i += blockDim.x) x[i] = tile[i];
}

// The inverse transform's LDS pass, the coset scale and the forward transform's LDS pass on
// the same tile in one kernel (the tiles coincide: both passes take T consecutive elements), so
// the tile makes one HBM round trip instead of two.  Bit-identical to k_ntt_lds<true> with
// `scale` followed by k_ntt_lds<false>.
__global__ void __launch_bounds__(512) k_ntt_lds_pair(Fr* __restrict__ a, size_t n, int logt,
                                                      const Fr* __restrict__ tw_inv, const Fr* __restrict__ tw_fwd,
                                                      int nvec, size_t vstride, const Fr* __restrict__ scale) {
  ZK_WT(WT_NTT_LDS);
  ZK_LIGHT();
  __shared__ Fr tile[NTT_LDS_N];
  const size_t T = (size_t)1 << logt;
  const size_t tiles_per_vec = n >> logt;
  const size_t tile_id = blockIdx.x;
  const size_t v = tile_id / tiles_per_vec;
  if (v >= (size_t)nvec) return;
  const size_t base = (tile_id - v * tiles_per_vec) * T;
  Fr* x = a + v * vstride + base;
  for (size_t i = threadIdx.x; i < T; i += blockDim.x) tile[i] = x[i];
  __syncthreads();
  const size_t nbf = T >> 1;
  for (int s = 0; s < logt; s++) {  // DIF, spans T/2 .. 1
    const size_t half = T >> (s + 1), twstride = n / (half << 1);
    for (size_t t = threadIdx.x; t < nbf; t += blockDim.x) {
      const size_t j = t & (half - 1), i0 = ((t - j) << 1) + j, i1 = i0 + half;
      const Fr u = tile[i0], w = tile[i1];
      tile[i0] = fp_add(u, w);
      tile[i1] = fp_mul(fp_sub(u, w), tw_inv[j * twstride]);
    }
    __syncthreads();
  }
  for (size_t i = threadIdx.x; i < T; i += blockDim.x) tile[i] = fp_mul(tile[i], scale[base + i]);
  __syncthreads();
  for (int s = 0; s < logt; s++) {  // DIT, spans 1 .. T/2
    const size_t half = (size_t)1 << s, twstride = n / (half << 1);
    for (size_t t = threadIdx.x; t < nbf; t += blockDim.x) {
      const size_t j = t & (half - 1), i0 = ((t - j) << 1) + j, i1 = i0 + half;
      const Fr u = tile[i0], w = fp_mul(tile[i1], tw_fwd[j * twstride]);
      tile[i0] = fp_add(u, w);
      tile[i1] = fp_sub(u, w);
    }
    __syncthreads();
  }
  for (size_t i = threadIdx.x; i < T; i += blockDim.x) x[i] = tile[i];
}

// Same stages, two at a time: each thread takes the 4 elements of a radix-4 butterfly
// (i0, i0 + q, i0 + 2q, i0 + 3q) through two radix-2 stages in registers, so a tile needs half the
// LDS round trips and barriers and each thread has two independent products in flight per stage.
// The products are the radix-2 ones (in a prime field the radix-4 rotation by the 4th root of
// unity is a full product too), so the result is bit-identical to k_ntt_lds.
template <bool DIF>
__global__ void __launch_bounds__(256) k_ntt_lds4(Fr* __restrict__ a, size_t n, int logt, const Fr* __restrict__ tw,
                                                  int nvec, size_t vstride, const Fr* __restrict__ scale) {
  __shared__ Fr tile[NTT_LDS_N];
  const uint32_t T = 1u << logt;
  const size_t tiles_per_vec = n >> logt;
  const size_t tile_id = blockIdx.x;
  const size_t v = tile_id / tiles_per_vec;
  if (v >= (size_t)nvec) return;
  Fr* x = a + v * vstride + (tile_id - v * tiles_per_vec) * T;
  for (uint32_t i = threadIdx.x; i < T; i += blockDim.x) tile[i] = x[i];
  __syncthreads();
  const uint32_t t = threadIdx.x;
  int s = 0;
  for (; s + 1 < logt; s += 2) {
    if (t < (T >> 2)) {
      if (DIF) {  // spans h1 = T >> (s + 1), h2 = h1 / 2
        const uint32_t h2 = T >> (s + 2), h1 = h2 << 1;
        const uint32_t j = t & (h2 - 1), i0 = ((t - j) << 2) + j;
        const size_t st1 = n / (2 * (size_t)h1), st2 = 2 * st1;
        const Fr xa = tile[i0], xb = tile[i0 + h2], xc = tile[i0 + h1], xd = tile[i0 + h1 + h2];
        const Fr a1 = fp_add(xa, xc), c1 = fp_mul(fp_sub(xa, xc), tw[j * st1]);
        const Fr b1 = fp_add(xb, xd), d1 = fp_mul(fp_sub(xb, xd), tw[(j + h2) * st1]);
        const Fr w2 = tw[j * st2];
        tile[i0] = fp_add(a1, b1);
        tile[i0 + h2] = fp_mul(fp_sub(a1, b1), w2);
        tile[i0 + h1] = fp_add(c1, d1);
        tile[i0 + h1 + h2] = fp_mul(fp_sub(c1, d1), w2);
      } else {  // spans h1 = 2^s, h2 = 2 h1
        const uint32_t h1 = 1u << s, h2 = h1 << 1;
        const uint32_t j = t & (h1 - 1), i0 = ((t - j) << 2) + j;
        const size_t st1 = n / (2 * (size_t)h1), st2 = st1 / 2;
        const Fr w1 = tw[j * st1];
        const Fr xa = tile[i0], xb = fp_mul(tile[i0 + h1], w1), xc = tile[i0 + h2], xd = fp_mul(tile[i0 + h2 + h1], w1);
        const Fr a1 = fp_add(xa, xb), b1 = fp_sub(xa, xb), c1 = fp_add(xc, xd), d1 = fp_sub(xc, xd);
        const Fr c2 = fp_mul(c1, tw[j * st2]), d2 = fp_mul(d1, tw[(j + h1) * st2]);
        tile[i0] = fp_add(a1, c2);
        tile[i0 + h2] = fp_sub(a1, c2);
        tile[i0 + h1] = fp_add(b1, d2);
        tile[i0 + h2 + h1] = fp_sub(b1, d2);
      }
    }
    __syncthreads();
  }
  if (s < logt) {  // odd tile exponent: the last radix-2 stage
    const uint32_t half = DIF ? (T >> (s + 1)) : (1u << s);
    const size_t twstride = n / (2 * (size_t)half);
    for (uint32_t q = t; q < (T >> 1); q += blockDim.x) {
      const uint32_t j = q & (half - 1), i0 = ((q - j) << 1) + j, i1 = i0 + half;
      const Fr u = tile[i0], w = tile[i1], tws = tw[j * twstride];
      if (DIF) {
        tile[i0] = fp_add(u, w);
        tile[i1] = fp_mul(fp_sub(u, w), tws);
      } else {
        const Fr wt = fp_mul(w, tws);
        tile[i0] = fp_add(u, wt);
        tile[i1] = fp_sub(u, wt);
      }
    }
    __syncthreads();
  }
  const size_t base = (tile_id - v * tiles_per_vec) * T;
  if (scale)  // fused coset scale (inverse pass): x[p] *= inc^bitrev(p) / n
    for (uint32_t i = threadIdx.x; i < T; i += blockDim.x) x[i] = fp_mul(tile[i], scale[base + i]);
  else
    for (uint32_t i = threadIdx.x; i < T; i += blockDim.x) x[i] = tile[i];
}

// Measured on MI355X (M, 3 x 2^18): NTT stage 0.243/0.245 ms per proof radix-2 vs 0.250/0.250
// radix-4, bench flat (profiles/r02_s4_ab_ntt_radix4.log): the pass is bound by its products, not
// by the LDS round trips or barriers.  Radix-2 stays the default.
#ifndef NTT_RADIX4
#define NTT_RADIX4 0
#endif

// The top k stages (spans n/2 .. n/2^k) of a DIF (or the last k of a DIT) transform only combine
// elements that share their low (logn - k) index bits: a "column" of 2^k elements with stride
// 2^(logn-k).  One workgroup takes NTT_COL_TILE / 2^k consecutive columns (rows of consecutive
// elements are contiguous in memory), runs the k stages in LDS and writes back: one global pass
// instead of k radix-2 passes.
constexpr int NTT_COL_TILE_LOG = 10;
constexpr int NTT_COL_TILE = 1 << NTT_COL_TILE_LOG;
template <bool DIF>
__global__ void __launch_bounds__(256) k_ntt_cols(Fr* __restrict__ a, int logn, int k, const Fr* __restrict__ tw,
                                                  int nvec, size_t vstride) {
  ZK_WT(DIF ? WT_NTT_COLS_INV : WT_NTT_COLS_FWD);
  ZK_LIGHT();
  __shared__ Fr tile[NTT_COL_TILE];
  const size_t n = (size_t)1 << logn;
  const int lowlog = logn - k;                 // column stride 2^lowlog
  const size_t M = (size_t)1 << k;             // elements per column
  const size_t C = (size_t)NTT_COL_TILE >> k;  // columns per workgroup (k <= 11)
  const size_t groups = ((size_t)1 << lowlog) / C;
  const size_t v = blockIdx.x / groups;
  if (v >= (size_t)nvec) return;
  const size_t col0 = (blockIdx.x - v * groups) * C;
  Fr* x = a + v * vstride;
  for (size_t q = threadIdx.x; q < NTT_COL_TILE; q += blockDim.x) {
    const size_t c = q % C, m = q / C;
    tile[q] = x[col0 + c + (m << lowlog)];
  }
  __syncthreads();
  const size_t nbf = NTT_COL_TILE >> 1;
  for (int s = 0; s < k; s++) {
    const size_t mhalf = DIF ? (M >> (s + 1)) : ((size_t)1 << s);  // span in column units
    const size_t half = mhalf << lowlog;                               // span in global units
    const size_t twstride = n / (half << 1);
    for (size_t t = threadIdx.x; t < nbf; t += blockDim.x) {
      const size_t c = t % C, mt = t / C;  // butterfly mt of column c
      const size_t mj = mt & (mhalf - 1);
      const size_t m0 = ((mt - mj) << 1) + mj, m1 = m0 + mhalf;
      const size_t i0 = m0 * C + c, i1 = m1 * C + c;
      const Fr tws = tw[(col0 + c + (mj << lowlog)) * twstride];
      Fr u = tile[i0], w = tile[i1];
      if (DIF) {
        tile[i0] = fp_add(u, w);
        tile[i1] = fp_mul(fp_sub(u, w), tws);
      } else {
        w = fp_mul(w, tws);
        tile[i0] = fp_add(u, w);
        tile[i1] = fp_sub(u, w);
      }
    }
    __syncthreads();
  }
  for (size_t q = threadIdx.x; q < NTT_COL_TILE; q += blockDim.x) {
    const size_t c = q % C, m = q / C;
    x[col0 + c + (m << lowlog)] = tile[q];
  }
}

__global__ void k_ntt_scale(Fr* __restrict__ a, size_t n, const Fr* __restrict__ tab, int nvec,
                            size_t vstride) {
  size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * nvec) return;
  size_t v = t / n;
  size_t p = t - v * n;
  a[v * vstride + p] = fp_mul(a[v * vstride + p], tab[p]);
}


static inline Fr fr_from_limbs(const uint32_t v[8]) {
  Fr r;
  for (int i = 0; i < 8; i++) r.v[i] = v[i];
  return r;
}

__global__ void k_fr_to_mont_one(Fr* out, Fr in) { *out = fp_to_mont(in); }

hipError_t ntt_plan_alloc(NttPlan& pl, int logn, hipStream_t st) {
  pl.logn = logn;
  pl.n = (size_t)1 << logn;
  size_t half = pl.n > 1 ? pl.n / 2 : 1;
  ZK_CHECK(hipMalloc(&pl.tw_fwd, half * sizeof(Fr)));
  ZK_CHECK(hipMalloc(&pl.tw_inv, half * sizeof(Fr)));
  ZK_CHECK(hipMalloc(&pl.coset, pl.n * sizeof(Fr)));
  // roots in Montgomery form (converted on device)
  Fr* tmp;
  ZK_CHECK(hipMalloc(&tmp, 4 * sizeof(Fr)));
  uint32_t inc_std[8];
  for (int i = 0; i < 8; i++) inc_std[i] = (logn == 28) ? FR_SHIFT[i] : FR_ROOT[logn + 1][i];
  hipLaunchKernelGGL(k_fr_to_mont_one, dim3(1), dim3(1), 0, st, tmp + 0, fr_from_limbs(FR_ROOT[logn]));
  hipLaunchKernelGGL(k_fr_to_mont_one, dim3(1), dim3(1), 0, st, tmp + 1, fr_from_limbs(FR_ROOT_INV[logn]));
  hipLaunchKernelGGL(k_fr_to_mont_one, dim3(1), dim3(1), 0, st, tmp + 2, fr_from_limbs(inc_std));
  hipLaunchKernelGGL(k_fr_to_mont_one, dim3(1), dim3(1), 0, st, tmp + 3, fr_from_limbs(FR_INV_2K[logn]));
  Fr h[4];
  ZK_CHECK(hipMemcpyAsync(h, tmp, sizeof(h), hipMemcpyDeviceToHost, st));
  ZK_CHECK(hipStreamSynchronize(st));
  ZK_CHECK(hipFree(tmp));
  hipLaunchKernelGGL(k_ntt_twiddles, dim3(zk_grid(half, 256)), dim3(256), 0, st, pl.tw_fwd, half, h[0]);
  hipLaunchKernelGGL(k_ntt_twiddles, dim3(zk_grid(half, 256)), dim3(256), 0, st, pl.tw_inv, half, h[1]);
  hipLaunchKernelGGL(k_ntt_coset_table, dim3(zk_grid(pl.n, 256)), dim3(256), 0, st, pl.coset, pl.n,
                     logn, h[2], h[3]);
  return hipGetLastError();
}

void ntt_plan_free(NttPlan& pl) {
  if (pl.tw_fwd) (void)hipFree(pl.tw_fwd);
  if (pl.tw_inv) (void)hipFree(pl.tw_inv);
  if (pl.coset) (void)hipFree(pl.coset);
  pl = NttPlan();
}

// DIF pass of the inverse transform (natural -> bit-reversed), 1/n and the coset scale fused
// into the last (LDS) pass when `scale` is given.  The stages above the LDS tile run as one
// column pass (logn <= 21) or as radix-2 global passes (larger domains).
static hipError_t ntt_dif(const NttPlan& pl, Fr* d, const Fr* tw, int nvec, size_t vstride, const Fr* scale,
                          hipStream_t st) {
  const size_t n = pl.n;
  const int logt = pl.logn < NTT_LDS_LOG ? pl.logn : NTT_LDS_LOG;
  const int top = pl.logn - logt;
  const int kcol = top <= NTT_COL_TILE_LOG ? top : 0;  // one column pass, or radix-2 passes (logn > 21)
  const size_t nb = (n >> 1) * nvec;
  for (int s = 0; s < top - kcol; s++) {
    size_t half = n >> (s + 1);
    hipLaunchKernelGGL(k_ntt_dif_stage, dim3(zk_grid(nb, 256)), dim3(256), 0, st, d, n, half, tw, n / (2 * half),
                       nvec, vstride);
  }
  if (kcol > 0) {
    const unsigned groups = (unsigned)((((size_t)1 << (pl.logn - kcol)) / ((size_t)NTT_COL_TILE >> kcol)) * nvec);
    hipLaunchKernelGGL(k_ntt_cols<true>, dim3(groups), dim3(256), 0, st, d, pl.logn, kcol, tw, nvec, vstride);
  }
  if (logt > 0 && NTT_RADIX4)
    hipLaunchKernelGGL(k_ntt_lds4<true>, dim3((unsigned)((n >> logt) * nvec)), dim3(256), 0, st, d, n, logt, tw,
                       nvec, vstride, scale);
  else if (logt > 0)
    hipLaunchKernelGGL(k_ntt_lds<true>, dim3((unsigned)((n >> logt) * nvec)), dim3(512), 0, st, d, n, logt, tw,
                       nvec, vstride, scale);
  else if (scale)
    hipLaunchKernelGGL(k_ntt_scale, dim3(zk_grid(pl.n * nvec, 256)), dim3(256), 0, st, d, pl.n, scale, nvec, vstride);
  return hipGetLastError();
}

// DIT pass (bit-reversed -> natural).
static hipError_t ntt_dit(const NttPlan& pl, Fr* d, const Fr* tw, int nvec, size_t vstride, hipStream_t st) {
  const size_t n = pl.n;
  const int logt = pl.logn < NTT_LDS_LOG ? pl.logn : NTT_LDS_LOG;
  const int top = pl.logn - logt;
  const int kcol = top <= NTT_COL_TILE_LOG ? top : 0;
  const size_t nb = (n >> 1) * nvec;
  if (logt > 0 && NTT_RADIX4)
    hipLaunchKernelGGL(k_ntt_lds4<false>, dim3((unsigned)((n >> logt) * nvec)), dim3(256), 0, st, d, n, logt, tw,
                       nvec, vstride, (const Fr*)nullptr);
  else if (logt > 0)
    hipLaunchKernelGGL(k_ntt_lds<false>, dim3((unsigned)((n >> logt) * nvec)), dim3(512), 0, st, d, n, logt, tw,
                       nvec, vstride, (const Fr*)nullptr);
  if (kcol > 0) {
    const unsigned groups = (unsigned)((((size_t)1 << (pl.logn - kcol)) / ((size_t)NTT_COL_TILE >> kcol)) * nvec);
    hipLaunchKernelGGL(k_ntt_cols<false>, dim3(groups), dim3(256), 0, st, d, pl.logn, kcol, tw, nvec, vstride);
  }
  for (int s = logt + kcol; s < pl.logn; s++) {
    size_t half = (size_t)1 << s;
    hipLaunchKernelGGL(k_ntt_dit_stage, dim3(zk_grid(nb, 256)), dim3(256), 0, st, d, n, half, tw, n / (2 * half),
                       nvec, vstride);
  }
  return hipGetLastError();
}

// In place: nvec vectors (stride vstride) of evaluations on the domain -> evaluations on
// the odd coset (snarkjs ifft + batchApplyKey + fft).
#ifndef NTT_LDS_PAIR
#define NTT_LDS_PAIR 1
#endif
hipError_t ntt_coset_shift(const NttPlan& pl, Fr* d, int nvec, size_t vstride, hipStream_t st) {
  const int logt = pl.logn < NTT_LDS_LOG ? pl.logn : NTT_LDS_LOG;
  const int top = pl.logn - logt;
  if (!NTT_LDS_PAIR || NTT_RADIX4 || logt == 0 || top == 0 || top > NTT_COL_TILE_LOG) {
    ZK_CHECK(ntt_dif(pl, d, pl.tw_inv, nvec, vstride, pl.coset, st));
    return ntt_dit(pl, d, pl.tw_fwd, nvec, vstride, st);
  }
  // column pass (inverse, top stages) -> fused LDS pair -> column pass (forward, top stages)
  const unsigned groups = (unsigned)((((size_t)1 << (pl.logn - top)) / ((size_t)NTT_COL_TILE >> top)) * nvec);
  hipLaunchKernelGGL(k_ntt_cols<true>, dim3(groups), dim3(256), 0, st, d, pl.logn, top, pl.tw_inv, nvec, vstride);
  hipLaunchKernelGGL(k_ntt_lds_pair, dim3((unsigned)((pl.n >> logt) * nvec)), dim3(512), 0, st, d, pl.n, logt,
                     pl.tw_inv, pl.tw_fwd, nvec, vstride, pl.coset);
  hipLaunchKernelGGL(k_ntt_cols<false>, dim3(groups), dim3(256), 0, st, d, pl.logn, top, pl.tw_fwd, nvec, vstride);
  return hipGetLastError();
}

// Plain transforms (natural order in and out) for parity tests: inverse includes 1/n.
__global__ void k_bitrev_copy(const Fr* __restrict__ in, Fr* __restrict__ out, size_t n, int logn) {
  size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  size_t q = logn ? (__brevll((unsigned long long)p) >> (64 - logn)) : 0;
  out[q] = in[p];
}

hipError_t zk_wtrace_bind_ntt(const WtBuf& b) { return zk_wtrace_bind_tu(b); }

}  // namespace zkfl
