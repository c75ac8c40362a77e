// Setup-side group primitives (see setup.h for the snarkjs commands they serve).
//
// One lane per scalar multiplication, left-to-right double-and-add over XYZZ coordinates with
// the affine base added by madd-2008-s.  These run once per ceremony step, so the kernels are
// plain and general (any scalar, infinity anywhere) rather than tuned: a pot17 `prepare phase2`
// is ~20 M G1-equivalent scalar multiplications, ~1 s on one MI355X.
#include "setup.h"

#include <vector>

#include "common.h"
#include "curve.h"
#include "fr_consts.h"
#include "ntt.h"

namespace zkfl {
namespace {

// k * P for a standard-form scalar (8 little-endian u32 limbs): curve.h's double-and-add, the
// routine the dev ceremony's k_gen_mul has always used (its limb loop unrolled, so the scalar
// stays in registers)
template <class F>
ZK_DEV XYZZ<F> smul_aff(const Affine<F>& a, const uint32_t k[8]) {
  return xyzz_scalar_mul<F>(xyzz_from_affine<F>(a), k);
}

template <class F>
ZK_DEV XYZZ<F> smul_xyzz(const XYZZ<F>& p, const uint32_t k[8]) {
  return xyzz_scalar_mul<F>(p, k);
}

template <class F>
__global__ void __launch_bounds__(64) k_scale(const Affine<F>* __restrict__ pts, const uint32_t* __restrict__ sc,
                                              size_t n, Affine<F>* __restrict__ out) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t k[8];
  for (int j = 0; j < 8; j++) k[j] = sc[8 * i + j];
  out[i] = xyzz_to_affine<F>(smul_aff<F>(pts[i], k));
}

// One chunk of consecutive terms of one row per lane: MUL = sum of coef_t * bases[idx_t]
// (level 0), else the sum of the previous level's partial sums.
template <class F, bool MUL>
__global__ void __launch_bounds__(64) k_lc_chunks(const Affine<F>* __restrict__ bases, const uint32_t* __restrict__ idx,
                                                  const uint32_t* __restrict__ coefs, const XYZZ<F>* __restrict__ items,
                                                  const uint32_t* __restrict__ cs, size_t nchunks,
                                                  XYZZ<F>* __restrict__ part) {
  size_t c = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nchunks) return;
  const uint32_t t0 = cs[c], t1 = cs[c + 1];
  XYZZ<F> acc = xyzz_inf<F>();
  for (uint32_t t = t0; t < t1; t++) {
    if (MUL) {
      uint32_t k[8];
      for (int j = 0; j < 8; j++) k[j] = coefs[8 * (size_t)t + j];
      acc = xyzz_add<F>(acc, smul_aff<F>(bases[idx[t]], k));
    } else {
      acc = xyzz_add<F>(acc, items[t]);
    }
  }
  part[c] = acc;
}

// rows with one partial sum left -> affine; empty rows -> infinity (all-zero bytes)
template <class F>
__global__ void __launch_bounds__(64) k_lc_out(const XYZZ<F>* __restrict__ items, const uint32_t* __restrict__ rp,
                                               size_t n_out, Affine<F>* __restrict__ out) {
  size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_out) return;
  out[r] = rp[r + 1] > rp[r] ? xyzz_to_affine<F>(items[rp[r]]) : xyzz_to_affine<F>(xyzz_inf<F>());
}

template <class F>
__global__ void __launch_bounds__(64) k_to_xyzz(const Affine<F>* __restrict__ in, size_t n, XYZZ<F>* __restrict__ x) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  x[i] = xyzz_from_affine<F>(in[i]);
}

// One decimation-in-frequency stage over the group: (a, c) -> (a + c, w^k (a - c)), natural
// order in, bit-reversed out after the last stage.  tw = the inverse root powers (Montgomery Fr).
template <class F>
__global__ void __launch_bounds__(64) k_gfft_dif(XYZZ<F>* __restrict__ x, size_t n, size_t span,
                                                 const Fr* __restrict__ tw, size_t tstride) {
  size_t b = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n / 2) return;
  const size_t blk = b / span, k = b - blk * span;
  const size_t i = blk * 2 * span + k, j = i + span;
  const XYZZ<F> a = x[i], c = x[j];
  x[i] = xyzz_add<F>(a, c);
  XYZZ<F> d = xyzz_add<F>(a, xyzz_neg<F>(c));
  if (k) {
    const Fr w = fp_from_mont(tw[k * tstride]);
    d = smul_xyzz<F>(d, w.v);
  }
  x[j] = d;
}

// out[j] = (1/n) * x[bitrev(j)], affine
template <class F>
__global__ void __launch_bounds__(64) k_gfft_out(const XYZZ<F>* __restrict__ x, size_t n, int logn, Fr ninv,
                                                 Affine<F>* __restrict__ out) {
  size_t j = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const size_t src = logn ? (size_t)(__brevll((unsigned long long)j) >> (64 - logn)) : 0;
  out[j] = xyzz_to_affine<F>(smul_xyzz<F>(x[src], ninv.v));
}

struct DevBufs {
  std::vector<void*> p;
  template <class T>
  hipError_t alloc(T** out, size_t bytes) {
    void* q = nullptr;
    hipError_t e = hipMalloc(&q, bytes ? bytes : 1);
    if (e == hipSuccess) p.push_back(q);
    *out = static_cast<T*>(q);
    return e;
  }
  ~DevBufs() {
    for (void* q : p) (void)hipFree(q);
  }
};

template <class F>
hipError_t scale_t(hipStream_t st, const uint8_t* points, const uint8_t* scalars, size_t n, uint8_t* out) {
  if (n == 0) return hipSuccess;
  DevBufs b;
  Affine<F>*d_p, *d_o;
  uint32_t* d_s;
  ZK_CHECK(b.alloc(&d_p, n * sizeof(Affine<F>)));
  ZK_CHECK(b.alloc(&d_o, n * sizeof(Affine<F>)));
  ZK_CHECK(b.alloc(&d_s, n * 32));
  ZK_CHECK(hipMemcpyAsync(d_p, points, n * sizeof(Affine<F>), hipMemcpyHostToDevice, st));
  ZK_CHECK(hipMemcpyAsync(d_s, scalars, n * 32, hipMemcpyHostToDevice, st));
  hipLaunchKernelGGL(k_scale<F>, dim3(zk_grid(n, 64)), dim3(64), 0, st, d_p, d_s, n, d_o);
  ZK_CHECK(hipGetLastError());
  ZK_CHECK(hipMemcpyAsync(out, d_o, n * sizeof(Affine<F>), hipMemcpyDeviceToHost, st));
  return hipStreamSynchronize(st);
}

template <class F>
hipError_t lagrange_t(hipStream_t st, const uint8_t* points, int logn, uint8_t* out) {
  const size_t n = (size_t)1 << logn;
  DevBufs b;
  Affine<F>* d_a;
  XYZZ<F>* d_x;
  ZK_CHECK(b.alloc(&d_a, n * sizeof(Affine<F>)));
  ZK_CHECK(b.alloc(&d_x, n * sizeof(XYZZ<F>)));
  NttPlan pl;
  ZK_CHECK(ntt_plan_alloc(pl, logn, st));  // tw_inv[m] = w^-m, m < n/2
  hipError_t e = hipMemcpyAsync(d_a, points, n * sizeof(Affine<F>), hipMemcpyHostToDevice, st);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_to_xyzz<F>, dim3(zk_grid(n, 64)), dim3(64), 0, st, d_a, n, d_x);
    for (int s = logn - 1; s >= 0; s--) {
      const size_t span = (size_t)1 << s;
      hipLaunchKernelGGL(k_gfft_dif<F>, dim3(zk_grid(n / 2, 64)), dim3(64), 0, st, d_x, n, span, pl.tw_inv,
                         n / (2 * span));
    }
    Fr ninv;
    for (int i = 0; i < 8; i++) ninv.v[i] = FR_INV_2K[logn][i];
    hipLaunchKernelGGL(k_gfft_out<F>, dim3(zk_grid(n, 64)), dim3(64), 0, st, d_x, n, logn, ninv, d_a);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(out, d_a, n * sizeof(Affine<F>), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  ntt_plan_free(pl);
  return e;
}

constexpr uint32_t LC_L0 = 8;   // terms per lane at level 0 (scalar multiplications)
constexpr uint32_t LC_L = 16;   // partial sums per lane at the later levels

// chunk boundaries of a level: every non-empty row split into pieces of <= L items;
// crp[r] = index of row r's first chunk.  Returns the largest chunk count of any row.
size_t make_chunks(const std::vector<uint64_t>& rp, uint32_t L, std::vector<uint32_t>& cs, std::vector<uint32_t>& crp) {
  const size_t n_out = rp.size() - 1;
  cs.clear();
  crp.assign(n_out + 1, 0);
  size_t most = 0;
  for (size_t r = 0; r < n_out; r++) {
    crp[r] = (uint32_t)cs.size();
    size_t cnt = 0;
    for (uint64_t t = rp[r]; t < rp[r + 1]; t += L, cnt++) cs.push_back((uint32_t)t);
    most = cnt > most ? cnt : most;
  }
  crp[n_out] = (uint32_t)cs.size();
  cs.push_back((uint32_t)rp[n_out]);
  return most;
}

template <class F>
hipError_t lincomb_t(hipStream_t st, const uint8_t* bases, size_t n_bases, size_t n_out, const uint64_t* rowptr,
                     const uint32_t* idx, const uint8_t* coefs, uint8_t* out) {
  if (n_out == 0) return hipSuccess;
  const size_t nnz = rowptr[n_out];
  DevBufs b;
  Affine<F>*d_b, *d_o;
  uint32_t *d_i, *d_c;
  ZK_CHECK(b.alloc(&d_b, n_bases * sizeof(Affine<F>)));
  ZK_CHECK(b.alloc(&d_o, n_out * sizeof(Affine<F>)));
  ZK_CHECK(b.alloc(&d_i, nnz * 4));
  ZK_CHECK(b.alloc(&d_c, nnz * 32));
  if (n_bases) ZK_CHECK(hipMemcpyAsync(d_b, bases, n_bases * sizeof(Affine<F>), hipMemcpyHostToDevice, st));
  if (nnz) {
    ZK_CHECK(hipMemcpyAsync(d_i, idx, nnz * 4, hipMemcpyHostToDevice, st));
    ZK_CHECK(hipMemcpyAsync(d_c, coefs, nnz * 32, hipMemcpyHostToDevice, st));
  }
  std::vector<uint64_t> rp(rowptr, rowptr + n_out + 1);
  std::vector<uint32_t> cs, crp;
  XYZZ<F>* items = nullptr;  // the previous level's partial sums
  bool first = true;
  for (;;) {
    const size_t most = make_chunks(rp, first ? LC_L0 : LC_L, cs, crp);
    const size_t nch = cs.size() - 1;
    uint32_t *d_cs, *d_crp;
    XYZZ<F>* part;
    ZK_CHECK(b.alloc(&d_cs, cs.size() * 4));
    ZK_CHECK(b.alloc(&d_crp, crp.size() * 4));
    ZK_CHECK(b.alloc(&part, nch * sizeof(XYZZ<F>)));
    ZK_CHECK(hipMemcpyAsync(d_cs, cs.data(), cs.size() * 4, hipMemcpyHostToDevice, st));
    ZK_CHECK(hipMemcpyAsync(d_crp, crp.data(), crp.size() * 4, hipMemcpyHostToDevice, st));
    if (nch) {
      if (first)
        hipLaunchKernelGGL((k_lc_chunks<F, true>), dim3(zk_grid(nch, 64)), dim3(64), 0, st, d_b, d_i, d_c, items, d_cs,
                           nch, part);
      else
        hipLaunchKernelGGL((k_lc_chunks<F, false>), dim3(zk_grid(nch, 64)), dim3(64), 0, st, d_b, d_i, d_c, items,
                           d_cs, nch, part);
      ZK_CHECK(hipGetLastError());
    }
    // host copies of cs / crp must outlive the async uploads
    ZK_CHECK(hipStreamSynchronize(st));
    items = part;
    first = false;
    if (most <= 1) {
      hipLaunchKernelGGL(k_lc_out<F>, dim3(zk_grid(n_out, 64)), dim3(64), 0, st, items, d_crp, n_out, d_o);
      ZK_CHECK(hipGetLastError());
      break;
    }
    for (size_t r = 0; r <= n_out; r++) rp[r] = crp[r];
  }
  ZK_CHECK(hipMemcpyAsync(out, d_o, n_out * sizeof(Affine<F>), hipMemcpyDeviceToHost, st));
  return hipStreamSynchronize(st);
}

}  // namespace

hipError_t setup_scale(bool g2, hipStream_t st, const uint8_t* points, const uint8_t* scalars, size_t n,
                       uint8_t* out) {
  return g2 ? scale_t<Fq2Ops>(st, points, scalars, n, out) : scale_t<FqOps>(st, points, scalars, n, out);
}

hipError_t setup_lagrange(bool g2, hipStream_t st, const uint8_t* points, int logn, uint8_t* out) {
  return g2 ? lagrange_t<Fq2Ops>(st, points, logn, out) : lagrange_t<FqOps>(st, points, logn, out);
}

hipError_t setup_lincomb(bool g2, hipStream_t st, const uint8_t* bases, size_t n_bases, size_t n_out,
                         const uint64_t* rowptr, const uint32_t* idx, const uint8_t* coefs, uint8_t* out) {
  return g2 ? lincomb_t<Fq2Ops>(st, bases, n_bases, n_out, rowptr, idx, coefs, out)
            : lincomb_t<FqOps>(st, bases, n_bases, n_out, rowptr, idx, coefs, out);
}

}  // namespace zkfl
