// Batch-affine rounds in front of the G1 bucket accumulation (MSM_G1_AFFINE, the default).
//
// Why: the G1 accumulation is VALU-bound (86% of SIMD cycles busy, profiles/r03_sq_counters.txt)
// on the XYZZ mixed addition, 10 Montgomery products per sorted entry.  An affine addition is 3
// products once its inverse (x1 - x0)^-1 is known, and Montgomery's trick shares ONE inversion among
// all additions of a round: 3 more products per addition (exclusive prefix product, then two on the
// way back).  So each round pairs neighbouring entries of the same bucket and replaces two XYZZ
// additions by one affine addition (6 products) + one XYZZ addition of the sum.
//
// Layout: lane c owns the sorted entries [c L, c L + L) (L = MSM_G1_L = 32), as the XYZZ kernel
// did; a round pairs items (2j, 2j + 1) of the lane's item list when they are in the same bucket,
// both finite and x1 != x0 (else both stay items).  Two rounds, then the lane adds its remaining
// items (~L / 4) into XYZZ accumulators with the same run / stitching-item logic as
// k_msm_accumulate, so the tails (msm.h) are unchanged.
//
// The inversion of a round is shared by the whole MSM through a product tree:
//   prep   (per lane) exclusive prefix products of its d_j = x1 - x0, lane product -> leaf of its
//          workgroup's heap (256 leaves, 511 nodes, stored to `tree`), workgroup product -> wgprod
//   root   (one workgroup) product of the workgroup products (4 per thread serially, then a heap
//          over 1024 threads in LDS), ONE inversion (thread 0, binary extended Euclid), inverses back down -> wginv
//   apply  (per lane) the workgroup heap from `tree`, inverses down to the leaves, then the lane
//          walks its pairs backwards: inv_j = inv_run * prefix_j, inv_run *= d_j, affine sum.
// Items refer to a base (index | sign << 31) or to a sum of the previous round (AFF_PT | slot).
#pragma once
#include "field29.h"
#include "msm_api.h"

namespace zkfl {

// root inversion: 1 binary extended Euclid (f29_inv_bgcd), 0 Fermat (f29_inv: 316 dependent products)
#ifndef MSM_AFF_INV_BGCD
#define MSM_AFF_INV_BGCD 1
#endif
constexpr int AFF_WG = 256;                 // lanes per workgroup (heap leaves)
constexpr int AFF_L = MSM_L;                // sorted entries per lane
constexpr int AFF_P = AFF_L / 2;            // pairs per lane and round (<= items / 2)
constexpr int AFF_ROOT_T = 1024;            // threads of the root workgroup
constexpr int AFF_ROOT_K = 4;               // workgroup products per root thread
constexpr uint32_t AFF_PT = 0x40000000u;    // item ref: a sum of the previous round (slot in the low bits)
constexpr uint32_t AFF_SIGN = 0x80000000u;  // item ref: negated base
static_assert(AFF_L <= 64 && AFF_L % 2 == 0, "affine rounds: item lists of <= 64 entries per lane");

ZK_DEV void aff_st(uint32_t* p, size_t stride, const F29& v) {
#pragma unroll
  for (int i = 0; i < 9; i++) p[i * stride] = v.v[i];
}
ZK_DEV F29 aff_ld(const uint32_t* p, size_t stride) {
  F29 v;
#pragma unroll
  for (int i = 0; i < 9; i++) v.v[i] = p[i * stride];
  return v;
}

// The point an item refers to (canonical coordinates, the base's sign applied) and whether it is
// infinity (a base stored as (0, 0)).
ZK_DEV Affine<FqOps29> aff_item(uint32_t ref, const Affine<FqOps>* __restrict__ bases,
                                const Affine<FqOps>* __restrict__ prev, size_t lanes, size_t c, bool& inf) {
  if (ref & AFF_PT) {
    inf = false;
    return MsmIO<FqOps29>::ld_aff(prev, (size_t)(ref & 0xFFFFu) * lanes + c);
  }
  Affine<FqOps29> a = MsmIO<FqOps29>::ld_aff(bases, ref & 0x3FFFFFFFu);
  uint32_t z = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) z |= a.x.v[i] | a.y.v[i];
  inf = z == 0;
  if ((ref & AFF_SIGN) && !inf) {  // p - y: y != 0 on the prime-order curve, so canonical
    a.y = f29_ksub(P29::K1_1, f29_zero(), a.y);
    f29_norm(a.y);
  }
  return a;
}

// Heap product over the workgroup's leaves h[256..511] (LDS, F29): h[i] = h[2i] h[2i+1], active
// threads contiguous per level (so mostly whole waves are idle, not partial ones).
ZK_DEV void aff_heap_up(F29* h, int t) {
#pragma unroll 1
  for (int lvl = AFF_WG / 2; lvl >= 1; lvl >>= 1) {
    if (t < lvl) h[lvl + t] = f29_mul(h[2 * (lvl + t)], h[2 * (lvl + t) + 1]);
    __syncthreads();
  }
}
// Inverses down the heap in place: on entry h[1] = 1 / root, every other node its product; on
// exit h[256 + t] = 1 / leaf t.
ZK_DEV void aff_heap_down(F29* h, int t) {
#pragma unroll 1
  for (int lvl = 1; lvl < AFF_WG; lvl <<= 1) {
    if (t < lvl) {
      const int i = lvl + t;
      const F29 inv = h[i], l = h[2 * i], r = h[2 * i + 1];
      h[2 * i] = f29_mul(inv, r);
      h[2 * i + 1] = f29_mul(inv, l);
    }
    __syncthreads();
  }
}

// The lane's product -> its workgroup heap: up-sweep, heap stored to `tree`, root to wgprod.
ZK_DEV void aff_lane_product_out(F29* h, int t, const F29& pr, uint32_t* __restrict__ tree,
                                 uint32_t* __restrict__ wgprod) {
  h[AFF_WG + t] = pr;
  __syncthreads();
  aff_heap_up(h, t);
  uint32_t* tw = tree + (size_t)blockIdx.x * 512 * 9;
  for (int i = t; i < 2 * AFF_WG; i += AFF_WG) aff_st(tw + (size_t)i * 9, 1, h[i]);
  if (t == 0) aff_st(wgprod + (size_t)blockIdx.x * 9, 1, h[1]);
}

// Inverse of this lane's product of the previous prep (heap from `tree`, root inverse from wginv).
ZK_DEV F29 aff_lane_inverse(F29* h, int t, const uint32_t* __restrict__ tree, const uint32_t* __restrict__ wginv) {
  const uint32_t* tw = tree + (size_t)blockIdx.x * 512 * 9;
  for (int i = t; i < 2 * AFF_WG; i += AFF_WG) h[i] = aff_ld(tw + (size_t)i * 9, 1);
  __syncthreads();
  if (t == 0) h[1] = aff_ld(wginv + (size_t)blockIdx.x * 9, 1);
  __syncthreads();
  aff_heap_down(h, t);
  const F29 r = h[AFF_WG + t];
  __syncthreads();  // h is reused by the caller
  return r;
}

// Round-1 pair decision and difference for entries a, b (positions in the sorted array).
ZK_DEV bool aff_pair1(const uint16_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                      const Affine<FqOps>* __restrict__ bases, uint32_t a, uint32_t p1, Affine<FqOps29>& A,
                      Affine<FqOps29>& B, F29& d) {
  if (a + 1 >= p1 || keys[a] != keys[a + 1]) return false;
  bool ia, ib;
  A = aff_item(vals[a], bases, nullptr, 0, 0, ia);
  B = aff_item(vals[a + 1], bases, nullptr, 0, 0, ib);
  if (ia || ib) return false;
  d = f29_sub_canon(B.x, A.x);
  return !f29_is_zero(d);
}

// Round 1 prep: exclusive prefix products of the lane's pair differences.
static __global__ void __launch_bounds__(AFF_WG) k_aff_prep1(const uint16_t* __restrict__ keys,
                                                             const uint32_t* __restrict__ vals,
                                                             const Affine<FqOps>* __restrict__ bases,
                                                             const uint32_t* __restrict__ nnz_ptr, MsmAffScratch s) {
  __shared__ F29 h[2 * AFF_WG];
  const int t = threadIdx.x;
  const size_t c = (size_t)blockIdx.x * AFF_WG + t;
  const uint32_t nnz = *nnz_ptr;
  const size_t p0 = c * AFF_L;
  F29 pr = f29_const(P29::ONE);
  if (p0 < nnz) {
    const uint32_t p1 = (uint32_t)(p0 + AFF_L < nnz ? p0 + AFF_L : nnz);
    for (int j = 0; j < AFF_P; j++) {
      Affine<FqOps29> A, B;
      F29 d;
      if (aff_pair1(keys, vals, bases, (uint32_t)p0 + 2 * j, p1, A, B, d)) {
        aff_st(s.pref + (size_t)j * 9 * s.lanes + c, s.lanes, pr);
        pr = f29_mul(pr, d);
      }
    }
  }
  aff_lane_product_out(h, t, pr, s.tree, s.wgprod);
}

// One workgroup: the MSM's single inversion of a round.
static __global__ void __launch_bounds__(AFF_ROOT_T) k_aff_root(MsmAffScratch s, uint32_t nwg) {
  __shared__ F29 h[2 * AFF_ROOT_T];
  const int t = threadIdx.x;
  F29 ex[AFF_ROOT_K];  // exclusive prefixes of this thread's workgroup products
  F29 pr = f29_const(P29::ONE);
#pragma unroll
  for (int k = 0; k < AFF_ROOT_K; k++) {
    const uint32_t w = (uint32_t)t * AFF_ROOT_K + k;
    ex[k] = pr;
    if (w < nwg) pr = f29_mul(pr, aff_ld(s.wgprod + (size_t)w * 9, 1));
  }
  h[AFF_ROOT_T + t] = pr;
  __syncthreads();
#pragma unroll 1
  for (int lvl = AFF_ROOT_T / 2; lvl >= 1; lvl >>= 1) {
    if (t < lvl) h[lvl + t] = f29_mul(h[2 * (lvl + t)], h[2 * (lvl + t) + 1]);
    __syncthreads();
  }
  if (t == 0) h[1] = MSM_AFF_INV_BGCD ? f29_inv_bgcd(h[1]) : f29_inv(h[1]);
  __syncthreads();
#pragma unroll 1
  for (int lvl = 1; lvl < AFF_ROOT_T; lvl <<= 1) {
    if (t < lvl) {
      const int i = lvl + t;
      const F29 inv = h[i], l = h[2 * i], r = h[2 * i + 1];
      h[2 * i] = f29_mul(inv, r);
      h[2 * i + 1] = f29_mul(inv, l);
    }
    __syncthreads();
  }
  F29 inv = h[AFF_ROOT_T + t];  // 1 / (this thread's product)
#pragma unroll
  for (int k = AFF_ROOT_K - 1; k >= 0; k--) {
    const uint32_t w = (uint32_t)t * AFF_ROOT_K + k;
    if (w < nwg) {
      aff_st(s.wginv + (size_t)w * 9, 1, f29_mul(inv, ex[k]));
      inv = f29_mul(inv, aff_ld(s.wgprod + (size_t)w * 9, 1));
    }
  }
}

// Round 1 apply + round 2 prep.  The lane walks its round-1 pairs backwards (descending
// positions: inv is 1 / (d_0 .. d_j) of the paired j), so its items come out in descending
// position order: a round-1 sum (stored to pts[0], kept in registers) or the unpaired entries.
// Round-2 pairs are consecutive items of THAT emission order (e_2i, e_2i+1), decided on the fly
// from registers; their exclusive prefix products go to pref, the pairing bits to mask2.  The
// item list (emission order) goes to key1 / ref1 / cnt1.
static __global__ void __launch_bounds__(AFF_WG) k_aff_apply1(const uint16_t* __restrict__ keys,
                                                              const uint32_t* __restrict__ vals,
                                                              const Affine<FqOps>* __restrict__ bases,
                                                              const uint32_t* __restrict__ nnz_ptr, MsmAffScratch s) {
  __shared__ F29 h[2 * AFF_WG];
  const int t = threadIdx.x;
  const size_t c = (size_t)blockIdx.x * AFF_WG + t;
  const uint32_t nnz = *nnz_ptr;
  const size_t p0 = c * AFF_L;
  F29 inv = aff_lane_inverse(h, t, s.tree, s.wginv);
  F29 pr = f29_const(P29::ONE);
  if (p0 < nnz) {
    const uint32_t p1 = (uint32_t)(p0 + AFF_L < nnz ? p0 + AFF_L : nnz);
    Affine<FqOps>* __restrict__ out = s.pts[0];
    uint32_t n1 = 0, mask2 = 0;
    uint16_t pkey = 0;
    bool pok = false;
    F29 px = f29_zero();
    auto emit = [&](uint16_t key, uint32_t ref, const F29& x, bool ok) {
      s.key1[(size_t)n1 * s.lanes + c] = key;
      s.ref1[(size_t)n1 * s.lanes + c] = ref;
      if ((n1 & 1) == 0) {  // first of a round-2 pair
        pkey = key;
        px = x;
        pok = ok;
      } else if (key == pkey && ok && pok) {
        const F29 d = f29_sub_canon(x, px);
        if (!f29_is_zero(d)) {
          aff_st(s.pref + (size_t)(AFF_P + (n1 >> 1)) * 9 * s.lanes + c, s.lanes, pr);  // round-2 half
          pr = f29_mul(pr, d);
          mask2 |= 1u << (n1 >> 1);
        }
      }
      n1++;
    };
    for (int j = AFF_P - 1; j >= 0; j--) {
      const uint32_t a = (uint32_t)p0 + 2 * j;
      if (a >= p1) continue;
      const bool has_b = a + 1 < p1;
      bool ia, ib = true;
      const Affine<FqOps29> A = aff_item(vals[a], bases, nullptr, 0, 0, ia);
      Affine<FqOps29> B = A;
      if (has_b) B = aff_item(vals[a + 1], bases, nullptr, 0, 0, ib);
      bool paired = false;
      F29 d;
      if (has_b && !ia && !ib && keys[a] == keys[a + 1]) {
        d = f29_sub_canon(B.x, A.x);
        paired = !f29_is_zero(d);
      }
      if (paired) {
        const F29 ij = f29_mul(inv, aff_ld(s.pref + (size_t)j * 9 * s.lanes + c, s.lanes));
        inv = f29_mul(inv, d);
        const Affine<FqOps29> S = f29_affine_add(A, B, ij);
        Affine<FqOps> o;
        f29_unpack(o.x.v, S.x);
        f29_unpack(o.y.v, S.y);
        out[(size_t)j * s.lanes + c] = o;
        emit(keys[a], AFF_PT | (uint32_t)j, S.x, true);
      } else {
        if (has_b) emit(keys[a + 1], vals[a + 1], B.x, !ib);
        emit(keys[a], vals[a], A.x, !ia);
      }
    }
    s.cnt1[c] = (uint8_t)n1;
    s.mask2[c] = mask2;
  }
  aff_lane_product_out(h, t, pr, s.tree, s.wgprod);
}

// Round 2 apply + the XYZZ accumulation of what is left (k_msm_accumulate's run logic).  The
// item list is walked backwards = ascending positions, which is also the back-substitution
// order of the round-2 prefixes, so every round-2 sum goes straight into the accumulator.
template <int MINW>
__global__ void __launch_bounds__(AFF_WG) __attribute__((amdgpu_waves_per_eu(MINW))) k_aff_apply2_acc(
    const uint16_t* __restrict__ keys, const Affine<FqOps>* __restrict__ bases, const uint32_t* __restrict__ nnz_ptr,
    MsmAffScratch s, uint32_t* __restrict__ item_key, XYZZ<FqOps>* __restrict__ item_val,
    XYZZ<FqOps>* __restrict__ buckets) {
  using F = FqOps29;
  __shared__ F29 h[2 * AFF_WG];
  const int t = threadIdx.x;
  const size_t c = (size_t)blockIdx.x * AFF_WG + t;
  const uint32_t nnz = *nnz_ptr;
  const size_t p0 = c * AFF_L;
  F29 inv = aff_lane_inverse(h, t, s.tree, s.wginv);
  if (p0 >= nnz) return;  // no barrier follows
  const uint32_t p1 = (uint32_t)(p0 + AFF_L < nnz ? p0 + AFF_L : nnz);
  const uint32_t n1 = s.cnt1[c], mask2 = s.mask2[c];
  bool slot0 = false, slot1 = false, first_run = true;
  XYZZ<F> acc = xyzz_inf<F>();
  uint32_t cur = keys[p0];
  // a run is emitted when the next item's key differs (items ascend by key) or at the end
  auto feed = [&](uint32_t key, const Affine<F>& a) {
    if (key != cur) {
      const bool open_left = first_run && p0 > 0 && keys[p0 - 1] == cur;
      msm_emit_run<F>(cur, acc, true, open_left, false, buckets, item_key + 2 * c, item_val + 2 * c, slot0, slot1);
      acc = xyzz_inf<F>();
      cur = key;
      first_run = false;
    }
    acc = xyzz_madd_signed<F>(acc, a, false);
  };
  auto item = [&](uint32_t e, bool& inf) {
    return aff_item(s.ref1[(size_t)e * s.lanes + c], bases, s.pts[0], s.lanes, c, inf);
  };
  // one madd call site (the XYZZ addition is large): each round-2 pair yields its sum, an
  // unpaired pair its one or two items, fed through the same inner loop
#pragma unroll 1
  for (int i = (int)((n1 - 1) >> 1); i >= 0; i--) {
    const uint32_t e0 = 2 * i, e1 = e0 + 1;  // e1 precedes e0 in position
    const bool paired = (mask2 >> i & 1) != 0;
    const int cnt = paired ? 1 : (e1 < n1 ? 2 : 1);
#pragma unroll 1
    for (int q = 0; q < cnt; q++) {
      const uint32_t e = paired ? e0 : (cnt == 2 && q == 0 ? e1 : e0);
      bool inf;
      Affine<F> a = item(e, inf);
      if (paired) {
        const Affine<F> B = item(e1, inf);
        const F29 d = f29_sub_canon(B.x, a.x);
        const F29 ij = f29_mul(inv, aff_ld(s.pref + (size_t)(AFF_P + i) * 9 * s.lanes + c, s.lanes));
        inv = f29_mul(inv, d);
        a = f29_affine_add(a, B, ij);
      }
      feed(s.key1[(size_t)e * s.lanes + c], a);
    }
  }
  const bool open_left = first_run && p0 > 0 && keys[p0 - 1] == cur;
  const bool open_right = p1 < nnz && keys[p1] == cur;
  msm_emit_run<F>(cur, acc, true, open_left, open_right, buckets, item_key + 2 * c, item_val + 2 * c, slot0, slot1);
  if (!slot0) item_key[2 * c] = (uint32_t)keys[p0] | MSM_ITEM_DUMMY;
  if (!slot1) item_key[2 * c + 1] = (uint32_t)keys[p1 - 1] | MSM_ITEM_DUMMY;
}

// entries: the most (base, window) pairs one accumulation covers (cap x W)
inline hipError_t msm_aff_alloc(MsmAffScratch& s, size_t entries) {
  s.lanes = (entries + AFF_L - 1) / AFF_L;
  s.wgs = (s.lanes + AFF_WG - 1) / AFF_WG;
  s.lanes = s.wgs * AFF_WG;
  if (s.wgs > (size_t)AFF_ROOT_T * AFF_ROOT_K) return hipErrorInvalidValue;
  ZK_CHECK(hipMalloc(&s.pref, (size_t)2 * AFF_P * 9 * s.lanes * 4));  // round 1 | round 2
  ZK_CHECK(hipMalloc(&s.tree, s.wgs * 512 * 9 * 4));
  ZK_CHECK(hipMalloc(&s.wgprod, s.wgs * 9 * 4));
  ZK_CHECK(hipMalloc(&s.wginv, s.wgs * 9 * 4));
  ZK_CHECK(hipMalloc(&s.pts[0], (size_t)AFF_P * s.lanes * sizeof(Affine<FqOps>)));
  ZK_CHECK(hipMalloc(&s.mask2, s.lanes * 4));
  ZK_CHECK(hipMalloc(&s.key1, (size_t)AFF_L * s.lanes * 2));
  ZK_CHECK(hipMalloc(&s.ref1, (size_t)AFF_L * s.lanes * 4));
  ZK_CHECK(hipMalloc(&s.cnt1, s.lanes));
  return hipSuccess;
}

inline void msm_aff_free(MsmAffScratch& s) {
  void* ptrs[] = {s.pref, s.tree, s.wgprod, s.wginv, s.pts[0], s.mask2, s.key1, s.ref1, s.cnt1};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  s = MsmAffScratch();
}

// The five launches of one G1 accumulation (bases b, sorted pairs, tail t); chunk count bounded
// by the scratch (host-side upper bound: lanes beyond the device nnz only feed ones to the trees).
template <int MINW>
hipError_t msm_aff_accumulate(const MsmBases<FqOps>& b, const uint16_t* keys, const uint32_t* vals,
                              MsmTail<FqOps>& t, const MsmAffScratch& s, hipStream_t st) {
  const size_t lanes = (b.n * msm_w_of(b.c) + AFF_L - 1) / AFF_L;
  const uint32_t wgs = (uint32_t)((lanes + AFF_WG - 1) / AFF_WG);
  if (wgs > s.wgs || lanes > t.max_chunks) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_aff_prep1, dim3(wgs), dim3(AFF_WG), 0, st, keys, vals, b.bases_w, t.nnz, s);
  hipLaunchKernelGGL(k_aff_root, dim3(1), dim3(AFF_ROOT_T), 0, st, s, wgs);
  hipLaunchKernelGGL(k_aff_apply1, dim3(wgs), dim3(AFF_WG), 0, st, keys, vals, b.bases_w, t.nnz, s);
  hipLaunchKernelGGL(k_aff_root, dim3(1), dim3(AFF_ROOT_T), 0, st, s, wgs);
  hipLaunchKernelGGL((k_aff_apply2_acc<MINW>), dim3(wgs), dim3(AFF_WG), 0, st, keys, b.bases_w, t.nnz, s,
                     t.item_key[0], t.item_val[0], t.buckets);
  return hipGetLastError();
}

}  // namespace zkfl
