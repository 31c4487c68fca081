// ssort.hpp -- sample sort of records with unique 128-bit keys (hi, lo), ascending, in four
// launches and no host round trip.  It replaces the rocPRIM onesweep chains on the C2 path
// (one chain of 5-8 radix passes plus a lookback reset per pass for every key: ~1 ms of sorts
// and ~0.45 ms of fills per 1M-point partition).
//
// Every caller supplies its keys through a functor (KeyF: index -> SKey) and consumes the order
// through another (EmitF: rank, SKey), so key construction and the consumer's gather are fused
// into the first and last kernels.  Keys must be unique (callers put a tie breaker -- an index
// or an id pair -- in `lo`), so the order is fully determined whatever order the scatter's
// atomics place records in, and ties in `hi` never unbalance the buckets.
//
//  1. ss_splitters: 8192 pseudo-random samples sorted by one workgroup in LDS; every
//     (8192/nb)-th is a splitter; zeroes the counters;
//  2. ss_count:  bucket of every record (binary search over the splitters in LDS, 16
//     searches in flight per thread), per-workgroup LDS histogram -> global bucket counts;
//     the bucket id is kept (u16);
//  3. ss_scatter: bucket starts (every workgroup scans the nb counts itself), per-workgroup
//     ranges reserved with one atomic per (workgroup, bucket), records written to them;
//  4. ss_bucket: one workgroup per bucket sorts it (8 records per thread: a register network,
//     then merge-path rounds through LDS) and emits it from registers.  A bucket above SS_CAP
//     (rare: ~4x its expected size) is sorted by its workgroup in SS_CAP chunks and merged
//     pairwise through global scratch -- slower, same result.
// Buckets average <= 1024 records; nb <= SS_MAXB (splitters in LDS).  Larger inputs return
// false and the caller keeps its radix path.
#pragma once
#include "common.hpp"

namespace hdb {

struct SKey {
    uint64_t hi, lo;
};
__device__ __forceinline__ bool sk_less(const SKey &a, const SKey &b) {
    return a.hi < b.hi || (a.hi == b.hi && a.lo < b.lo);
}

constexpr int SS_E = 8;         // records per thread in the LDS merge sorts
constexpr int SS_S = 8192;      // samples: one 1024-thread workgroup sorts them (128 KiB of LDS)
constexpr int SS_CAP = 4096;    // bucket records sorted in LDS (512 threads x 8, 64 KiB)
constexpr int SS_BT = 512;      // ss_bucket / ss_single threads
constexpr int SS_CT = 256;      // ss_count / ss_scatter threads
constexpr int SS_ITEMS = 16;    // records per ss_count / ss_scatter thread
constexpr int SS_MAXB = 4096;   // buckets (splitters 64 KiB in LDS)
constexpr int SS_AVG = 1024;    // target records per bucket

struct SsPlan {
    int64_t n = 0;
    int nb = 1;        // buckets (power of two)
    int64_t ngrp = 0;  // ss_count / ss_scatter workgroups
    int cap = SS_CAP;  // bucket size sorted in LDS; larger buckets take the chunked merge (tests lower it)
    size_t o_buf = 0, o_buf2 = 0, o_bkt = 0, o_spl = 0, o_cnt = 0, o_cur = 0, o_start = 0, bytes = 0;
};

// nb = 0: n too large for the sample sort
inline SsPlan ss_plan(int64_t n, int cap = SS_CAP) {
    SsPlan p;
    p.n = n;
    p.cap = cap >= 2 && cap <= SS_CAP ? cap : SS_CAP;
    if (n <= p.cap) {
        p.nb = 1;
    } else {
        int nb = 2;
        while ((int64_t)nb * SS_AVG < n) nb <<= 1;
        if (nb > SS_MAXB) {
            p.nb = 0;
            return p;
        }
        p.nb = nb;
    }
    p.ngrp = ceil_div(n, (int64_t)SS_CT * SS_ITEMS);
    auto rnd = [](size_t b) { return (b + 255) & ~size_t(255); };
    size_t off = 0;
    auto take = [&](size_t b) {
        size_t o = off;
        off += rnd(b);
        return o;
    };
    if (p.nb > 1) {
        p.o_buf = take(16 * (size_t)n);
        p.o_buf2 = take(16 * (size_t)n);
        p.o_bkt = take(2 * (size_t)n);
        p.o_spl = take(16 * (size_t)p.nb);
        p.o_cnt = take(4 * (size_t)p.nb);
        p.o_cur = take(4 * (size_t)p.nb);
        p.o_start = take(4 * (size_t)p.nb + 4);
    }
    p.bytes = off + 256;
    return p;
}

__device__ __forceinline__ uint64_t ss_mix(uint64_t x) {  // splitmix64 finaliser
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

__device__ __forceinline__ SKey ss_max_key() { return SKey{~0ull, ~0ull}; }  // padding (never a real key)

// component-wise selects: a conditional on the struct itself becomes a select of two stack
// addresses and puts the records in scratch
__device__ __forceinline__ SKey ss_sel(bool c, const SKey &x, const SKey &y) {
    return SKey{c ? x.hi : y.hi, c ? x.lo : y.lo};
}
__device__ __forceinline__ void ss_cas(SKey &a, SKey &b) {
    const bool sw = sk_less(b, a);
    const SKey x = ss_sel(sw, b, a), y = ss_sel(sw, a, b);
    a = x;
    b = y;
}

// E = 8 records in registers, ascending: Batcher's odd-even merge network (19 comparators)
__device__ __forceinline__ void ss_regsort8(SKey (&v)[8]) {
    ss_cas(v[0], v[1]); ss_cas(v[2], v[3]); ss_cas(v[4], v[5]); ss_cas(v[6], v[7]);
    ss_cas(v[0], v[2]); ss_cas(v[1], v[3]); ss_cas(v[4], v[6]); ss_cas(v[5], v[7]);
    ss_cas(v[1], v[2]); ss_cas(v[5], v[6]);
    ss_cas(v[0], v[4]); ss_cas(v[1], v[5]); ss_cas(v[2], v[6]); ss_cas(v[3], v[7]);
    ss_cas(v[2], v[4]); ss_cas(v[3], v[5]);
    ss_cas(v[1], v[2]); ss_cas(v[3], v[4]); ss_cas(v[5], v[6]);
}

// LDS index swizzle: thread t's 8 records (t*8 + k) land in distinct bank groups across 8
// consecutive lanes (16-byte records, 128-byte thread stride)
__device__ __forceinline__ int ss_sw(int i) { return i ^ ((i >> 3) & 7); }

// Merge sort of nthr * 8 records (nthr a power of two <= blockDim.x): thread t holds positions
// [8t, 8t + 8) in v, unsorted on entry, sorted on exit.  Register network, then pairwise
// merge-path rounds through LDS (s: nthr * 8 records; equal keys take the left run first).
// Every thread of the block calls it (barriers); threads >= nthr carry no records.
__device__ __forceinline__ void ss_msort(SKey (&v)[SS_E], SKey *s, int nthr) {
    const int t = threadIdx.x;
    const bool act = t < nthr;
    if (act) ss_regsort8(v);
    for (int w = SS_E; w < nthr * SS_E; w <<= 1) {
        if (act) {
#pragma unroll
            for (int k = 0; k < SS_E; k++) s[ss_sw(t * SS_E + k)] = v[k];
        }
        __syncthreads();
        if (act) {
            const int o = t * SS_E, base = o & ~(2 * w - 1), d = o - base;
            int lo = d > w ? d - w : 0, hi = d < w ? d : w;
            while (lo < hi) {  // the number of left-run records among the pair's first d outputs
                const int mid = (lo + hi) >> 1;
                if (!sk_less(s[ss_sw(base + w + d - 1 - mid)], s[ss_sw(base + mid)])) lo = mid + 1;
                else hi = mid;
            }
            int ia = lo, ib = d - lo;
            SKey a = s[ss_sw(base + (ia < w ? ia : w - 1))], b = s[ss_sw(base + w + (ib < w ? ib : w - 1))];
#pragma unroll
            for (int k = 0; k < SS_E; k++) {
                const bool ta = ib >= w || (ia < w && !sk_less(b, a));
                v[k] = ss_sel(ta, a, b);
                if (ta) {
                    if (++ia < w) a = s[ss_sw(base + ia)];
                } else {
                    if (++ib < w) b = s[ss_sw(base + w + ib)];
                }
            }
        }
        __syncthreads();
    }
}

__device__ __forceinline__ int ss_nthr(int64_t m) {  // power-of-two thread count for m records
    int nt = 1;
    while ((int64_t)nt * SS_E < m) nt <<= 1;
    return nt;
}

// ---- 1. splitters: SS_S pseudo-random samples sorted by one workgroup, every (SS_S/nb)-th
// one kept; zeroes the bucket counters
template <class KeyF>
__global__ __launch_bounds__(1024) void ss_splitters(KeyF kf, int64_t n, int nb, SKey *__restrict__ spl,
                                                     int32_t *__restrict__ cnt, int32_t *__restrict__ cur) {
    __shared__ SKey s[SS_S];
    const int t = threadIdx.x;
    for (int b = t; b < nb; b += 1024) {
        cnt[b] = 0;
        cur[b] = 0;
    }
    SKey v[SS_E];
#pragma unroll
    for (int k = 0; k < SS_E; k++) {
        const uint64_t j = (uint64_t)t * SS_E + k;
        v[k] = kf((int64_t)(ss_mix(j ^ 0x5eed5eedull) % (uint64_t)n));
    }
    ss_msort(v, s, 1024);
    const int per = SS_S / nb;
#pragma unroll
    for (int k = 0; k < SS_E; k++) {
        const int r = t * SS_E + k + 1;
        if (r % per == 0 && r < SS_S) spl[r / per - 1] = v[k];
    }
}

// ---- 2. bucket counts: bucket of x = number of splitters <= x (nb - 1 sorted splitters)
template <class KeyF>
__global__ __launch_bounds__(SS_CT) void ss_count(KeyF kf, int64_t n, int nb, const SKey *__restrict__ gspl,
                                                  uint16_t *__restrict__ bkt, int32_t *__restrict__ cnt) {
    __shared__ SKey spl[SS_MAXB];
    __shared__ int32_t h[SS_MAXB];
    for (int t = threadIdx.x; t < nb - 1; t += SS_CT) spl[t] = gspl[t];
    for (int t = threadIdx.x; t < nb; t += SS_CT) h[t] = 0;
    const int64_t base = (int64_t)blockIdx.x * SS_CT * SS_ITEMS + threadIdx.x;
    SKey x[SS_ITEMS];
    int idx[SS_ITEMS];
#pragma unroll
    for (int k = 0; k < SS_ITEMS; k++) {
        const int64_t i = base + (int64_t)k * SS_CT;
        x[k] = i < n ? kf(i) : ss_max_key();
        idx[k] = 0;
    }
    __syncthreads();
    for (int step = nb >> 1; step >= 1; step >>= 1) {  // all searches advance together (ILP)
#pragma unroll
        for (int k = 0; k < SS_ITEMS; k++)
            if (!sk_less(x[k], spl[idx[k] + step - 1])) idx[k] += step;
    }
#pragma unroll
    for (int k = 0; k < SS_ITEMS; k++) {
        const int64_t i = base + (int64_t)k * SS_CT;
        if (i < n) {
            bkt[i] = (uint16_t)idx[k];
            atomicAdd(&h[idx[k]], 1);
        }
    }
    __syncthreads();
    for (int t = threadIdx.x; t < nb; t += SS_CT)
        if (h[t]) atomicAdd(&cnt[t], h[t]);
}

// exclusive scan of v[0, nb) in LDS (nb <= SS_MAXB, SS_CT threads, in place)
__device__ __forceinline__ void ss_block_scan(int32_t *v, int nb, int32_t *wsum) {
    const int per = (nb + SS_CT - 1) / SS_CT;  // <= 16
    const int t0 = threadIdx.x * per;
    int32_t s = 0;
    for (int k = 0; k < per; k++)
        if (t0 + k < nb) s += v[t0 + k];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int32_t x = s;
    for (int o = 1; o < 64; o <<= 1) {
        const int32_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    int32_t pre = 0;
    for (int w = 0; w < wv; w++) pre += wsum[w];
    int32_t run = pre + x - s;  // exclusive prefix of this thread's range
    for (int k = 0; k < per; k++)
        if (t0 + k < nb) {
            const int32_t c = v[t0 + k];
            v[t0 + k] = run;
            run += c;
        }
    __syncthreads();
}

// ---- 3. scatter into bucket order
template <class KeyF>
__global__ __launch_bounds__(SS_CT) void ss_scatter(KeyF kf, int64_t n, int nb, const uint16_t *__restrict__ bkt,
                                                    const int32_t *__restrict__ cnt, int32_t *__restrict__ cur,
                                                    int32_t *__restrict__ start, SKey *__restrict__ buf) {
    __shared__ int32_t st[SS_MAXB];
    __shared__ int32_t h[SS_MAXB];
    __shared__ int32_t wsum[4];
    for (int t = threadIdx.x; t < nb; t += SS_CT) {
        st[t] = cnt[t];
        h[t] = 0;
    }
    const int64_t base = (int64_t)blockIdx.x * SS_CT * SS_ITEMS + threadIdx.x;
    int mb[SS_ITEMS];
#pragma unroll
    for (int k = 0; k < SS_ITEMS; k++) {
        const int64_t i = base + (int64_t)k * SS_CT;
        mb[k] = i < n ? (int)bkt[i] : -1;
    }
    __syncthreads();
    ss_block_scan(st, nb, wsum);
    if (blockIdx.x == 0) {
        for (int t = threadIdx.x; t < nb; t += SS_CT) start[t] = st[t];
        if (threadIdx.x == 0) start[nb] = (int32_t)n;
    }
#pragma unroll
    for (int k = 0; k < SS_ITEMS; k++)
        if (mb[k] >= 0) atomicAdd(&h[mb[k]], 1);
    __syncthreads();
    // reserve this workgroup's range in every bucket it touches
    for (int t = threadIdx.x; t < nb; t += SS_CT)
        if (h[t]) st[t] += atomicAdd(&cur[t], h[t]);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < SS_ITEMS; k++) {
        if (mb[k] < 0) continue;
        const int pos = atomicAdd(&st[mb[k]], 1);
        buf[pos] = kf(base + (int64_t)k * SS_CT);
    }
}

// ---- 4. per-bucket sort + emit
// rank of x in the sorted run a[0, m) (unique keys: strict count)
__device__ __forceinline__ int64_t ss_count_less(const SKey *a, int64_t m, const SKey &x) {
    int64_t lo = 0, hi = m;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (sk_less(a[mid], x)) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// buf_in and bufB are the same buffer at the call site (the chunked merge's second scratch is
// the scatter output, read before it is overwritten): neither may be __restrict__
template <class EmitF>
__global__ __launch_bounds__(SS_BT) void ss_bucket(EmitF ef, const SKey *buf_in, SKey *__restrict__ bufA,
                                                   SKey *bufB, const int32_t *__restrict__ start, int cap) {
    __shared__ SKey s[SS_CAP];
    const int64_t s0 = start[blockIdx.x], m = start[blockIdx.x + 1] - s0;
    if (m <= 0) return;
    const int t = threadIdx.x;
    SKey v[SS_E];
    if (m <= cap) {
        const int nthr = ss_nthr(m);
#pragma unroll
        for (int k = 0; k < SS_E; k++) {
            const int64_t p = (int64_t)t * SS_E + k;
            v[k] = p < m ? buf_in[s0 + p] : ss_max_key();
        }
        ss_msort(v, s, nthr);
#pragma unroll
        for (int k = 0; k < SS_E; k++) {
            const int64_t p = (int64_t)t * SS_E + k;
            if (p < m) ef(s0 + p, v[k]);
        }
        return;
    }
    // big bucket: cap-record chunks sorted in LDS into bufA, then pairwise merges A <-> B
    for (int64_t c0 = 0; c0 < m; c0 += cap) {
        const int len = (int)(m - c0 < cap ? m - c0 : cap);
#pragma unroll
        for (int k = 0; k < SS_E; k++) {
            const int p = t * SS_E + k;
            v[k] = p < len ? buf_in[s0 + c0 + p] : ss_max_key();
        }
        ss_msort(v, s, ss_nthr(len));
#pragma unroll
        for (int k = 0; k < SS_E; k++) {
            const int p = t * SS_E + k;
            if (p < len) bufA[s0 + c0 + p] = v[k];
        }
    }
    SKey *src = bufA + s0, *dst = bufB + s0;
    for (int64_t wdt = cap; wdt < m; wdt <<= 1) {
        __threadfence_block();
        __syncthreads();
        for (int64_t i = t; i < m; i += SS_BT) {
            const int64_t pair = i / (2 * wdt), l0 = pair * 2 * wdt;
            const int64_t l1 = l0 + wdt < m ? l0 + wdt : m, r1 = l0 + 2 * wdt < m ? l0 + 2 * wdt : m;
            const SKey x = src[i];
            int64_t o;
            if (i < l1) o = l0 + (i - l0) + ss_count_less(src + l1, r1 - l1, x);
            else o = l0 + (i - l1) + ss_count_less(src + l0, l1 - l0, x);
            dst[o] = x;
        }
        SKey *tmp = src;
        src = dst;
        dst = tmp;
    }
    __threadfence_block();
    __syncthreads();
    for (int64_t i = t; i < m; i += SS_BT) ef(s0 + i, src[i]);
}

// nb == 1: one workgroup, keys straight from the functor
template <class KeyF, class EmitF>
__global__ __launch_bounds__(SS_BT) void ss_single(KeyF kf, EmitF ef, int64_t n) {
    __shared__ SKey s[SS_CAP];
    const int t = threadIdx.x;
    SKey v[SS_E];
#pragma unroll
    for (int k = 0; k < SS_E; k++) {
        const int64_t p = (int64_t)t * SS_E + k;
        v[k] = p < n ? kf(p) : ss_max_key();
    }
    ss_msort(v, s, ss_nthr(n));
#pragma unroll
    for (int k = 0; k < SS_E; k++) {
        const int64_t p = (int64_t)t * SS_E + k;
        if (p < n) ef(p, v[k]);
    }
}

// Enqueues the sort on `st` with scratch at `base` (ss_plan(n).bytes); false: n too large.
template <class KeyF, class EmitF>
bool ssort(const SsPlan &p, char *base, KeyF kf, EmitF ef, hipStream_t st) {
    const int64_t n = p.n;
    if (n <= 0) return true;
    if (p.nb == 0) return false;
    if (p.nb == 1) {
        hipLaunchKernelGGL((ss_single<KeyF, EmitF>), dim3(1), dim3(SS_BT), 0, st, kf, ef, n);
        HIP_CHECK(hipGetLastError());
        return true;
    }
    SKey *buf = (SKey *)(base + p.o_buf), *buf2 = (SKey *)(base + p.o_buf2), *spl = (SKey *)(base + p.o_spl);
    uint16_t *bkt = (uint16_t *)(base + p.o_bkt);
    int32_t *cnt = (int32_t *)(base + p.o_cnt), *cur = (int32_t *)(base + p.o_cur),
            *start = (int32_t *)(base + p.o_start);
    hipLaunchKernelGGL((ss_splitters<KeyF>), dim3(1), dim3(1024), 0, st, kf, n, p.nb, spl, cnt, cur);
    hipLaunchKernelGGL((ss_count<KeyF>), dim3((unsigned)p.ngrp), dim3(SS_CT), 0, st, kf, n, p.nb, spl, bkt, cnt);
    hipLaunchKernelGGL((ss_scatter<KeyF>), dim3((unsigned)p.ngrp), dim3(SS_CT), 0, st, kf, n, p.nb, bkt, cnt, cur, start,
                       buf);
    hipLaunchKernelGGL((ss_bucket<EmitF>), dim3((unsigned)p.nb), dim3(SS_BT), 0, st, ef, buf, buf2, buf, start, p.cap);
    HIP_CHECK(hipGetLastError());
    return true;
}

}  // namespace hdb
