// ssort.hpp -- sample sort of records with unique 128-bit keys (hi, lo), ascending, in five
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
//  1. ss_sample: S = nb x 4 pseudo-random samples, sorted per 1024-sample chunk in LDS;
//  2. ss_split:  each sample's rank over all chunks (its chunk rank + binary searches in the
//     other chunks, ties by chunk) -> every 4th sample is a splitter; zeroes the counters;
//  3. ss_count:  bucket of every record (binary search over the splitters in LDS), per-
//     workgroup LDS histogram -> global bucket counts; the bucket id is kept (u16);
//  4. ss_scatter: bucket starts (every workgroup scans the nb counts itself), per-workgroup
//     ranges reserved with one atomic per (workgroup, bucket), records written to them;
//  5. ss_bucket: one workgroup per bucket sorts it in LDS (bitonic) and emits it.  A bucket
//     above SS_CAP (rare: ~4x its expected size) is sorted by its workgroup in SS_CAP chunks
//     and merged pairwise through global scratch -- slower, same result.
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

constexpr int SS_CHUNK = 1024;  // samples per ss_sample workgroup (512 threads x 2)
constexpr int SS_OVS = 4;       // samples per bucket
constexpr int SS_CAP = 4096;    // bucket records sorted in LDS (64 KiB)
constexpr int SS_BT = 512;      // ss_bucket / ss_sample threads
constexpr int SS_CT = 256;      // ss_count / ss_scatter threads
constexpr int SS_ITEMS = 16;    // records per ss_count / ss_scatter thread
constexpr int SS_MAXB = 4096;   // buckets (splitters 64 KiB in LDS)
constexpr int SS_AVG = 1024;    // target records per bucket

struct SsPlan {
    int64_t n = 0;
    int nb = 1;     // buckets (power of two)
    int S = 0;      // samples
    int nchunk = 0;
    int64_t ngrp = 0;  // ss_count / ss_scatter workgroups
    int cap = SS_CAP;  // bucket size sorted in LDS; larger buckets take the chunked merge (tests lower it)
    size_t o_buf = 0, o_buf2 = 0, o_bkt = 0, o_samp = 0, o_spl = 0, o_cnt = 0, o_cur = 0, o_start = 0, bytes = 0;
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
        p.S = nb * SS_OVS;
        if (p.S < SS_CHUNK) p.S = SS_CHUNK;
        p.nchunk = p.S / SS_CHUNK;
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
        p.o_samp = take(16 * (size_t)p.S);
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

// Ascending bitonic sort of s[0, P) in LDS (P a power of two, padded by the caller), all
// threads of the block; ends with a barrier.
template <int BT>
__device__ __forceinline__ void ss_bitonic(SKey *s, int P) {
    for (int k = 2; k <= P; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int t = threadIdx.x; t < (P >> 1); t += BT) {
                const int i = 2 * t - (t & (j - 1));
                const int l = i + j;
                const SKey a = s[i], b = s[l];
                const bool up = (i & k) == 0;
                if (sk_less(b, a) == up) {
                    s[i] = b;
                    s[l] = a;
                }
            }
            __syncthreads();
        }
    }
}

__device__ __forceinline__ SKey ss_max_key() { return SKey{~0ull, ~0ull}; }

// ---- 1. samples, sorted per chunk
template <class KeyF>
__global__ __launch_bounds__(SS_BT) void ss_sample(KeyF kf, int64_t n, int S, SKey *__restrict__ samp) {
    __shared__ SKey s[SS_CHUNK];
    const int c = blockIdx.x;
    for (int t = threadIdx.x; t < SS_CHUNK; t += SS_BT) {
        const uint64_t j = (uint64_t)c * SS_CHUNK + t;
        const int64_t i = (int64_t)(ss_mix(j ^ 0x5eed5eedull) % (uint64_t)n);
        s[t] = kf(i);
    }
    __syncthreads();
    ss_bitonic<SS_BT>(s, SS_CHUNK);
    for (int t = threadIdx.x; t < SS_CHUNK; t += SS_BT) samp[(int64_t)c * SS_CHUNK + t] = s[t];
}

// ---- 2. global sample ranks -> splitters; zero the bucket counters
static __global__ void ss_split(const SKey *__restrict__ samp, int S, int nchunk, int nb, SKey *__restrict__ spl,
                         int32_t *__restrict__ cnt, int32_t *__restrict__ cur) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    for (int b = j; b < nb; b += gridDim.x * blockDim.x) {
        cnt[b] = 0;
        cur[b] = 0;
    }
    if (j >= S) return;
    const int c = j / SS_CHUNK;
    const SKey x = samp[j];
    int rank = j - c * SS_CHUNK;
    for (int o = 0; o < nchunk; o++) {
        if (o == c) continue;
        const SKey *a = samp + (int64_t)o * SS_CHUNK;
        // chunks before c: count elements <= x; after c: < x (equal samples ordered by chunk)
        int lo = 0, hi = SS_CHUNK;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            const bool before = o < c ? !sk_less(x, a[mid]) : sk_less(a[mid], x);
            if (before) lo = mid + 1;
            else hi = mid;
        }
        rank += lo;
    }
    const int per = S / nb;
    if ((rank + 1) % per == 0 && rank + 1 < S) spl[(rank + 1) / per - 1] = x;
}

// bucket of x = number of splitters <= x (splitters sorted ascending, nb - 1 of them)
__device__ __forceinline__ int ss_bucket_of(const SKey *spl, int nb, const SKey &x) {
    int lo = 0, hi = nb - 1;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (!sk_less(x, spl[mid])) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// ---- 3. bucket counts
template <class KeyF>
__global__ __launch_bounds__(SS_CT) void ss_count(KeyF kf, int64_t n, int nb, const SKey *__restrict__ gspl,
                                                  uint16_t *__restrict__ bkt, int32_t *__restrict__ cnt) {
    __shared__ SKey spl[SS_MAXB];
    __shared__ int32_t h[SS_MAXB];
    for (int t = threadIdx.x; t < nb - 1; t += SS_CT) spl[t] = gspl[t];
    for (int t = threadIdx.x; t < nb; t += SS_CT) h[t] = 0;
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * SS_CT * SS_ITEMS;
    for (int k = 0; k < SS_ITEMS; k++) {
        const int64_t i = base + (int64_t)k * SS_CT + threadIdx.x;
        if (i >= n) break;
        const int b = ss_bucket_of(spl, nb, kf(i));
        bkt[i] = (uint16_t)b;
        atomicAdd(&h[b], 1);
    }
    __syncthreads();
    for (int t = threadIdx.x; t < nb; t += SS_CT)
        if (h[t]) atomicAdd(&cnt[t], h[t]);
}

// exclusive scan of v[0, nb) in LDS (nb <= SS_MAXB, SS_CT threads, in place); returns the total
__device__ __forceinline__ int32_t ss_block_scan(int32_t *v, int nb, int32_t *wsum) {
    const int per = (nb + SS_CT - 1) / SS_CT;  // <= 16
    const int t0 = threadIdx.x * per;
    int32_t s = 0;
    for (int k = 0; k < per; k++)
        if (t0 + k < nb) s += v[t0 + k];
    // inclusive scan of the per-thread sums across the block
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
    const int32_t tot = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
    return tot;
}

// ---- 4. scatter into bucket order
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
    __syncthreads();
    ss_block_scan(st, nb, wsum);
    if (blockIdx.x == 0) {
        for (int t = threadIdx.x; t < nb; t += SS_CT) start[t] = st[t];
        if (threadIdx.x == 0) start[nb] = (int32_t)n;
    }
    const int64_t base = (int64_t)blockIdx.x * SS_CT * SS_ITEMS;
    uint16_t mb[SS_ITEMS];
    for (int k = 0; k < SS_ITEMS; k++) {
        const int64_t i = base + (int64_t)k * SS_CT + threadIdx.x;
        mb[k] = i < n ? bkt[i] : 0;
        if (i < n) atomicAdd(&h[mb[k]], 1);
    }
    __syncthreads();
    // reserve this workgroup's range in every bucket it touches
    for (int t = threadIdx.x; t < nb; t += SS_CT)
        if (h[t]) st[t] += atomicAdd(&cur[t], h[t]);
    __syncthreads();
    for (int k = 0; k < SS_ITEMS; k++) {
        const int64_t i = base + (int64_t)k * SS_CT + threadIdx.x;
        if (i >= n) break;
        const int pos = atomicAdd(&st[mb[k]], 1);
        buf[pos] = kf(i);
    }
}

// ---- 5. per-bucket sort + emit
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

template <class EmitF>
__global__ __launch_bounds__(SS_BT) void ss_bucket(EmitF ef, const SKey *__restrict__ buf_in, SKey *__restrict__ bufA,
                                                   SKey *__restrict__ bufB, const int32_t *__restrict__ start,
                                                   int cap) {
    __shared__ SKey s[SS_CAP];
    const int64_t s0 = start[blockIdx.x], m = start[blockIdx.x + 1] - s0;
    if (m <= 0) return;
    if (m <= cap) {
        int P = 1;
        while (P < m) P <<= 1;
        for (int t = threadIdx.x; t < P; t += SS_BT) s[t] = t < m ? buf_in[s0 + t] : ss_max_key();
        __syncthreads();
        ss_bitonic<SS_BT>(s, P);
        for (int t = threadIdx.x; t < m; t += SS_BT) ef(s0 + t, s[t]);
        return;
    }
    // big bucket: cap-record chunks sorted in LDS into bufA, then pairwise merges A <-> B
    for (int64_t c0 = 0; c0 < m; c0 += cap) {
        const int len = (int)(m - c0 < cap ? m - c0 : cap);
        int P = 1;
        while (P < len) P <<= 1;
        for (int t = threadIdx.x; t < P; t += SS_BT) s[t] = t < len ? buf_in[s0 + c0 + t] : ss_max_key();
        __syncthreads();
        ss_bitonic<SS_BT>(s, P);
        for (int t = threadIdx.x; t < len; t += SS_BT) bufA[s0 + c0 + t] = s[t];
        __syncthreads();
    }
    SKey *src = bufA + s0, *dst = bufB + s0;
    for (int64_t wdt = cap; wdt < m; wdt <<= 1) {
        __threadfence_block();
        __syncthreads();
        for (int64_t i = threadIdx.x; i < m; i += SS_BT) {
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
    for (int64_t i = threadIdx.x; i < m; i += SS_BT) ef(s0 + i, src[i]);
}

// nb == 1: load through the key functor directly
template <class KeyF, class EmitF>
__global__ __launch_bounds__(SS_BT) void ss_single(KeyF kf, EmitF ef, int64_t n) {
    __shared__ SKey s[SS_CAP];
    int P = 1;
    while (P < n) P <<= 1;
    for (int t = threadIdx.x; t < P; t += SS_BT) s[t] = t < n ? kf(t) : ss_max_key();
    __syncthreads();
    ss_bitonic<SS_BT>(s, P);
    for (int t = threadIdx.x; t < n; t += SS_BT) ef(t, s[t]);
}

// Enqueues the sort on `st` with scratch at `base` (ss_plan(n).bytes); false: n too large.
template <class KeyF, class EmitF>
bool ssort(const SsPlan &p, char *base, KeyF kf, EmitF ef, hipStream_t st) {
    const int64_t n = p.n;
    if (n <= 0) return true;
    if (p.nb == 0) return false;
    if (p.nb == 1 && n <= p.cap) {
        hipLaunchKernelGGL((ss_single<KeyF, EmitF>), dim3(1), dim3(SS_BT), 0, st, kf, ef, n);
        HIP_CHECK(hipGetLastError());
        return true;
    }
    SKey *buf = (SKey *)(base + p.o_buf), *buf2 = (SKey *)(base + p.o_buf2), *samp = (SKey *)(base + p.o_samp),
         *spl = (SKey *)(base + p.o_spl);
    uint16_t *bkt = (uint16_t *)(base + p.o_bkt);
    int32_t *cnt = (int32_t *)(base + p.o_cnt), *cur = (int32_t *)(base + p.o_cur),
            *start = (int32_t *)(base + p.o_start);
    hipLaunchKernelGGL((ss_sample<KeyF>), dim3(p.nchunk), dim3(SS_BT), 0, st, kf, n, p.S, samp);
    hipLaunchKernelGGL(ss_split, dim3((unsigned)ceil_div(p.S, 256)), dim3(256), 0, st, samp, p.S, p.nchunk, p.nb, spl,
                       cnt, cur);
    hipLaunchKernelGGL((ss_count<KeyF>), dim3((unsigned)p.ngrp), dim3(SS_CT), 0, st, kf, n, p.nb, spl, bkt, cnt);
    hipLaunchKernelGGL((ss_scatter<KeyF>), dim3((unsigned)p.ngrp), dim3(SS_CT), 0, st, kf, n, p.nb, bkt, cnt, cur, start,
                       buf);
    hipLaunchKernelGGL((ss_bucket<EmitF>), dim3((unsigned)p.nb), dim3(SS_BT), 0, st, ef, buf, buf2, buf, start, p.cap);
    HIP_CHECK(hipGetLastError());
    return true;
}

}  // namespace hdb
