// Sparse emulation of torch.sort's tie order for the top-p filter (parity mode).
//
// The reference's top_k_top_p_filtering (hf_export/modeling_t5gemma_voice.py:84-130) sorts
// the whole row of V logits after the top-k filter, so every entry is -inf except the top-k
// survivors. torch 2.10's CPU sort (stable=False) runs libstdc++'s std::sort over
// (value, index) pairs with a value-only descending comparator (SURVEY a14' 5; GCC 11, the
// compiler torch 2.10 was built with): introsort (median-of-3 pivot, Hoare partition,
// depth limit 2 floor(log2 n), ranges of <= 16 left alone) then one insertion sort over the
// whole array. Equal values end in an order fixed by that run, and the top-p cut keeps the
// first members of a tie group it cuts through.
//
// Only the survivors' final positions matter (all other entries are indistinguishable
// -inf values), so this follows the algorithm on the survivors alone:
// * ranges holding no survivor are skipped (nothing observable happens in them);
// * a partition whose pivot is -inf swaps the k-th -inf slot from the left with the k-th
//   slot from the right until the pointers meet -- closed form: survivor at p in the last
//   K slots moves to the (last - 1 - p)-th -inf slot, K from one walk over the survivors;
// * a partition on a survivor pivot is simulated move by move; its right pointer jumps
//   over -inf runs to the previous survivor >= pivot;
// * the final insertion sort moves each survivor left to just after the nearest survivor
//   >= it (or to slot 0).
// O(S^2 log n) worst case for S survivors, O(S log n) typical. Unsupported (fail != 0, the caller falls back to the host
// std::sort): a heapsort fallback (depth limit reached), stack overflow, NaN values.
// Shared by the device sampler (one thread, LDS arrays) and the host (tests, C-ABI).
#pragma once
#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define SE_HD __host__ __device__ __forceinline__
#else
#define SE_HD inline
#endif

namespace t5g {

constexpr int SE_STACK = 96;   // pending ranges (each holds a survivor)

struct SortEmu {
    int n;        // array length (V)
    int S;        // survivors
    int* pos;     // [S] positions, ascending
    float* val;   // [S] values (finite)
    int* tag;     // [S] caller tags, carried with the values
    int fail;
};

SE_HD int se_lower(const SortEmu& E, int p) {   // first array index with pos >= p
    int lo = 0, hi = E.S;
    while (lo < hi) {
        const int m = (lo + hi) >> 1;
        if (E.pos[m] < p) lo = m + 1;
        else hi = m;
    }
    return lo;
}
SE_HD float se_val(const SortEmu& E, int p) {
    const int i = se_lower(E, p);
    return (i < E.S && E.pos[i] == p) ? E.val[i] : -INFINITY;
}
// move array entry i to position np, keeping the arrays ordered by position
SE_HD void se_move(SortEmu& E, int i, int np) {
    const float v = E.val[i];
    const int t = E.tag[i];
    if (np > E.pos[i]) {
        while (i + 1 < E.S && E.pos[i + 1] < np) {
            E.pos[i] = E.pos[i + 1]; E.val[i] = E.val[i + 1]; E.tag[i] = E.tag[i + 1];
            ++i;
        }
    } else {
        while (i > 0 && E.pos[i - 1] > np) {
            E.pos[i] = E.pos[i - 1]; E.val[i] = E.val[i - 1]; E.tag[i] = E.tag[i - 1];
            --i;
        }
    }
    E.pos[i] = np; E.val[i] = v; E.tag[i] = t;
}
// std::iter_swap of the slots p and q
SE_HD void se_swap(SortEmu& E, int p, int q) {
    if (p == q) return;
    const int a = se_lower(E, p), b = se_lower(E, q);
    const bool ha = a < E.S && E.pos[a] == p, hb = b < E.S && E.pos[b] == q;
    if (ha && hb) {
        const float v = E.val[a]; E.val[a] = E.val[b]; E.val[b] = v;
        const int t = E.tag[a]; E.tag[a] = E.tag[b]; E.tag[b] = t;
    } else if (ha) {
        se_move(E, a, q);
    } else if (hb) {
        se_move(E, b, p);
    }
}
SE_HD bool se_any(const SortEmu& E, int lo, int hi) {   // a survivor in [lo, hi)
    const int i = se_lower(E, lo);
    return i < E.S && E.pos[i] < hi;
}

// std::__move_median_to_first(result, a, b, c) with comp(x, y) = x > y
SE_HD void se_median_to_first(SortEmu& E, int result, int a, int b, int c) {
    const float va = se_val(E, a), vb = se_val(E, b), vc = se_val(E, c);
    int m;
    if (va > vb) {
        if (vb > vc) m = b;
        else if (va > vc) m = c;
        else m = a;
    } else if (va > vc) m = a;
    else if (vb > vc) m = c;
    else m = b;
    se_swap(E, result, m);
}

// std::__unguarded_partition(first, last, pivot) with the pivot value at slot pivot_pos
SE_HD int se_partition(SortEmu& E, int first, int last, int pivot_pos) {
    const float pv = se_val(E, pivot_pos);
    if (pv == -INFINITY) {
        // the left pointer stops on every -inf slot, the right one on every slot:
        // iteration k swaps f(k) (the k-th -inf slot from `first`) with l(k) = last - 1 - k
        // until f(K) >= l(K). With c survivors of the range before it, f(k) = first + k + c
        // on a k interval: walk the intervals for the smallest k with 2k >= last-1-first-c.
        const int i0 = se_lower(E, first), i1 = se_lower(E, last);
        const long span = (long)last - 1 - first;
        long K = 0, fK = first;
        for (int c = 0; c <= i1 - i0; ++c) {
            const long klo = c == 0 ? 0 : (long)E.pos[i0 + c - 1] - first - c + 1;
            const long khi = c == i1 - i0 ? span + 1 : (long)E.pos[i0 + c] - first - c - 1;
            if (klo > khi) continue;
            const long kneed = span - c <= 0 ? 0 : (span - c + 1) / 2;
            const long k = klo > kneed ? klo : kneed;
            if (k <= khi) {
                K = k;
                fK = first + k + c;
                break;
            }
        }
        long ret = fK;
        if (K > 0 && ret > (long)last - K) ret = (long)last - K;   // stops on the slot swapped last
        // survivors in the last K slots move to the -inf slots f(last - 1 - p) (every one
        // left of slot last - K: f(k) <= f(K - 1) < l(K - 1)); visiting them by decreasing p
        // visits k increasing, so one walk over the survivors below the region finds them
        const int jm = se_lower(E, (int)((long)last - K));
        int c = 0;
        for (int j = i1 - 1; j >= jm; --j) {
            const long k = (long)last - 1 - E.pos[j];
            while (i0 + c < jm && E.pos[i0 + c] <= first + k + c) ++c;
            E.pos[j] = (int)(first + k + c);
        }
        // the moved ones (now in decreasing slot order) back into slot order
        for (int j = i0 + 1; j < i1; ++j) {
            const int pj = E.pos[j], tj = E.tag[j];
            const float vj = E.val[j];
            int k = j - 1;
            while (k >= i0 && E.pos[k] > pj) {
                E.pos[k + 1] = E.pos[k]; E.val[k + 1] = E.val[k]; E.tag[k + 1] = E.tag[k];
                --k;
            }
            E.pos[k + 1] = pj; E.val[k + 1] = vj; E.tag[k + 1] = tj;
        }
        return (int)ret;
    }
    // survivor pivot: simulate
    int f = first, l = last;
    for (;;) {
        while (se_val(E, f) > pv) ++f;
        --l;
        {   // while (pv > *l) --l: to the previous slot holding a value >= pv (the pivot's
            // own slot bounds it)
            int j = se_lower(E, l + 1) - 1;
            while (j >= 0 && E.val[j] < pv) --j;
            if (j < 0) { E.fail = 3; return f; }
            l = E.pos[j];
        }
        if (!(f < l)) return f;
        se_swap(E, f, l);
        ++f;
    }
}

// std::sort over the whole array; afterwards pos[] holds the survivors' final slots
SE_HD int se_sort(SortEmu& E) {
    E.fail = 0;
    for (int i = 0; i < E.S; ++i)
        if (E.val[i] != E.val[i]) { E.fail = 1; return E.fail; }   // NaN: comparator special case
    if (E.n <= 1 || E.S == 0) return 0;
    int lg = 0;
    while ((2L << lg) <= E.n) ++lg;   // std::__lg(n)
    int st_first[SE_STACK], st_last[SE_STACK], st_depth[SE_STACK];
    int sp = 0;
    st_first[sp] = 0; st_last[sp] = E.n; st_depth[sp] = 2 * lg; ++sp;
    while (sp > 0) {
        --sp;
        int first = st_first[sp], last = st_last[sp], depth = st_depth[sp];
        while (last - first > 16 && se_any(E, first, last)) {
            if (depth == 0) { E.fail = 4; return E.fail; }   // heapsort fallback: not emulated
            --depth;
            const int mid = first + (last - first) / 2;
            se_median_to_first(E, first, first + 1, mid, last - 1);
            const int cut = se_partition(E, first + 1, last, first);
            if (E.fail) return E.fail;
            if (se_any(E, cut, last)) {
                if (sp == SE_STACK) { E.fail = 5; return E.fail; }
                st_first[sp] = cut; st_last[sp] = last; st_depth[sp] = depth; ++sp;
            }
            last = cut;
        }
    }
    // final insertion sort: each survivor, in slot order, moves left past -inf slots and
    // smaller survivors to just after the nearest survivor >= it (slot 0 if none)
    for (int i = 0; i < E.S; ++i) {
        const float v = E.val[i];
        int j = i - 1;
        while (j >= 0 && E.val[j] < v) --j;
        const int np = j >= 0 ? E.pos[j] + 1 : 0;
        if (j < 0 && E.pos[i] >= 16) { E.fail = 6; return E.fail; }   // no sentinel: cannot happen after introsort
        if (np == E.pos[i]) continue;
        // survivors j+1 .. i-1 shift right by one slot, survivor i lands at np
        const int t = E.tag[i];
        for (int k = i; k > j + 1; --k) {
            E.pos[k] = E.pos[k - 1] + 1; E.val[k] = E.val[k - 1]; E.tag[k] = E.tag[k - 1];
        }
        E.pos[j + 1] = np; E.val[j + 1] = v; E.tag[j + 1] = t;
    }
    return 0;
}

#if defined(__HIPCC__)
// ---- the same replay on one wave: survivor i of S <= 63 in lane i, lanes kept sorted by
// slot (inactive lanes: slot INT_MAX, value -inf), so "index by slot" is the lane index and
// the rank / membership / lookup queries are ballots. Every function is called by all 64
// lanes of the wave with uniform arguments; the pending-range stack lives in LDS
// (st_* [SE_STACK], this wave only). Same steps, same results as se_sort.
struct SEWave {
    int n, S;
    int pos;      // this lane's survivor slot (INT_MAX: none)
    float val;
    int tag;
    int fail;
};

__device__ __forceinline__ int sew_lane() { return (int)(threadIdx.x & 63); }
__device__ __forceinline__ int sew_rank_lt(const SEWave& W, int p) { return __popcll(__ballot(W.pos < p)); }
__device__ __forceinline__ bool sew_any(const SEWave& W, int lo, int hi) { return __ballot(W.pos >= lo && W.pos < hi) != 0ull; }
__device__ __forceinline__ int sew_rdi(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ float sew_rdf(float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); }
__device__ __forceinline__ float sew_val_at(const SEWave& W, int p) {
    const unsigned long long m = __ballot(W.pos == p);
    return m ? sew_rdf(W.val, __ffsll((long long)m) - 1) : -INFINITY;
}
// lanes back into slot order (bitonic network over the 64 lanes)
__device__ __forceinline__ void sew_sort_lanes(SEWave& W) {
    const int lane = sew_lane();
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1)
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const int pp = __shfl_xor(W.pos, j, 64);
            const float pv = __shfl_xor(W.val, j, 64);
            const int pt = __shfl_xor(W.tag, j, 64);
            const bool up = (lane & k) == 0, lower = (lane & j) == 0;
            const bool take = lower == up ? pp < W.pos : pp > W.pos;
            if (take) { W.pos = pp; W.val = pv; W.tag = pt; }
        }
}
// std::iter_swap of the slots p != q
__device__ __forceinline__ void sew_swap(SEWave& W, int p, int q) {
    if (p == q) return;
    const int lane = sew_lane();
    const unsigned long long mp = __ballot(W.pos == p), mq = __ballot(W.pos == q);
    if (mp && mq) {   // both hold survivors: exchange value and tag (slots keep their order)
        const int lp = __ffsll((long long)mp) - 1, lq = __ffsll((long long)mq) - 1;
        const float vp = sew_rdf(W.val, lp), vq = sew_rdf(W.val, lq);
        const int tp = sew_rdi(W.tag, lp), tq = sew_rdi(W.tag, lq);
        if (lane == lp) { W.val = vq; W.tag = tq; }
        if (lane == lq) { W.val = vp; W.tag = tp; }
    } else if (mp || mq) {
        if (W.pos == p) W.pos = q;
        else if (W.pos == q) W.pos = p;
        sew_sort_lanes(W);
    }
}
__device__ __forceinline__ void sew_median_to_first(SEWave& W, int result, int a, int b, int c) {
    const float va = sew_val_at(W, a), vb = sew_val_at(W, b), vc = sew_val_at(W, c);
    int m;
    if (va > vb) {
        if (vb > vc) m = b;
        else if (va > vc) m = c;
        else m = a;
    } else if (va > vc) m = a;
    else if (vb > vc) m = c;
    else m = b;
    sew_swap(W, result, m);
}
__device__ __forceinline__ int sew_partition(SEWave& W, int first, int last, int pivot_pos) {
    const int lane = sew_lane();
    const float pv = sew_val_at(W, pivot_pos);
    if (pv == -INFINITY) {   // se_partition's closed form, every interval / survivor on its own lane
        const int i0 = sew_rank_lt(W, first), i1 = sew_rank_lt(W, last);
        const int span = last - 1 - first;
        const int c = lane - i0;
        const int prev = __shfl_up(W.pos, 1, 64);
        const int klo = c == 0 ? 0 : prev - first - c + 1;
        const int khi = c == i1 - i0 ? span + 1 : W.pos - first - c - 1;
        const int kneed = span - c <= 0 ? 0 : (span - c + 1) / 2;
        const int k = klo > kneed ? klo : kneed;
        const unsigned long long ok = __ballot(lane >= i0 && lane <= i1 && klo <= khi && k <= khi);
        int K = 0, fK = first;
        if (ok) {
            const int cs = __ffsll((long long)ok) - 1;
            K = sew_rdi(k, cs);
            fK = first + K + (cs - i0);
        }
        int ret = fK;
        if (K > 0 && ret > last - K) ret = last - K;
        const int jm = sew_rank_lt(W, last - K);
        // survivors j in [jm, i1) move to the (last - 1 - pos)-th -inf slot from first:
        // slot first + k + c, c = #staying survivors t (lanes [i0, jm)) with
        // pos_t - (t - i0) <= first + k (non-decreasing in t: a binary search)
        // (every lane runs the search: a shuffle reads only from active lanes)
        const int d = (lane >= i0 && lane < jm) ? W.pos - (lane - i0) : 0x7fffffff;
        const bool mover = lane >= jm && lane < i1;
        const int kj = mover ? last - 1 - W.pos : 0;
        int lo = i0, hi = jm;
        for (int it = 0; it < 7; ++it) {
            const int mid = (lo + hi) >> 1;
            const int dm = __shfl(d, mid & 63, 64);
            if (lo < hi) {
                if (dm <= first + kj) lo = mid + 1;
                else hi = mid;
            }
        }
        if (mover) W.pos = first + kj + (lo - i0);
        sew_sort_lanes(W);
        return ret;
    }
    // survivor pivot: the Hoare loop, each step a wave query
    int f = first, l = last;
    for (;;) {
        while (sew_val_at(W, f) > pv) ++f;
        --l;
        const unsigned long long m = __ballot(W.pos <= l && W.val >= pv && W.pos != 0x7fffffff);
        if (!m) { W.fail = 3; return f; }
        l = sew_rdi(W.pos, 63 - __clzll((long long)m));
        if (!(f < l)) return f;
        sew_swap(W, f, l);
        ++f;
    }
}

// se_sort on one wave. Inputs in lanes 0..S-1 sorted by slot; returns the fail code
// (0: lanes 0..S-1 hold the survivors in final slot order).
__device__ inline int se_sort_wave(SEWave& W, int* st_first, int* st_last, int* st_depth) {
    const int lane = sew_lane();
    W.fail = 0;
    if (__ballot(lane < W.S && W.val != W.val)) { W.fail = 1; return W.fail; }
    if (W.n <= 1 || W.S == 0) return 0;
    int lg = 0;
    while ((2L << lg) <= W.n) ++lg;
    int sp = 0;
    if (lane == 0) { st_first[0] = 0; st_last[0] = W.n; st_depth[0] = 2 * lg; }
    ++sp;
    while (sp > 0) {
        --sp;
        __builtin_amdgcn_wave_barrier();
        int first = __builtin_amdgcn_readfirstlane(st_first[sp]);
        int last = __builtin_amdgcn_readfirstlane(st_last[sp]);
        int depth = __builtin_amdgcn_readfirstlane(st_depth[sp]);
        while (last - first > 16 && sew_any(W, first, last)) {
            if (depth == 0) { W.fail = 4; return W.fail; }
            --depth;
            const int mid = first + (last - first) / 2;
            sew_median_to_first(W, first, first + 1, mid, last - 1);
            const int cut = sew_partition(W, first + 1, last, first);
            if (W.fail) return W.fail;
            if (sew_any(W, cut, last)) {
                if (sp == SE_STACK) { W.fail = 5; return W.fail; }
                if (lane == 0) { st_first[sp] = cut; st_last[sp] = last; st_depth[sp] = depth; }
                __builtin_amdgcn_wave_barrier();
                ++sp;
            }
            last = cut;
        }
    }
    // final insertion sort, survivor by survivor in slot order
    for (int i = 0; i < W.S; ++i) {
        const float v = sew_rdf(W.val, i);
        const int pi = sew_rdi(W.pos, i), t = sew_rdi(W.tag, i);
        const unsigned long long m = __ballot(lane < i && W.val >= v);
        const int j = m ? 63 - __clzll((long long)m) : -1;
        const int np = j >= 0 ? sew_rdi(W.pos, j) + 1 : 0;
        if (j < 0 && pi >= 16) { W.fail = 6; return W.fail; }
        if (np == pi) continue;
        const int up_p = __shfl_up(W.pos, 1, 64), up_t = __shfl_up(W.tag, 1, 64);
        const float up_v = __shfl_up(W.val, 1, 64);
        if (lane > j + 1 && lane <= i) { W.pos = up_p + 1; W.val = up_v; W.tag = up_t; }
        if (lane == j + 1) { W.pos = np; W.val = v; W.tag = t; }
    }
    return 0;
}
#endif

}  // namespace t5g
