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

}  // namespace t5g
