// mev_nsort.h — the neighbour order of get_observations: std::sort by distance.
//
// The reference collects, for ego i, every other alive ego (index order) and then
// every alive NPC (cpp/IntersectionEnv.cpp:466-488) and sorts them with
// std::sort(..., a.dist < b.dist) (:490), keeping the first NEIGHBOR_COUNT.
// std::sort is not stable.  With at most 16 candidates libstdc++ runs only its
// insertion sort, which is stable, so the device's stable top-5 equals it.  With
// more, __introsort_loop first partitions the array (median-of-three pivot into
// *first, unguarded Hoare partition, heapsort below 2*lg(n) levels) and the final
// insertion sort then orders that permutation stably: equal distances come out in
// the order the partitions left them, not in push order.  Exact ties are common:
// two cars on one spawn point, or spawn points symmetric to the ego.
//
// This header restates the GCC 11 libstdc++ algorithm this image's reference build
// links (bits/stl_algo.h __sort, __introsort_loop, __unguarded_partition_pivot,
// __move_median_to_first, __unguarded_partition; bits/stl_heap.h __make_heap,
// __adjust_heap, __push_heap, __pop_heap, __sort_heap) over an accessor, so that
// the same code runs on the host (tests/native/nsort_check.cpp compares it with
// std::sort itself) and on the device, where the array lives in a wave's lanes and
// every index is wave-uniform (obs_exact_neighbours in mev_kernels.hip).
//
// Only the first NEIGHBOR_COUNT entries are needed.  They are the first five of the
// stable order of the partitioned array P (the final insertion sort is stable), and
// only elements no farther than the fifth-smallest distance `dlim` can be among
// them.  A right part [cut, last) holds only elements >= its pivot, so when the
// pivot exceeds dlim the part holds none of them and is not partitioned further:
// the positions of the elements that matter are the ones the full sort leaves.
#pragma once

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define MEV_NS_HD __host__ __device__ __forceinline__
#else
#define MEV_NS_HD static inline
#endif

namespace mev {

struct NRef {
    float d;
    int id;
};

// Acc: NRef get(int) const; void set(int, NRef).  Stack: void push(int); int pop(); int size().
template <class Acc>
MEV_NS_HD void ns_swap(Acc& a, int i, int j) {
    const NRef t = a.get(i);
    a.set(i, a.get(j));
    a.set(j, t);
}

// __push_heap over [f, ...): hole / top relative to f
template <class Acc>
MEV_NS_HD void ns_push_heap(Acc& a, int f, int hole, int top, NRef v) {
    int parent = (hole - 1) / 2;
    while (hole > top && a.get(f + parent).d < v.d) {
        a.set(f + hole, a.get(f + parent));
        hole = parent;
        parent = (hole - 1) / 2;
    }
    a.set(f + hole, v);
}

// __adjust_heap
template <class Acc>
MEV_NS_HD void ns_adjust_heap(Acc& a, int f, int hole, int len, NRef v) {
    const int top = hole;
    int sc = hole;
    while (sc < (len - 1) / 2) {
        sc = 2 * (sc + 1);
        if (a.get(f + sc).d < a.get(f + sc - 1).d) sc--;
        a.set(f + hole, a.get(f + sc));
        hole = sc;
    }
    if ((len & 1) == 0 && sc == (len - 2) / 2) {
        sc = 2 * (sc + 1);
        a.set(f + hole, a.get(f + sc - 1));
        hole = sc - 1;
    }
    ns_push_heap(a, f, hole, top, v);
}

// __partial_sort(first, last, last): __make_heap (__heap_select's loop is empty) + __sort_heap
template <class Acc>
MEV_NS_HD void ns_heapsort(Acc& a, int f, int len) {
#ifdef MEV_NS_COUNT_HEAP
    ++MEV_NS_COUNT_HEAP;  // host test hook (tests/native/nsort_check.cpp)
#endif
    // one loop, one __adjust_heap site (the device inlines it once): steps t < m are
    // __make_heap's (parent = m - 1 - t, down to 0), the rest __sort_heap's pops
    // (l = len - 1 - (t - m), down to 1)
    const int m = len >= 2 ? (len - 2) / 2 + 1 : 0;
    const int steps = m + (len > 1 ? len - 1 : 0);
    for (int t = 0; t < steps; ++t) {
        int hole, hlen;
        NRef v;
        if (t < m) {
            hole = m - 1 - t;
            hlen = len;
            v = a.get(f + hole);
        } else {
            const int l = len - 1 - (t - m);
            v = a.get(f + l);
            a.set(f + l, a.get(f));
            hole = 0;
            hlen = l;
        }
        ns_adjust_heap(a, f, hole, hlen, v);
    }
}

// __unguarded_partition_pivot(first, last): returns the cut; *pivot_d = the pivot's distance
template <class Acc>
MEV_NS_HD int ns_partition(Acc& a, int first, int last, float* pivot_d) {
    const int ia = first + 1, ib = first + (last - first) / 2, ic = last - 1;
    const float da = a.get(ia).d, db = a.get(ib).d, dc = a.get(ic).d;
    int m;  // __move_median_to_first
    if (da < db) m = db < dc ? ib : (da < dc ? ic : ia);
    else m = da < dc ? ia : (db < dc ? ic : ib);
    ns_swap(a, first, m);
    const float pv = a.get(first).d;
    int lo = first + 1, hi = last;  // __unguarded_partition(first + 1, last, first)
    for (;;) {
        while (a.get(lo).d < pv) ++lo;
        --hi;
        while (pv < a.get(hi).d) --hi;
        if (!(lo < hi)) break;
        ns_swap(a, lo, hi);
        ++lo;
    }
    *pivot_d = pv;
    return lo;
}

MEV_NS_HD int ns_lg(int n) {  // std::__lg
    int lg = 0;
    while ((2 << lg) <= n) ++lg;
    return lg;
}

// __introsort_loop(0, n, 2 lg n).  The reference recurses into the right part and loops
// on the left; the parts are disjoint, so the order they are worked in does not change
// the result.  Pending right parts go to `st` as first | last << 8 | depth << 16.
// Right parts whose pivot exceeds dlim are skipped (header comment; dlim = +inf: the
// whole sort).
template <class Acc, class Stack>
MEV_NS_HD void ns_introsort(Acc& a, int n, float dlim, Stack& st) {
    int first = 0, last = n, depth = 2 * ns_lg(n);
    for (;;) {
        while (last - first > 16) {
            if (depth == 0) {
                ns_heapsort(a, first, last - first);
                break;
            }
            --depth;
            float pv;
            const int cut = ns_partition(a, first, last, &pv);
            if (!(dlim < pv)) st.push(cut | (last << 8) | (depth << 16));
            last = cut;
        }
        if (st.size() == 0) break;
        const int w = st.pop();
        first = w & 0xff;
        last = (w >> 8) & 0xff;
        depth = w >> 16;
    }
}

// The first `k` (<= 5) of the stable order of P[0, n) by distance: ids into out[].
template <class Acc>
MEV_NS_HD int ns_stable_top(const Acc& a, int n, int k, int* out) {
    float bd[5];
    int nb = 0;
    for (int p = 0; p < n; ++p) {
        const NRef r = a.get(p);
        int pos = nb;
        while (pos > 0 && r.d < bd[pos - 1]) --pos;
        if (pos >= k) continue;
        const int lastq = nb < k ? nb : k - 1;
        for (int q = lastq; q > pos; --q) { bd[q] = bd[q - 1]; out[q] = out[q - 1]; }
        bd[pos] = r.d;
        out[pos] = r.id;
        if (nb < k) ++nb;
    }
    return nb;
}

}  // namespace mev
