// stl_sort.hpp -- bit-for-bit restatement of GCC 11 libstdc++ std::sort
// (introsort: bits/stl_algo.h __introsort_loop / __final_insertion_sort and
// bits/stl_heap.h) for host and device.
//
// Why: the reference orders candidate paths with std::sort on an index array
// (mink, src/SCLLUTDecoder.cpp:8-21; argsort, src/FastSCLLUTDecoder.cpp:7-17).
// std::sort is not stable above 16 elements, so with the frequent ties of
// quantized LLR magnitudes the survivor order -- and therefore the decoded
// bits -- depends on the exact introsort steps (SURVEY.md §8(a) hazard H1).
// The FastSCL-LUT R1 node sorts 32 magnitudes at N=1024, so the device must
// replay those steps exactly.  tests/test_stl_sort.py checks this file against
// std::sort itself on tie-heavy inputs.
//
// `Seq` supplies: int get(int p); void set(int p, int e); bool less(int e1, int e2)
// where elements are int indices and less() compares their keys.
#pragma once

#if defined(__HIPCC__)
#define QPD_HD __host__ __device__ __forceinline__
#else
#define QPD_HD inline
#endif

namespace qpd {
namespace stl {

constexpr int kThreshold = 16;  // _S_threshold

QPD_HD int lg(int n) {  // std::__lg: floor(log2(n)), n > 0
    int r = 0;
    while (n >>= 1) ++r;
    return r;
}

template <class Seq>
QPD_HD void push_heap(Seq &s, int first, int hole, int top, int value) {
    int parent = (hole - 1) / 2;
    while (hole > top && s.less(s.get(first + parent), value)) {
        s.set(first + hole, s.get(first + parent));
        hole = parent;
        parent = (hole - 1) / 2;
    }
    s.set(first + hole, value);
}

template <class Seq>
QPD_HD void adjust_heap(Seq &s, int first, int hole, int len, int value) {
    const int top = hole;
    int child = hole;
    while (child < (len - 1) / 2) {
        child = 2 * (child + 1);
        if (s.less(s.get(first + child), s.get(first + child - 1))) --child;
        s.set(first + hole, s.get(first + child));
        hole = child;
    }
    if ((len & 1) == 0 && child == (len - 2) / 2) {
        child = 2 * (child + 1);
        s.set(first + hole, s.get(first + child - 1));
        hole = child - 1;
    }
    push_heap(s, first, hole, top, value);
}

template <class Seq>
QPD_HD void make_heap(Seq &s, int first, int last) {
    const int len = last - first;
    if (len < 2) return;
    int parent = (len - 2) / 2;
    while (true) {
        int value = s.get(first + parent);
        adjust_heap(s, first, parent, len, value);
        if (parent == 0) return;
        --parent;
    }
}

template <class Seq>
QPD_HD void pop_heap(Seq &s, int first, int last, int result) {
    int value = s.get(result);
    s.set(result, s.get(first));
    adjust_heap(s, first, 0, last - first, value);
}

// __partial_sort(first, last, last): heap_select then sort_heap.
template <class Seq>
QPD_HD void heap_sort(Seq &s, int first, int last) {
    make_heap(s, first, last);
    // heap_select's scan of [middle, last) is empty when middle == last.
    while (last - first > 1) {
        --last;
        pop_heap(s, first, last, last);
    }
}

template <class Seq>
QPD_HD void move_median_to_first(Seq &s, int result, int a, int b, int c) {
    const int ea = s.get(a), eb = s.get(b), ec = s.get(c);
    int pick;
    if (s.less(ea, eb)) {
        if (s.less(eb, ec)) pick = b;
        else if (s.less(ea, ec)) pick = c;
        else pick = a;
    } else if (s.less(ea, ec)) {
        pick = a;
    } else if (s.less(eb, ec)) {
        pick = c;
    } else {
        pick = b;
    }
    const int er = s.get(result), ep = s.get(pick);
    s.set(result, ep);
    s.set(pick, er);
}

template <class Seq>
QPD_HD int unguarded_partition(Seq &s, int first, int last, int pivot) {
    const int pv = s.get(pivot);
    while (true) {
        while (s.less(s.get(first), pv)) ++first;
        --last;
        while (s.less(pv, s.get(last))) --last;
        if (!(first < last)) return first;
        const int t = s.get(first);
        s.set(first, s.get(last));
        s.set(last, t);
        ++first;
    }
}

template <class Seq>
QPD_HD void unguarded_linear_insert(Seq &s, int last) {
    const int val = s.get(last);
    int next = last - 1;
    while (s.less(val, s.get(next))) {
        s.set(last, s.get(next));
        last = next;
        --next;
    }
    s.set(last, val);
}

template <class Seq>
QPD_HD void insertion_sort(Seq &s, int first, int last) {
    if (first == last) return;
    for (int i = first + 1; i != last; ++i) {
        const int val = s.get(i);
        if (s.less(val, s.get(first))) {
            for (int k = i; k > first; --k) s.set(k, s.get(k - 1));  // move_backward
            s.set(first, val);
        } else {
            unguarded_linear_insert(s, i);
        }
    }
}

template <class Seq>
QPD_HD void final_insertion_sort(Seq &s, int first, int last) {
    if (last - first > kThreshold) {
        insertion_sort(s, first, first + kThreshold);
        for (int i = first + kThreshold; i != last; ++i) unguarded_linear_insert(s, i);
    } else {
        insertion_sort(s, first, last);
    }
}

// __introsort_loop with its tail recursion on the right part turned into an
// explicit stack (at most 2*lg(n)+1 <= 33 pending ranges for n < 2^16).
template <class Seq>
QPD_HD void introsort_loop(Seq &s, int first, int last, int depth_limit) {
    int st_first[40], st_last[40], st_depth[40];
    int sp = 0;
    st_first[sp] = first;
    st_last[sp] = last;
    st_depth[sp] = depth_limit;
    ++sp;
    while (sp > 0) {
        --sp;
        int f = st_first[sp], l = st_last[sp], dl = st_depth[sp];
        while (l - f > kThreshold) {
            if (dl == 0) {
                heap_sort(s, f, l);
                break;
            }
            --dl;
            const int mid = f + (l - f) / 2;
            move_median_to_first(s, f, f + 1, mid, l - 1);
            const int cut = unguarded_partition(s, f + 1, l, f);
            // The reference recurses on [cut, l) first, then loops on [f, cut).
            // Both halves are disjoint, so evaluating [f, cut) after [cut, l)
            // (stack order below) gives the same final array.
            st_first[sp] = f;
            st_last[sp] = cut;
            st_depth[sp] = dl;
            ++sp;
            f = cut;
        }
    }
}

// std::sort for last - first <= 2 * kThreshold + 1: a partition of a range
// of at most 33 elements leaves at most one side above the threshold, so the
// recursion of __introsort_loop degenerates into a loop and needs no stack
// (same steps, same final array as sort()).
template <class Seq>
QPD_HD void sort_small(Seq &s, int first, int last) {
    if (first == last) return;
    int f = first, l = last, dl = lg(last - first) * 2;
    while (l - f > kThreshold) {
        if (dl == 0) {
            heap_sort(s, f, l);
            break;
        }
        --dl;
        const int mid = f + (l - f) / 2;
        move_median_to_first(s, f, f + 1, mid, l - 1);
        const int cut = unguarded_partition(s, f + 1, l, f);
        if (l - cut > kThreshold)
            f = cut;  // the reference's recursion on [cut, l); [f, cut) is then too short to touch
        else
            l = cut;  // the reference's loop on [f, cut); [cut, l) was too short to touch
    }
    final_insertion_sort(s, first, last);
}

// sort_small when only the first m outputs are read (the R1 node's m = min(L-1,
// temp) survivor layers): the same steps, minus those that cannot reach them.
// A partition leaves [first, cut) <= pivot <= [cut, last), and no later step
// moves an element of a right block before an element of a left block (the
// guarded insertion's `val < *first` and the unguarded insertion's
// `val < *prev` are false across such a boundary).  So once a block boundary c
// with c - first >= m is known, the order of [first, c) is final-insertion-sort
// of [first, c) alone: the right part's partitioning and its insertions are
// skipped.  Positions >= c of the array are left unsorted.
//
// partition_prefix runs the partitioning part and returns that end; the final
// insertion sort of [first, end) is then a STABLE sort of the block as the
// partitions left it (insertion_sort and unguarded_linear_insert move an
// element only past strictly greater keys), so its first m outputs are the m
// smallest entries by (key, position in the block) -- which the device finds
// with packed min trees instead of the O(n^2) insertions (r1_prep).
template <class Seq>
QPD_HD int partition_prefix(Seq &s, int first, int last, int m) {
    int f = first, l = last, dl = lg(last - first) * 2, end = last;
    while (l - f > kThreshold) {
        if (dl == 0) {
            heap_sort(s, f, l);
            break;
        }
        --dl;
        const int mid = f + (l - f) / 2;
        move_median_to_first(s, f, f + 1, mid, l - 1);
        const int cut = unguarded_partition(s, f + 1, l, f);
        if (cut - first >= m && cut < end) end = cut;  // a block boundary past the needed prefix
        if (l - cut > kThreshold) {
            if (cut >= end) break;  // the reference's recursion on [cut, l) lies past the prefix
            f = cut;
        } else {
            l = cut;
        }
    }
    return end;
}

template <class Seq>
QPD_HD void sort_small_prefix(Seq &s, int first, int last, int m) {
    if (first == last) return;
    final_insertion_sort(s, first, partition_prefix(s, first, last, m));
}

template <class Seq>
QPD_HD void sort(Seq &s, int first, int last) {
    if (first == last) return;
    introsort_loop(s, first, last, lg(last - first) * 2);
    final_insertion_sort(s, first, last);
}

}  // namespace stl
}  // namespace qpd
