// Deterministic selection/heap primitives shared by host and device code.
//
// The reference's keypoint order is defined by std::nth_element inside
// cv::KeyPointsFilter::retainBest (ORBextractor.cc:734, :750) and its
// active-matching heap by std::priority_queue (Observability.cc:1325). Both are
// order-dependent under ties (FAST scores are small integers), so the device
// runs a faithful port of the libstdc++ algorithms (introselect with
// median-of-three pivot, unguarded Hoare partition, heap_select fallback,
// insertion sort; binary heap sift-up/sift-down) instead of a GPU sort.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define GF_HD __host__ __device__ __forceinline__
#else
#define GF_HD inline
#endif

namespace gfsel {

// Keypoint record packed as score<<24 | y<<12 | x; comparator of retainBest is
// KeypointResponseGreater (response == FAST score).
struct RespGreater {
    GF_HD bool operator()(uint32_t a, uint32_t b) const { return (a >> 24) > (b >> 24); }
};

template <class T>
GF_HD void swap_(T& a, T& b) {
    T t = a;
    a = b;
    b = t;
}

GF_HD int lg_(int n) { return 31 - __builtin_clz((unsigned)n); }

template <class T, class C>
GF_HD void push_heap_hole(T* a, int hole, int top, T value, C comp) {
    int parent = (hole - 1) / 2;
    while (hole > top && comp(a[parent], value)) {
        a[hole] = a[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    a[hole] = value;
}

template <class T, class C>
GF_HD void adjust_heap(T* a, int hole, int len, T value, C comp) {
    const int top = hole;
    int second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (comp(a[second], a[second - 1])) second--;
        a[hole] = a[second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        a[hole] = a[second - 1];
        hole = second - 1;
    }
    push_heap_hole(a, hole, top, value, comp);
}

template <class T, class C>
GF_HD void make_heap(T* a, int len, C comp) {
    if (len < 2) return;
    int parent = (len - 2) / 2;
    while (true) {
        T v = a[parent];
        adjust_heap(a, parent, len, v, comp);
        if (parent == 0) return;
        parent--;
    }
}

// std::push_heap on [0, len) where the new element already sits at a[len-1].
template <class T, class C>
GF_HD void push_heap(T* a, int len, C comp) {
    T v = a[len - 1];
    push_heap_hole(a, len - 1, 0, v, comp);
}

// std::pop_heap on [0, len): moves the top to a[len-1].
template <class T, class C>
GF_HD void pop_heap(T* a, int len, C comp) {
    if (len > 1) {
        T v = a[len - 1];
        a[len - 1] = a[0];
        adjust_heap(a, 0, len - 1, v, comp);
    }
}

template <class T, class C>
GF_HD void heap_select(T* a, int first, int middle, int last, C comp) {
    make_heap(a + first, middle - first, comp);
    for (int i = middle; i < last; ++i)
        if (comp(a[i], a[first])) {
            // __pop_heap(first, middle, i)
            T v = a[i];
            a[i] = a[first];
            adjust_heap(a + first, 0, middle - first, v, comp);
        }
}

template <class T, class C>
GF_HD void move_median_to_first(T* a, int result, int x, int y, int z, C comp) {
    if (comp(a[x], a[y])) {
        if (comp(a[y], a[z]))
            swap_(a[result], a[y]);
        else if (comp(a[x], a[z]))
            swap_(a[result], a[z]);
        else
            swap_(a[result], a[x]);
    } else if (comp(a[x], a[z]))
        swap_(a[result], a[x]);
    else if (comp(a[y], a[z]))
        swap_(a[result], a[z]);
    else
        swap_(a[result], a[y]);
}

template <class T, class C>
GF_HD int unguarded_partition(T* a, int first, int last, int pivot, C comp) {
    while (true) {
        while (comp(a[first], a[pivot])) ++first;
        --last;
        while (comp(a[pivot], a[last])) --last;
        if (!(first < last)) return first;
        swap_(a[first], a[last]);
        ++first;
    }
}

template <class T, class C>
GF_HD void insertion_sort(T* a, int first, int last, C comp) {
    if (first == last) return;
    for (int i = first + 1; i != last; ++i) {
        if (comp(a[i], a[first])) {
            T v = a[i];
            for (int k = i; k > first; --k) a[k] = a[k - 1];
            a[first] = v;
        } else {
            T v = a[i];
            int j = i, nx = i - 1;
            while (comp(v, a[nx])) {
                a[j] = a[nx];
                j = nx;
                --nx;
            }
            a[j] = v;
        }
    }
}

// std::nth_element(a+first, a+nth, a+last, comp) — libstdc++ __introselect.
template <class T, class C>
GF_HD void nth_element(T* a, int first, int nth, int last, C comp) {
    if (first == last || nth == last) return;
    int depth = 2 * lg_(last - first);
    while (last - first > 3) {
        if (depth == 0) {
            heap_select(a, first, nth + 1, last, comp);
            swap_(a[first], a[nth]);
            return;
        }
        --depth;
        int mid = first + (last - first) / 2;
        move_median_to_first(a, first, first + 1, mid, last - 1, comp);
        int cut = unguarded_partition(a, first + 1, last, first, comp);
        if (cut <= nth)
            first = cut;
        else
            last = cut;
    }
    insertion_sort(a, first, last, comp);
}

// KeyPointsFilter::retainBest + truncation to n (ORBextractor.cc:734-736):
// the first n entries after nth_element(begin, begin + n - 1, end).
// Returns the retained count.
template <class T, class C>
GF_HD int retain_best_truncate(T* a, int size, int n, C comp) {
    if (n < 0 || size <= n) return size;
    if (n == 0) return 0;
    nth_element(a, 0, n - 1, size, comp);
    return n;
}

}  // namespace gfsel
