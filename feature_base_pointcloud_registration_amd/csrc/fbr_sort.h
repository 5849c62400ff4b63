// fbr_sort.h — exact single-lane emulation of libstdc++ 11 std::sort for the smoothness segments.
//
// featureExtraction.h:203 sorts cloudSmoothness[sp, ep) by curvature with std::sort, which is
// unstable: for equal curvatures the visit order of the corner/surf picks (and hence the feature
// masks) depends on libstdc++'s introsort.  Segments without ties (the common case) are sorted by
// the parallel rank sort in k_features.hip, which gives the same unique order; segments with ties
// (or NaNs) run this restatement of /usr/include/c++/11/bits/stl_algo.h (__introsort_loop,
// __unguarded_partition_pivot, __move_median_to_first, __final_insertion_sort, threshold 16,
// depth 2*floor(log2 n)) and stl_heap.h (__make_heap/__adjust_heap/__push_heap/__pop_heap) on LDS.
// tests/test_sort_emulation.py checks it against the host std::sort.
#pragma once
#include <hip/hip_runtime.h>

namespace fbr {

struct SmoothEntry {
  float v;
  int ind;
};

__host__ __device__ inline bool sm_lt(const SmoothEntry& a, const SmoothEntry& b) { return a.v < b.v; }
__host__ __device__ inline void sm_swap(SmoothEntry* a, int i, int j) {
  SmoothEntry t = a[i];
  a[i] = a[j];
  a[j] = t;
}

__host__ __device__ inline void sm_move_median_to_first(SmoothEntry* a, int result, int x, int y, int z) {
  if (sm_lt(a[x], a[y])) {
    if (sm_lt(a[y], a[z])) sm_swap(a, result, y);
    else if (sm_lt(a[x], a[z])) sm_swap(a, result, z);
    else sm_swap(a, result, x);
  } else if (sm_lt(a[x], a[z])) {
    sm_swap(a, result, x);
  } else if (sm_lt(a[y], a[z])) {
    sm_swap(a, result, z);
  } else {
    sm_swap(a, result, y);
  }
}

__host__ __device__ inline int sm_unguarded_partition(SmoothEntry* a, int first, int last, int pivot) {
  while (true) {
    while (sm_lt(a[first], a[pivot])) ++first;
    --last;
    while (sm_lt(a[pivot], a[last])) --last;
    if (!(first < last)) return first;
    sm_swap(a, first, last);
    ++first;
  }
}

// __adjust_heap on a[first .. first+len) with hole at holeIndex, inserting value.
__host__ __device__ inline void sm_adjust_heap(SmoothEntry* a, int first, long holeIndex, long len, SmoothEntry value) {
  const long topIndex = holeIndex;
  long secondChild = holeIndex;
  while (secondChild < (len - 1) / 2) {
    secondChild = 2 * (secondChild + 1);
    if (sm_lt(a[first + secondChild], a[first + secondChild - 1])) secondChild--;
    a[first + holeIndex] = a[first + secondChild];
    holeIndex = secondChild;
  }
  if ((len & 1) == 0 && secondChild == (len - 2) / 2) {
    secondChild = 2 * (secondChild + 1);
    a[first + holeIndex] = a[first + secondChild - 1];
    holeIndex = secondChild - 1;
  }
  // __push_heap
  long parent = (holeIndex - 1) / 2;
  while (holeIndex > topIndex && sm_lt(a[first + parent], value)) {
    a[first + holeIndex] = a[first + parent];
    holeIndex = parent;
    parent = (holeIndex - 1) / 2;
  }
  a[first + holeIndex] = value;
}

__host__ __device__ inline void sm_heap_sort(SmoothEntry* a, int first, int last) {
  const long len = last - first;
  if (len >= 2) {  // __make_heap
    long parent = (len - 2) / 2;
    while (true) {
      SmoothEntry value = a[first + parent];
      sm_adjust_heap(a, first, parent, len, value);
      if (parent == 0) break;
      parent--;
    }
  }
  while (last - first > 1) {  // __sort_heap
    --last;
    SmoothEntry value = a[last];  // __pop_heap(first, last, last)
    a[last] = a[first];
    sm_adjust_heap(a, first, 0, last - first, value);
  }
}

__host__ __device__ inline void sm_unguarded_linear_insert(SmoothEntry* a, int last) {
  SmoothEntry val = a[last];
  int next = last - 1;
  while (sm_lt(val, a[next])) {
    a[last] = a[next];
    last = next;
    --next;
  }
  a[last] = val;
}

__host__ __device__ inline void sm_insertion_sort(SmoothEntry* a, int first, int last) {
  if (first == last) return;
  for (int i = first + 1; i != last; ++i) {
    if (sm_lt(a[i], a[first])) {
      SmoothEntry val = a[i];
      for (int k = i; k > first; --k) a[k] = a[k - 1];
      a[first] = val;
    } else {
      sm_unguarded_linear_insert(a, i);
    }
  }
}

__host__ __device__ inline int sm_lg(long n) {
  int r = -1;
  while (n) {
    n >>= 1;
    ++r;
  }
  return r;
}

struct SortFrame {
  int first, last, depth;
};
constexpr int kSortStack = 32;  // >= 2*lg(n)+1 pending frames for n < 2^15

// std::sort(a, a + n, by_value()); `stack` holds kSortStack frames (LDS on the device, so the
// dynamically indexed stack does not live in scratch).  Partitions are disjoint, so handling the
// right-hand parts from an explicit stack instead of recursion gives the same array.
__host__ __device__ inline void std_sort_emul(SmoothEntry* a, int n, SortFrame* stack) {
  if (n <= 0) return;
  using Frame = SortFrame;
  int sp = 0;
  stack[sp++] = Frame{0, n, 2 * sm_lg(n)};
  while (sp > 0) {
    Frame f = stack[--sp];
    int first = f.first, last = f.last, depth = f.depth;
    while (last - first > 16) {
      if (depth == 0) {
        sm_heap_sort(a, first, last);
        break;
      }
      --depth;
      int mid = first + (last - first) / 2;
      sm_move_median_to_first(a, first, first + 1, mid, last - 1);
      int cut = sm_unguarded_partition(a, first + 1, last, first);
      if (sp < kSortStack) stack[sp++] = Frame{cut, last, depth};
      last = cut;
    }
  }
  // __final_insertion_sort
  if (n > 16) {
    sm_insertion_sort(a, 0, 16);
    for (int i = 16; i != n; ++i) sm_unguarded_linear_insert(a, i);
  } else {
    sm_insertion_sort(a, 0, n);
  }
}

inline void std_sort_emul(SmoothEntry* a, int n) {  // host convenience
  SortFrame stack[kSortStack];
  std_sort_emul(a, n, stack);
}

}  // namespace fbr
