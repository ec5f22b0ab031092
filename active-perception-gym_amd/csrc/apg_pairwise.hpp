// apg_pairwise.hpp — numpy's pairwise summation restated for device code.
//
// numpy reduces a contiguous float32 run with loops_utils.h.src pairwise_sum (PW_BLOCKSIZE 128):
// runs < 8 are summed in order; runs <= 128 use 8 strided accumulators combined as
// ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) plus an in-order tail; longer runs split at n/2 rounded down
// to a multiple of 8.  np.sum / np.mean over such a run return (0 + pairwise_sum) [/ n].
#pragma once
#include "apg_device.hpp"

namespace apg {

// numpy loops_utils.h.src pairwise_sum (PW_BLOCKSIZE 128) over n values x(i), f32 accumulators.
// The leaf is kept out of line: the recursion below expands into one call per leaf.
template <class F>
__device__ __noinline__ float pw_leaf(const F &x, int off, int n) {
  if (n < 8) {
    float r = 0.0f;
    for (int i = 0; i < n; i++) r = __fadd_rn(r, x(off + i));
    return r;
  }
  float r0 = x(off), r1 = x(off + 1), r2 = x(off + 2), r3 = x(off + 3);
  float r4 = x(off + 4), r5 = x(off + 5), r6 = x(off + 6), r7 = x(off + 7);
  int i = 8;
  for (; i < n - (n % 8); i += 8) {
    r0 = __fadd_rn(r0, x(off + i));
    r1 = __fadd_rn(r1, x(off + i + 1));
    r2 = __fadd_rn(r2, x(off + i + 2));
    r3 = __fadd_rn(r3, x(off + i + 3));
    r4 = __fadd_rn(r4, x(off + i + 4));
    r5 = __fadd_rn(r5, x(off + i + 5));
    r6 = __fadd_rn(r6, x(off + i + 6));
    r7 = __fadd_rn(r7, x(off + i + 7));
  }
  float res = __fadd_rn(__fadd_rn(__fadd_rn(r0, r1), __fadd_rn(r2, r3)), __fadd_rn(__fadd_rn(r4, r5), __fadd_rn(r6, r7)));
  for (; i < n; i++) res = __fadd_rn(res, x(off + i));
  return res;
}

template <int DEPTH, class F>
APG_DEV float pw_sum(const F &x, int off, int n) {
  if constexpr (DEPTH == 0) {
    return pw_leaf(x, off, n);  // callers keep n <= 128 << MAX_PW_DEPTH
  } else {
    if (n <= 128) return pw_leaf(x, off, n);
    int n2 = n / 2;
    n2 -= n2 % 8;
    return __fadd_rn(pw_sum<DEPTH - 1>(x, off, n2), pw_sum<DEPTH - 1>(x, off + n2, n - n2));
  }
}
constexpr int MAX_PW_DEPTH = 7;  // n <= 128 * 2^7 = 16384 summands
constexpr int MAX_PW_N = 128 << MAX_PW_DEPTH;


// The same sum over an array with element stride `st` (contiguous: st = 1), without function calls (a
// call in a kernel makes the compiler budget registers for the callee's ABI and can cut the
// occupancy of the whole kernel).
APG_DEV float pw_leaf_ptr(const float *x, int n, size_t st = 1) {
  if (n < 8) {
    float r = 0.0f;
    for (int i = 0; i < n; i++) r = __fadd_rn(r, x[i * st]);
    return r;
  }
  float r0 = x[0], r1 = x[st], r2 = x[2 * st], r3 = x[3 * st], r4 = x[4 * st], r5 = x[5 * st], r6 = x[6 * st],
        r7 = x[7 * st];
  int i = 8;
  for (; i < n - (n % 8); i += 8) {
    r0 = __fadd_rn(r0, x[i * st]);
    r1 = __fadd_rn(r1, x[(i + 1) * st]);
    r2 = __fadd_rn(r2, x[(i + 2) * st]);
    r3 = __fadd_rn(r3, x[(i + 3) * st]);
    r4 = __fadd_rn(r4, x[(i + 4) * st]);
    r5 = __fadd_rn(r5, x[(i + 5) * st]);
    r6 = __fadd_rn(r6, x[(i + 6) * st]);
    r7 = __fadd_rn(r7, x[(i + 7) * st]);
  }
  float res = __fadd_rn(__fadd_rn(__fadd_rn(r0, r1), __fadd_rn(r2, r3)), __fadd_rn(__fadd_rn(r4, r5), __fadd_rn(r6, r7)));
  for (; i < n; i++) res = __fadd_rn(res, x[i * st]);
  return res;
}

template <int DEPTH>
APG_DEV float pw_sum_ptr_d(const float *x, int n, size_t st) {
  if constexpr (DEPTH == 0) {
    return pw_leaf_ptr(x, n, st);
  } else {
    if (n <= 128) return pw_leaf_ptr(x, n, st);
    int n2 = n / 2;
    n2 -= n2 % 8;
    return __fadd_rn(pw_sum_ptr_d<DEPTH - 1>(x, n2, st), pw_sum_ptr_d<DEPTH - 1>(x + n2 * st, n - n2, st));
  }
}

// Call-free pairwise sum of n <= PW_PTR_MAX_N values (three split levels, eight inline leaves).
constexpr int PW_PTR_MAX_N = 968;  // three split levels leave every leaf <= 128 up to here
APG_DEV float pw_sum_ptr(const float *x, int n, size_t st = 1) { return pw_sum_ptr_d<3>(x, n, st); }
// The same for n <= PW_DEEP_MAX_N (seven levels, 128 inline leaves: for the kernels of long episodes only)
constexpr int PW_DEEP_MAX_N = 15368;
APG_DEV float pw_sum_ptr_deep(const float *x, int n, size_t st = 1) { return pw_sum_ptr_d<7>(x, n, st); }

}  // namespace apg
