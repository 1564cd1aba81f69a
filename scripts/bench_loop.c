/* The C2 bench's caller loop in C: what laserMapping does per scan around
 * the IKF update (laserMapping.cpp:772-774 -- a C++ call of
 * update_iterated_dyn_share_modified with the state and covariance the
 * filter carries), here `steps` updates from the same prior (x0, P0: the
 * same work every step), each through the product's C ABI
 * (slio_ikf_update_device, include/slio.h).  bench.py times this loop; the
 * Python loop it replaces added ~2.8 us of interpreter and ctypes overhead
 * per update (profiles/r05a_hostgap.json: py_return -> next_py_call 1.29 us,
 * py_call -> entry 1.48 us) that a compiled caller does not have.
 *
 * Built by __graft_entry__.build() / bench.py into scripts/libbench_loop.so;
 * the update function is passed in by address (libslio.so is loaded by
 * ctypes with local symbol binding). */
#include <stdint.h>
#include <string.h>

#include "slio.h"

typedef int (*update_fn)(slio_handle, slio_state*, double*, double, int, int, int, slio_allreduce_fn, void*,
                         slio_ikf_stats*);

int bench_c2_loop(update_fn fn, slio_handle h, const slio_state* x0, const double* P0, double R, int maxit,
                  int ext, int mode, slio_allreduce_fn reduce, void* reduce_ctx, int64_t steps, slio_state* x,
                  double* P, slio_ikf_stats* stats) {
  for (int64_t k = 0; k < steps; ++k) {
    *x = *x0;
    memcpy(P, P0, sizeof(double) * 576);
    const int rc = fn(h, x, P, R, maxit, ext, mode, reduce, reduce_ctx, stats);
    if (rc) return rc;
  }
  return 0;
}
