// slio_common.hpp — internal declarations shared by the device runtime
// (slio_device.hip) and the host IKF driver (slio_ikf.cpp).
#pragma once

#include <cstdint>
#include <string>

#include "../../include/slio.h"

#if defined(__HIPCC__)
#define SLIO_HD __host__ __device__
#else
#define SLIO_HD
#endif

namespace slio {

// thread-local last-error message behind slio_last_error()
void set_error(const std::string& msg);

// Reduction product table: product k accumulates row[pa[k]] * row[pb[k]]
// over the selected points of a pass, where the per-point row is
//   row[0..11] = h_x (esekfom.hpp:217-221), row[12] = h = -pd2 (esekfom.hpp:225),
//   row[13]    = 1 for an effective point (so the product counts m).
// k in [0, 78)  : H^T H upper triangle, row-major (i <= j)
// k in [78, 90) : H^T h
// k == 90       : m
constexpr int kRow = 14;
inline void product_table(uint8_t pa[SLIO_NPROD], uint8_t pb[SLIO_NPROD]) {
  int k = 0;
  for (int i = 0; i < 12; ++i)
    for (int j = i; j < 12; ++j) {
      pa[k] = (uint8_t)i;
      pb[k] = (uint8_t)j;
      ++k;
    }
  for (int i = 0; i < 12; ++i) {
    pa[k] = (uint8_t)i;
    pb[k] = 12;
    ++k;
  }
  pa[k] = 13;
  pb[k] = 13;
}

// Chunk / super-chunk geometry of the fixed summation tree.  The scan of n
// points is cut into C = ceil(n / SLIO_CHUNK) chunks; super-chunk s covers
// chunks [s*C/8, (s+1)*C/8); rank r of N owns super-chunks [r*8/N, (r+1)*8/N).
// The tree (chunk -> super -> total) does not depend on N, so 1/2/4/8 ranks
// produce bitwise-identical sums.
SLIO_HD inline int64_t num_chunks(int64_t n) { return (n + SLIO_CHUNK - 1) / SLIO_CHUNK; }
SLIO_HD inline int64_t super_lo(int64_t C, int s) { return (C * s) / SLIO_NSUPER; }
inline void rank_chunks(int64_t n, int rank, int nranks, int64_t* c0, int64_t* c1) {
  int64_t C = num_chunks(n);
  int per = SLIO_NSUPER / nranks;
  *c0 = super_lo(C, rank * per);
  *c1 = super_lo(C, (rank + 1) * per);
}

// Device-resident IKF control block (slio_ikf_update_device): the filter
// state, covariance and the esekfom.hpp:292-345 control flags live in HBM so
// a whole update runs without host round trips.
struct IkfCtl {
  slio_state x;      // x_ (current iterate)
  slio_state xprop;  // x_propagated
  double P[576];     // P_ (row-major)
  double P11i[144];  // (P[:D, :D])^-1 of P_ (D x D), fixed during an update (host)
  double G[288];     // P[:, :D] P11i (24 x D)                             (host)
  double dxn[24];    // x [-] x_propagated of the current iterate: 0 on the first
                     // pass (host), then written by the pass kernel (device)
  int32_t converge, t, done, search_now;
  int32_t passes, searches, valid_passes, mode;
  int64_t last_m;
  int32_t singular;
  int32_t published;  // mapped host block: set (release, system scope) after x, P and the flags
  int32_t seq;        // the update's sequence number (a fused group's passes and gates check it)
  int32_t timeout;    // mapped host block: set (system scope) by a device-side wait that gave up
  // PoseDev of x (rotation matrices formed) for the pass that follows, in slot
  // (passes completed) % kPoseSlots (device only): a slot is first read by a
  // pass after its writer's step, so a persistent update's scalar-cache loads
  // of it are never stale within the launch
  alignas(128) double pose[16][32];  // (each slot on cache lines of its own)
  double LM[300];    // Cholesky factor of S = P11i + H^T H / R (D x D), H^T H / R
                     // (upper triangle, 78) and 1 / diag of the factor, of the
                     // last valid pass (device only)
};

// P_DD^-1 (D x D) and G = P[:, :D] P_DD^-1 (24 x D) of an update's prior P,
// D = 6 or 12 (slio_ikf.cpp)
bool info_constants(const double* P, int D, double P11i[144], double G[288]);

// Live handles per HIP device (IKF, LIO-SAM and LeGO-LOAM handles; delta +1
// at create, -1 at destroy; returns the count after the change).  The
// persistent update assumes every workgroup of its launch is resident at
// once, which only holds when no other handle's kernels share the device.
int dev_users(int device, int delta);

}  // namespace slio
