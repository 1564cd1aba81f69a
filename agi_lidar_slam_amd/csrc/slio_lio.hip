// slio_lio.hip -- LIO-SAM front-end on gfx950.
//
// One scan = 6 launches on the handle's stream:
//   (no reset of the cell owners: they carry the scan's generation)
//   k_lio_claim   per point        projectPointCloud filters (:614-636); the
//                                  cell goes to the smallest point index
//                                  (atomicMin) = "first point wins" (:638)
//   k_lio_fill    block per ring   rangeMat / fullCloud for the winners, with
//                                  deskewPoint (:565-604) relative to the first
//                                  valid point; per-ring valid counts
//   k_lio_extract block per ring   cloudExtraction (:656-678): ring offsets,
//                                  start/endRingIndex, in-ring stream compaction
//   k_fe_pick     block per (ring, sector)  calculateSmoothness
//                                  (featureExtraction.cpp:108-131) +
//                                  markOccludedPoints (:137-177) of the sector
//                                  in pull form (each flag computed by its
//                                  owner, from LDS), extractFeatures (:183-296):
//                                  the sector's std::sort (bitonic), then
//                                  one wavefront per variant: the greedy edge /
//                                  flat picks (ballot over 64 candidates), once
//                                  per possible prefix of marks from the
//                                  previous sector (0..5 points); a 7th block
//                                  per ring sorts its VoxelGrid order (ring_vsort)
//   k_fe_ring     block per ring   variant chain (exact sequential result),
//                                  labels, corners, surfaceCloudScan, and
//                                  pcl::VoxelGrid (the presorted order, centroids)
//   k_lio_concat  block per ring   ring-ordered cloud_corner / cloud_surface
// Rings are independent in extractFeatures (suppression reaches 5 points, the
// gap between rings' candidate ranges is 10); sectors within a ring interact
// only through the marks a sector leaves on the next one's first <= 5 points
// (see PickVar), so all 6 x 6 (sector, variant) greedy runs go in parallel.
//
// Deterministic choices where the reference is implementation-defined match
// oracle/frontend_oracle.cpp: float trig as correctly
// rounded values (double evaluation), sort ties by point index, smoothness
// entries the reference never initialises are never picked.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "slio_common.hpp"
#include "slio_frontend.h"

namespace slio {
namespace lio {

#define LIO_HIP(call)                                                          \
  do {                                                                         \
    hipError_t e_ = (call);                                                    \
    if (e_ != hipSuccess) {                                                    \
      set_error(std::string(#call) + ": " + hipGetErrorString(e_));            \
      return SLIO_EDEVICE;                                                     \
    }                                                                          \
  } while (0)

constexpr int kMaxImu = 2000;          // queueLength (imageProjection.cpp:35)
constexpr int kCornerPerRing = 6 * 20;  // 6 sectors x 20 corners (featureExtraction.cpp:209)
constexpr int kFlatPerRing = 6 * 4;     // LeGO-LOAM: 6 sectors x 4 flats (featureAssociation.cpp:952)
enum FeatMode { kModeLio = 0, kModeLego = 1 };
constexpr uint32_t kNone = 0xffffffffu;

struct Geo {
  int n_scan, horizon, ds;
  float min_r, max_r;
  float ang_res_x;
  int64_t cells;
};

struct In {
  const float *x, *y, *z, *in;
  const uint16_t* ring;
  const float* time;
  int64_t n;
};

struct Deskew {
  const double *t, *rx, *ry, *rz;
  int cur;  // imuPointerCur
  double t0;  // timeScanCur
  int on;
  int sorted;  // imuTime non-decreasing: findRotation's scan is a binary search
};

// ---------------------------------------------------------------- math
__device__ __forceinline__ float fcos(float a) { return (float)cos((double)a); }
__device__ __forceinline__ float fsin(float a) { return (float)sin((double)a); }
__device__ __forceinline__ float fatan2(float y, float x) { return (float)atan2((double)y, (double)x); }

struct Aff {
  float m[3][4];
};

// pcl::getTransformation(0, 0, 0, roll, pitch, yaw) (pcl/common/impl/eigen.hpp)
__device__ Aff get_rot(float roll, float pitch, float yaw) {
  const float A = fcos(yaw), B = fsin(yaw), C = fcos(pitch), D = fsin(pitch), E = fcos(roll),
              F = fsin(roll), DE = D * E, DF = D * F;
  Aff t;
  t.m[0][0] = A * C;
  t.m[0][1] = A * DF - B * E;
  t.m[0][2] = B * F + A * DE;
  t.m[0][3] = 0.0f;
  t.m[1][0] = B * C;
  t.m[1][1] = A * E + B * DF;
  t.m[1][2] = B * DE - A * F;
  t.m[1][3] = 0.0f;
  t.m[2][0] = -D;
  t.m[2][1] = C * F;
  t.m[2][2] = C * E;
  t.m[2][3] = 0.0f;
  return t;
}

__device__ __forceinline__ float cof(const Aff& a, int i1, int i2, int j1, int j2) {
  return a.m[i1][j1] * a.m[i2][j2] - a.m[i1][j2] * a.m[i2][j1];
}

// Eigen Transform<float,3,Affine>::inverse(): 3x3 cofactor inverse, t' = -(R^-1 t)
__device__ Aff inverse(const Aff& a) {
  // cofactor_3x3<i, j>: i1 = (i+1)%3, i2 = (i+2)%3, j1 = (j+1)%3, j2 = (j+2)%3
  const float c00 = cof(a, 1, 2, 1, 2), c10 = cof(a, 2, 0, 1, 2), c20 = cof(a, 0, 1, 1, 2);
  const float det = (c00 * a.m[0][0] + c10 * a.m[1][0]) + c20 * a.m[2][0];
  const float invdet = 1.0f / det;
  Aff r;
  r.m[0][0] = c00 * invdet;
  r.m[0][1] = c10 * invdet;
  r.m[0][2] = c20 * invdet;
  r.m[1][0] = cof(a, 1, 2, 2, 0) * invdet;  // cofactor<0,1>
  r.m[1][1] = cof(a, 2, 0, 2, 0) * invdet;  // cofactor<1,1>
  r.m[1][2] = cof(a, 0, 1, 2, 0) * invdet;  // cofactor<2,1>
  r.m[2][0] = cof(a, 1, 2, 0, 1) * invdet;  // cofactor<0,2>
  r.m[2][1] = cof(a, 2, 0, 0, 1) * invdet;  // cofactor<1,2>
  r.m[2][2] = cof(a, 0, 1, 0, 1) * invdet;  // cofactor<2,2>
#pragma unroll
  for (int i = 0; i < 3; ++i)
    r.m[i][3] = -((r.m[i][0] * a.m[0][3] + r.m[i][1] * a.m[1][3]) + r.m[i][2] * a.m[2][3]);
  return r;
}

__device__ Aff compose(const Aff& l, const Aff& r) {
  Aff o;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int j = 0; j < 3; ++j)
      o.m[i][j] = (l.m[i][0] * r.m[0][j] + l.m[i][1] * r.m[1][j]) + l.m[i][2] * r.m[2][j];
    o.m[i][3] = ((l.m[i][0] * r.m[0][3] + l.m[i][1] * r.m[1][3]) + l.m[i][2] * r.m[2][3]) + l.m[i][3];
  }
  return o;
}

// findRotation (imageProjection.cpp:492-529)
__device__ void find_rotation(const Deskew& d, double pointTime, float& ox, float& oy, float& oz) {
  // the first f < cur with pointTime < imuTime[f], else cur: over a
  // non-decreasing table that predicate is monotone in f, so a binary search
  // finds the same f as the reference's linear scan (a NaN time: cur in both)
  int f = 0;
  if (d.sorted) {
    int lo = 0, n = d.cur;
    while (n > 0) {
      const int h = n >> 1;
      if (!(pointTime < d.t[lo + h])) {
        lo += h + 1;
        n -= h + 1;
      } else {
        n = h;
      }
    }
    f = lo;
  } else {
    while (f < d.cur) {
      if (pointTime < d.t[f]) break;
      ++f;
    }
  }
  if (pointTime > d.t[f] || f == 0) {
    ox = (float)d.rx[f];
    oy = (float)d.ry[f];
    oz = (float)d.rz[f];
  } else {
    const int b = f - 1;
    const double rf = (pointTime - d.t[b]) / (d.t[f] - d.t[b]);
    const double rb = (d.t[f] - pointTime) / (d.t[f] - d.t[b]);
    ox = (float)(d.rx[f] * rf + d.rx[b] * rb);
    oy = (float)(d.ry[f] * rf + d.ry[b] * rb);
    oz = (float)(d.rz[f] * rf + d.rz[b] * rb);
  }
}

__device__ __forceinline__ float point_range(float x, float y, float z) {
  return sqrtf(x * x + y * y + z * z);  // pointDistance, utility.h:382-384
}

// ---------------------------------------------------------------- block helpers
// exclusive scan of one int per thread over the block; returns the total
template <int NT>
__device__ int block_exclusive_scan(int v, int* scratch /* NT/64 + 1 */, int& excl) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) scratch[w] = x;
  __syncthreads();
  if (t == 0) {
    int s = 0;
    for (int q = 0; q < NT / 64; ++q) {
      const int c = scratch[q];
      scratch[q] = s;
      s += c;
    }
    scratch[NT / 64] = s;
  }
  __syncthreads();
  excl = scratch[w] + x - v;
  const int total = scratch[NT / 64];
  __syncthreads();
  return total;
}

// Bitonic sort of N = 64 * E * NW keys (K: 32 or 64 bits) in LDS (ascending), by the
// first NW wavefronts of the block; every thread of the block calls it (the
// cross-wavefront stages use block barriers).  Lane l of wavefront w holds
// elements e = 64 E w + E l + r, r < E, in registers: partner distances j < E
// are register compare-exchanges, E <= j < 64 E cross-lane shuffles of
// distance j / E, only j >= 64 E goes through LDS (log2(NW) (log2(NW) + 1) / 2
// of the stages).  Keys are unique (value bits << 32 | position), so the
// result is the stable sort of the values.  Barriers on entry and exit.
template <int NW, int E, typename K = uint64_t>
__device__ __forceinline__ void sort_keys_lds(K* key) {
  constexpr int N = 64 * E * NW;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const bool act = w < NW;
  const int e0 = 64 * E * w + E * lane;
  __syncthreads();  // the caller's writes of key[]
  K v[E];
#pragma unroll
  for (int r = 0; r < E; ++r) v[r] = act ? key[e0 + r] : K(0);
  auto cx = [](K a, K p, bool keep_min) { return keep_min ? (a < p ? a : p) : (a < p ? p : a); };
#pragma unroll
  for (int k = 2; k <= N; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j >= 64 * E) {
        __syncthreads();  // every wavefront's previous reads of key[] are done
        if (act)
#pragma unroll
          for (int r = 0; r < E; ++r) key[e0 + r] = v[r];
        __syncthreads();
        if (act)
#pragma unroll
          for (int r = 0; r < E; ++r) {
            const int e = e0 + r;
            const K p = key[e ^ j];
            v[r] = cx(v[r], p, ((e & k) == 0) == ((e & j) == 0));
          }
      } else if (j >= E) {
        if (act)
#pragma unroll
          for (int r = 0; r < E; ++r) {
            const int e = e0 + r;
            const K p = __shfl_xor(v[r], j / E, 64);
            v[r] = cx(v[r], p, ((e & k) == 0) == ((e & j) == 0));
          }
      } else {
#pragma unroll
        for (int r = 0; r < E; ++r) {
          if ((r & j) == 0) {
            const int e = e0 + r;
            const K a = v[r], b = v[r + j];
            const bool up = (e & k) == 0;
            v[r] = up ? (a < b ? a : b) : (a < b ? b : a);
            v[r + j] = up ? (a < b ? b : a) : (a < b ? a : b);
          }
        }
      }
    }
  }
  __syncthreads();
  if (act)
#pragma unroll
    for (int r = 0; r < E; ++r) key[e0 + r] = v[r];
  __syncthreads();
}

// Stable LSD radix sort (8-bit digits) of n <= NT * E (key, value) pairs in
// LDS by the low `bits` bits of the key, ascending; pairs with equal keys
// keep their input order.  Wavefront w ranks the contiguous segment
// [w * seg, (w + 1) * seg) of the input in rounds of 64 (a lane's peers with
// the same digit from 8 ballots, their running count per (wave, digit) in
// LDS), one block scan over the (digit, wave) counts gives every bucket's
// start, and each pair is scattered to its rank.  k0 / v0 hold the input and,
// on return, the sorted pairs (k1 / v1: the other buffer of each pass);
// cnt: 256 * NT / 64 ints; scratch: NT / 64 + 1 ints.  Every thread of the
// block calls it (block barriers inside).
template <int NT, int E>
__device__ __forceinline__ void radix_sort_pairs_lds(uint32_t* k0, int32_t* v0, uint32_t* k1, int32_t* v1,
                                                     int n, int bits, int* cnt, int* scratch) {
  constexpr int W = NT / 64;
  static_assert(256 * W % NT == 0, "radix counters");
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int seg = (n + W - 1) / W;
  const int s0 = min(w * seg, n), s1 = min(s0 + seg, n);
  const uint64_t lt = (1ull << lane) - 1;
  uint32_t* ks = k0;
  int32_t* vs = v0;
  uint32_t* kd = k1;
  int32_t* vd = v1;
  for (int sh = 0; sh < bits; sh += 8) {
    for (int q = t; q < 256 * W; q += NT) cnt[q] = 0;
    __syncthreads();
    uint32_t key[E];
    int32_t val[E], rank[E], dig[E];
#pragma unroll
    for (int k = 0; k < E; ++k) {
      const int i = s0 + 64 * k + lane;
      const bool ok = i < s1;
      key[k] = ok ? ks[i] : 0u;
      val[k] = ok ? vs[i] : 0;
      const int d = (int)((key[k] >> sh) & 255u);
      dig[k] = d;
      uint64_t peers = __ballot(ok);
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const uint64_t m = __ballot(ok && ((d >> b) & 1));
        peers &= ((d >> b) & 1) ? m : ~m;
      }
      // (a lane's own digit: cnt[d * W + w] before this round's peers)
      const int before = ok ? cnt[d * W + w] : 0;
      rank[k] = before + __popcll(peers & lt);
      __builtin_amdgcn_wave_barrier();
      if (ok && (peers & lt) == 0) cnt[d * W + w] = before + __popcll(peers);
      __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    // bucket starts: exclusive scan over (digit, wave) in digit-major order
    constexpr int P = 256 * W / NT;
    int loc[P], sum = 0;
#pragma unroll
    for (int j = 0; j < P; ++j) {
      loc[j] = cnt[t * P + j];
      sum += loc[j];
    }
    int excl;
    block_exclusive_scan<NT>(sum, scratch, excl);
#pragma unroll
    for (int j = 0; j < P; ++j) {
      cnt[t * P + j] = excl;
      excl += loc[j];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < E; ++k) {
      const int i = s0 + 64 * k + lane;
      if (i < s1) {
        const int dst = cnt[dig[k] * W + w] + rank[k];
        kd[dst] = key[k];
        vd[dst] = val[k];
      }
    }
    __syncthreads();
    uint32_t* tk = ks;
    ks = kd;
    kd = tk;
    int32_t* tv = vs;
    vs = vd;
    vd = tv;
  }
  if (ks != k0) {  // an odd number of passes: the result back into k0 / v0
    for (int i = t; i < n; i += NT) {
      k0[i] = ks[i];
      v0[i] = vs[i];
    }
    __syncthreads();
  }
}

// The same stable order by counting: element i of key[0, n) goes to place
// #{j : key[j] < key[i]} + #{j < i : key[j] == key[i]}, and pos[place] =
// first + i.  Every lane walks the whole list as broadcast 16-byte LDS reads
// (j below its wavefront's elements counts with <=, above with <), so the
// cost is n compares per element and no barrier between them: for a few
// hundred keys it beats the radix passes' scans.  key[n, round_up(n, 4)) must
// hold 0xffffffff; pos may alias nothing read here.
template <int NT, int E>
__device__ __forceinline__ void rank_sort_lds(const uint32_t* key, int n, int32_t* pos, int first) {
  const int t = threadIdx.x;
  const int n4 = (n + 3) & ~3;
  const uint4* k4 = reinterpret_cast<const uint4*>(key);
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int i = t + e * NT, wb = (i & ~63);
    if (wb >= n) break;  // wavefront-uniform
    const uint32_t ki = i < n ? key[i] : 0xffffffffu;
    int c = 0;
    const int a = min(wb, n4), b = min(wb + 64, n4);
#pragma unroll 8
    for (int j = 0; j < a; j += 4) {  // 8 reads in flight: the loop is LDS-latency bound
      const uint4 q = k4[j >> 2];
      c += (q.x <= ki) + (q.y <= ki) + (q.z <= ki) + (q.w <= ki);
    }
    for (int j = a; j < b; j += 4) {
      const uint4 q = k4[j >> 2];
      c += (q.x < ki || (q.x == ki && j < i)) + (q.y < ki || (q.y == ki && j + 1 < i)) +
           (q.z < ki || (q.z == ki && j + 2 < i)) + (q.w < ki || (q.w == ki && j + 3 < i));
    }
#pragma unroll 8
    for (int j = b; j < n4; j += 4) {
      const uint4 q = k4[j >> 2];
      c += (q.x < ki) + (q.y < ki) + (q.z < ki) + (q.w < ki);
    }
    if (i < n) pos[c] = first + i;
  }
  __syncthreads();
}

__device__ __forceinline__ int pow2ceil(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}

// ---------------------------------------------------------------- kernels
// Cell owners carry the scan's generation in their high word (hi = ~gen, so
// a newer scan's keys are smaller): atomicMin keeps the smallest point index
// of this scan and a cell holding an older scan's key reads as empty -- no
// reset of the owner table before every scan (rangeMat reset,
// imageProjection.cpp:146).
__global__ __launch_bounds__(256) void k_lio_claim(In in, Geo g, unsigned long long* owner, uint32_t hi,
                                                   uint32_t* block_first) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  bool ok = i < in.n;
  int64_t c = 0;
  if (ok) {
    const float px = in.x[i], py = in.y[i], pz = in.z[i];
    const float range = point_range(px, py, pz);
    const int row = in.ring[i];
    ok = !(range < g.min_r || range > g.max_r) && row >= 0 && row < g.n_scan && row % g.ds == 0;
    if (ok) {
      const float horizonAngle = (float)((double)(fatan2(px, py) * 180.0f) / M_PI);
      int col = (int)(-round(((double)horizonAngle - 90.0) / (double)g.ang_res_x) +
                      (double)(g.horizon / 2));
      if (col >= g.horizon) col -= g.horizon;
      ok = col >= 0 && col < g.horizon;
      c = col + (int64_t)row * g.horizon;
    }
  }
#ifndef SLIO_ABL_NOATOMIC
  if (ok) atomicMin(&owner[c], ((unsigned long long)hi << 32) | (unsigned long long)i);
#else
  if (ok && c < 0) owner[0] = 0;  // diagnostic: no cell atomics
#endif
  // first valid point (deskew reference): the block minimum goes to its own
  // slot (same-address device atomics serialise: 2k of them cost ~20 us)
  __shared__ uint32_t wmin[4];
  uint32_t v = ok ? (uint32_t)i : kNone;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, 64));
  if ((threadIdx.x & 63) == 0) wmin[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) block_first[blockIdx.x] = min(min(wmin[0], wmin[1]), min(wmin[2], wmin[3]));
}

constexpr int kRowThreads = 1024;
constexpr int kFillSplit = 8;     // blocks per ring in k_lio_fill (deskew trig on all CUs)
constexpr int kFillThreads = 256;
constexpr int kImuLds = 512;      // deskew table entries staged in LDS (larger tables stay in HBM)

__device__ __forceinline__ void fsincos(float a, float& s, float& c) {
  double sd, cd;
  sincos((double)a, &sd, &cd);
  s = (float)sd;
  c = (float)cd;
}

// pcl::getTransformation(0, 0, 0, roll, pitch, yaw) with paired sin/cos
__device__ Aff get_rot_sc(float roll, float pitch, float yaw) {
  float A, B, C, D, E, F;
  fsincos(yaw, B, A);
  fsincos(pitch, D, C);
  fsincos(roll, F, E);
  const float DE = D * E, DF = D * F;
  Aff t;
  t.m[0][0] = A * C;
  t.m[0][1] = A * DF - B * E;
  t.m[0][2] = B * F + A * DE;
  t.m[0][3] = 0.0f;
  t.m[1][0] = B * C;
  t.m[1][1] = A * E + B * DF;
  t.m[1][2] = B * DE - A * F;
  t.m[1][3] = 0.0f;
  t.m[2][0] = -D;
  t.m[2][1] = C * F;
  t.m[2][2] = C * E;
  t.m[2][3] = 0.0f;
  return t;
}

// grid (n_scan, kFillSplit): block (r, s) fills columns [s H / S, (s + 1) H / S) of ring r
__global__ __launch_bounds__(kFillThreads) void k_lio_fill(In in, Geo g, const unsigned long long* owner,
                                                           uint32_t hi,
                                                           const uint32_t* block_first, int nfirst,
                                                           Deskew d, float* range_mat,
                                                           float4* full, int32_t* row_part) {
  __shared__ Aff startInv;
  __shared__ int scratch[kFillThreads / 64 + 1];
  __shared__ uint32_t wmin[kFillThreads / 64];
  __shared__ double tb[4][kImuLds];
  const int r = blockIdx.x, sp = blockIdx.y;
  const int t = threadIdx.x;
  const bool desk = d.on && d.cur > 0;
  const int c0 = (int)((int64_t)g.horizon * sp / kFillSplit);
  const int c1 = (int)((int64_t)g.horizon * (sp + 1) / kFillSplit);
  // the thread's first cell: its owner and point loads go out before the
  // scan-start rotation below (independent chains, overlapped)
  const int colA = c0 + t;
  uint32_t oA = kNone;
  float pxA = 0.f, pyA = 0.f, pzA = 0.f, inA = 0.f, tmA = 0.f;
  if (colA < c1) {
    const unsigned long long ok = owner[colA + (int64_t)r * g.horizon];
    oA = (uint32_t)(ok >> 32) == hi ? (uint32_t)ok : kNone;
    if (oA != kNone) {
      pxA = in.x[oA];
      pyA = in.y[oA];
      pzA = in.z[oA];
      inA = in.in[oA];
      if (desk) tmA = in.time[oA];
    }
  }
  if (desk) {
    if (d.cur < kImuLds) {
      for (int q = t; q <= d.cur; q += kFillThreads) {
        tb[0][q] = d.t[q];
        tb[1][q] = d.rx[q];
        tb[2][q] = d.ry[q];
        tb[3][q] = d.rz[q];
      }
    }
    uint32_t v = kNone;
    for (int q = t; q < nfirst; q += kFillThreads) v = min(v, block_first[q]);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, 64));
    if ((t & 63) == 0) wmin[t >> 6] = v;
    __syncthreads();
    if (d.cur < kImuLds) {
      d.t = tb[0];
      d.rx = tb[1];
      d.ry = tb[2];
      d.rz = tb[3];
    }
    if (t == 0) {
      uint32_t f = wmin[0];
      for (int q = 1; q < kFillThreads / 64; ++q) f = min(f, wmin[q]);
      float rx = 0.f, ry = 0.f, rz = 0.f;
      if (f != kNone) find_rotation(d, d.t0 + (double)in.time[f], rx, ry, rz);
      startInv = inverse(get_rot_sc(rx, ry, rz));
    }
    __syncthreads();
  }
  int cnt = 0;
  for (int col = colA; col < c1; col += kFillThreads) {
    const int64_t c = col + (int64_t)r * g.horizon;
    uint32_t o;
    float px, py, pz, pin, ptm = 0.f;
    if (col == colA) {
      o = oA;
      px = pxA;
      py = pyA;
      pz = pzA;
      pin = inA;
      ptm = tmA;
    } else {
      const unsigned long long ok = owner[c];
      o = (uint32_t)(ok >> 32) == hi ? (uint32_t)ok : kNone;
      if (o != kNone) {
        px = in.x[o];
        py = in.y[o];
        pz = in.z[o];
        pin = in.in[o];
        if (desk) ptm = in.time[o];
      }
    }
    if (o == kNone) {
      range_mat[c] = FLT_MAX;
      continue;
    }
    float ox = px, oy = py, oz = pz;
    if (desk) {
      float rx, ry, rz;
      find_rotation(d, d.t0 + (double)ptm, rx, ry, rz);
      const Aff bt = compose(startInv, get_rot_sc(rx, ry, rz));
      ox = bt.m[0][0] * px + bt.m[0][1] * py + bt.m[0][2] * pz + bt.m[0][3];
      oy = bt.m[1][0] * px + bt.m[1][1] * py + bt.m[1][2] * pz + bt.m[1][3];
      oz = bt.m[2][0] * px + bt.m[2][1] * py + bt.m[2][2] * pz + bt.m[2][3];
    }
    range_mat[c] = point_range(px, py, pz);
    full[c] = make_float4(ox, oy, oz, pin);
    ++cnt;
  }
  int excl;
  const int total = block_exclusive_scan<kFillThreads>(cnt, scratch, excl);
  if (t == 0) row_part[r * kFillSplit + sp] = total;
}

struct CloudInfo {
  int32_t* start_ring;
  int32_t* end_ring;
  int32_t* col_ind;
  float* prange;
  float4* xyzi;
  int32_t* n_ext;
};

__global__ __launch_bounds__(kRowThreads) void k_lio_extract(Geo g, const float* range_mat,
                                                             const float4* full,
                                                             const int32_t* row_count, CloudInfo ci) {
  __shared__ int scratch[kRowThreads / 64 + 1];
  const int r = blockIdx.x;
  const int t = threadIdx.x;
  int part = 0;  // ring offset = sum of the partial counts of rings < r
  for (int q = t; q < r * kFillSplit; q += kRowThreads) part += row_count[q];
  int excl;
  const int off = block_exclusive_scan<kRowThreads>(part, scratch, excl);
  if (t == 0) {
    int cnt = 0;
    for (int q = 0; q < kFillSplit; ++q) cnt += row_count[r * kFillSplit + q];
    ci.start_ring[r] = off - 1 + 5;
    ci.end_ring[r] = off + cnt - 1 - 5;
    if (r == g.n_scan - 1) *ci.n_ext = off + cnt;
  }
  // thread t owns the contiguous columns [t * per, (t + 1) * per)
  const int per = (g.horizon + kRowThreads - 1) / kRowThreads;
  const int c0 = t * per, c1 = min(c0 + per, g.horizon);
  int cnt = 0;
  for (int col = c0; col < c1; ++col) cnt += range_mat[col + (int64_t)r * g.horizon] != FLT_MAX;
  block_exclusive_scan<kRowThreads>(cnt, scratch, excl);
  int k = off + excl;
  for (int col = c0; col < c1; ++col) {
    const int64_t c = col + (int64_t)r * g.horizon;
    const float rg = range_mat[c];
    if (rg != FLT_MAX) {
      ci.col_ind[k] = col;
      ci.prange[k] = rg;
      ci.xyzi[k] = full[c];
      ++k;
    }
  }
}

// calculateSmoothness + markOccludedPoints, pull form: flag i is set iff some
// j of the reference loop (:138-176) would set it.
__device__ __forceinline__ bool occ_a(const float* r, const int32_t* col, int j) {
  const int cd = abs(col[j + 1] - col[j]);
  return cd < 10 && (double)(r[j] - r[j + 1]) > 0.3;
}
__device__ __forceinline__ bool occ_b(const float* r, const int32_t* col, int j) {
  const int cd = abs(col[j + 1] - col[j]);
  return cd < 10 && !((double)(r[j] - r[j + 1]) > 0.3) && (double)(r[j + 1] - r[j]) > 0.3;
}

// calculateSmoothness + markOccludedPoints of position i of the extracted
// cloud (n points): r / col are range and column arrays indexed so that
// r[q], col[q] hold position q's for q in [i - 6, i + 6] (k_fe_pick stages
// them in LDS).
__device__ __forceinline__ void smooth_at(const float* r, const int32_t* col, int n, int i, float& curv,
                                          uint8_t& picked) {
  curv = 0.0f;
  int pk = 1;  // entries the reference never initialises: never picked
  if (i >= 5 && i < n - 5) {
    const float diffRange = r[i - 5] + r[i - 4] + r[i - 3] + r[i - 2] + r[i - 1] - r[i] * 10 +
                            r[i + 1] + r[i + 2] + r[i + 3] + r[i + 4] + r[i + 5];
    curv = diffRange * diffRange;
    pk = 0;
    const int jmax = n - 7;  // loop i < cloudSize - 6
    for (int j = max(i, 5); j <= min(i + 5, jmax); ++j)
      if (occ_a(r, col, j)) pk = 1;
    for (int j = max(i - 6, 5); j <= min(i - 1, jmax); ++j)
      if (occ_b(r, col, j)) pk = 1;
    if (i <= jmax) {
      const float diff1 = fabsf(r[i - 1] - r[i]);
      const float diff2 = fabsf(r[i + 1] - r[i]);
      if ((double)diff1 > 0.02 * (double)r[i] && (double)diff2 > 0.02 * (double)r[i]) pk = 1;
    }
  }
  picked = (uint8_t)pk;
}

struct FeatOut {
  int32_t* label;          // n_ext
  float4* corner_stage;    // n_scan * kCornerPerRing (pick order)
  int32_t* corner_count;   // n_scan
  float4* surf_stage;      // n_ext (ring r at its first extracted index)
  int32_t* surf_count;     // n_scan
  // LeGO-LOAM only
  int8_t* corner_sharp;    // n_scan * kCornerPerRing: 1 = cornerPointsSharp (label 2)
  int32_t* sharp_count;    // n_scan
  float4* flat_stage;      // n_scan * kFlatPerRing (pick order)
  int32_t* flat_count;     // n_scan
  const uint8_t* ground;   // segmentedCloudGroundFlag (n_ext)
};

struct FeatCfg {
  float edge_thr, surf_thr, leaf;
  int sort_cap;   // power of two >= max sector length
  int ring_cap;   // >= ring span incl. 5-point margins
  int vox_cap;    // power of two >= max ring length
};

constexpr int kFeatThreads = 1024;
// per (ring, sector): one wavefront per variant (waves 6-7 join the shared
// sector sort and reach phase only; all 8 sort the ring's VoxelGrid order in
// the 7th workgroup of a ring, ring_vsort)
constexpr int kPickThreads = 512;
static_assert(kPickThreads > 6 * 64, "waves past the 6 variants store the smoothness outputs");
// k_fe_pick's per-position LDS arrays: sort_cap + kPickPad entries (a sector,
// its 5-point margins, the last sector's extra point, and the 6-point halos
// of the staged range / columns, kHalo on each side)
constexpr int kPickPad = 32, kHalo = 6;

// Scratch of the feature stage, per ring r, sector j, variant v.
// Sectors of a ring interact only through the suppression marks a sector's
// picks leave on the first <= 5 points of the next one (reach <= 5,
// featureExtraction.cpp:220-237, 247-262), and those marks are a PREFIX of
// the next sector (every mark range starts right after its pick, at or before
// the sector's first point).  So each sector runs its greedy picks once per
// possible prefix length v = 0..5, all in parallel, and the ring's chain then
// selects, sector by sector, the variant the previous sectors' real marks
// call for: exactly the sequential reference's result.
struct PickVar {
  int32_t corner[20];  // edge picks in pick order (featureExtraction.cpp:209-218)
  int32_t flat[4];     // LeGO-LOAM flat picks in pick order
  int32_t ncorner;     // <= 20
  int32_t nflat;       // LeGO-LOAM: <= 4
  int32_t fwd_end;     // last position past ep newly flagged by this sector's picks (-1: none)
  int32_t pad;
};

struct FeatWork {
  int32_t* spos;      // [R][6][sort_cap]: sector positions in std::sort order
  PickVar* var;       // [R][6][6]
  int8_t* lab;        // [R][6][6][sort_cap]: labels of positions sp..ep
  // the ring's VoxelGrid order, sorted beside the picks (ring_vsort):
  // [R][kVsortN] (voxel << 32 | position) over every position of the ring's
  // live sectors, and per ring their number (-1: k_fe_ring sorts itself)
  uint64_t* vkey;
  int32_t* vinfo;
};
constexpr int kVsortN = 2048;  // ring_vsort: rings of up to this many positions

// sector j of a ring (featureExtraction.cpp:191-192)
__device__ __forceinline__ void sector_bounds(int start, int end, int j, int& sp, int& ep) {
  sp = (start * (6 - j) + end * j) / 6;
  ep = (start * (5 - j) + end * (j + 1)) / 6 - 1;
}

#ifdef SLIO_FE_STAMP
// diagnostic build only: k_fe_pick phase stamps per (ring, sector, variant)
__device__ unsigned long long g_fstamp[256 * 36][6];
#define FSTAMP(k)                                                                  \
  do {                                                                             \
    if ((threadIdx.x & 63) == 0 && blockIdx.y < 256 && (threadIdx.x >> 6) < 6)     \
      g_fstamp[blockIdx.y * 36 + blockIdx.x * 6 + (threadIdx.x >> 6)][k] =         \
          __builtin_amdgcn_s_memrealtime();                                        \
  } while (0)
__device__ unsigned long long g_rstamp[256][8];
__device__ unsigned long long g_vstamp[256][4];  // ring_vsort: start, keys built, sorted, end
#define VSTAMP(k)                                                                  \
  do {                                                                             \
    if (threadIdx.x == 0 && blockIdx.y < 256)                                      \
      g_vstamp[blockIdx.y][k] = __builtin_amdgcn_s_memrealtime();                  \
  } while (0)
#define RGSTAMP(k)                                                                 \
  do {                                                                             \
    if (threadIdx.x == 0 && blockIdx.x < 256)                                      \
      g_rstamp[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime();                  \
  } while (0)
#else
#define FSTAMP(k) \
  do {            \
  } while (0)
#define RGSTAMP(k) \
  do {             \
  } while (0)
#define VSTAMP(k) \
  do {            \
  } while (0)
#endif

// ---- ring_vsort: the 7th workgroup of ring r in k_fe_pick's grid, running
// beside the ring's six sector picks.  k_fe_ring's VoxelGrid (pcl::VoxelGrid
// on surfaceCloudScan, featureExtraction.cpp:265-269) sorts the ring's surface
// list -- the live sectors' positions whose label is <= 0 -- by voxel index
// (then list = position order).  That order does not depend on the picks:
// the voxel index over any bounding box holding the points is a mixed-radix
// number of (floor(z / leaf), floor(y / leaf), floor(x / leaf)), so its order
// and its equal runs are those of the triple, whatever the box; and removing
// the corner picks (label 1) from the sorted full list leaves the surface
// list sorted.  So the full list is sorted here, over its own bounding box,
// and k_fe_ring keeps the entries whose label is <= 0.  When this box would
// overflow PCL's index check (the surface list's box is no larger, so a pass
// here is a pass there) or the ring has more than kVsortN positions, vinfo is
// -1 and k_fe_ring sorts the surface list itself.
__device__ __forceinline__ void ring_vsort(const CloudInfo& ci, const FeatCfg& cfg, const FeatWork& fw,
                                           unsigned char* smem) {
  constexpr int kW = kPickThreads / 64;
  constexpr int kHeld = kVsortN / kPickThreads;  // points per thread, kept in registers
  static_assert(kVsortN % kPickThreads == 0, "ring_vsort layout");
  const int r = blockIdx.y, t = threadIdx.x, lane = t & 63, w = t >> 6;
  VSTAMP(0);
  const int start = ci.start_ring[r], end = ci.end_ring[r];
  __shared__ int s_lo[6], s_cnt[7];
  __shared__ float wmn[kPickThreads / 64][3], wmx[kPickThreads / 64][3];
  __shared__ int s_ok, s_minb[3], s_mul[3], s_bits;
  __shared__ int rscratch[kW + 1];
  if (t == 0) {
    int c = 0;
    for (int j = 0; j < 6; ++j) {
      int sp, ep;
      sector_bounds(start, end, j, sp, ep);
      s_lo[j] = sp;
      s_cnt[j] = c;
      if (sp < ep) c += ep - sp + 1;  // a live sector: positions sp..ep
    }
    s_cnt[6] = c;
  }
  __syncthreads();
  const int m = s_cnt[6];
  auto pos_of = [&](int i) {  // the i-th position of the live sectors, in order
    int j = 0;
#pragma unroll
    for (int jj = 1; jj < 6; ++jj) j = i >= s_cnt[jj] ? jj : j;
    return s_lo[j] + (i - s_cnt[j]);
  };
  if (end - start > kVsortN) {
    if (t == 0) fw.vinfo[r] = -1;
    return;
  }
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  float4 held[kHeld];
  int hq[kHeld];
#pragma unroll
  for (int k = 0; k < kHeld; ++k) {
    const int i = t + k * kPickThreads;
    hq[k] = i < m ? pos_of(i) : -1;
    held[k] = i < m ? ci.xyzi[hq[k]] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int k = 0; k < kHeld; ++k) {
    if (hq[k] < 0) continue;
    const float4 p = held[k];
    mn[0] = fminf(mn[0], p.x);
    mn[1] = fminf(mn[1], p.y);
    mn[2] = fminf(mn[2], p.z);
    mx[0] = fmaxf(mx[0], p.x);
    mx[1] = fmaxf(mx[1], p.y);
    mx[2] = fmaxf(mx[2], p.z);
  }
#pragma unroll
  for (int a = 0; a < 3; ++a) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      mn[a] = fminf(mn[a], __shfl_xor(mn[a], o, 64));
      mx[a] = fmaxf(mx[a], __shfl_xor(mx[a], o, 64));
    }
  }
  if (lane == 0)
    for (int a = 0; a < 3; ++a) {
      wmn[w][a] = mn[a];
      wmx[w][a] = mx[a];
    }
  __syncthreads();
  const float inv = 1.0f / cfg.leaf;
  if (t == 0) {
    float lo[3], hi[3];
    for (int a = 0; a < 3; ++a) {
      lo[a] = wmn[0][a];
      hi[a] = wmx[0][a];
      for (int q = 1; q < kPickThreads / 64; ++q) {
        lo[a] = fminf(lo[a], wmn[q][a]);
        hi[a] = fmaxf(hi[a], wmx[q][a]);
      }
    }
    // k_fe_ring's check on this box (PCL applyFilter's overflow test)
    const int64_t dx = (int64_t)((hi[0] - lo[0]) * inv) + 1;
    const int64_t dy = (int64_t)((hi[1] - lo[1]) * inv) + 1;
    const int64_t dz = (int64_t)((hi[2] - lo[2]) * inv) + 1;
    int64_t divb[3];
    for (int a = 0; a < 3; ++a) {
      s_minb[a] = (int)floorf(lo[a] * inv);
      divb[a] = (int64_t)((int)floorf(hi[a] * inv) - s_minb[a] + 1);
    }
    const int64_t cells = divb[0] * divb[1] * divb[2];
    s_ok = m > 0 && dx * dy * dz <= (int64_t)2147483647 && cells <= (int64_t)2147483647;
    s_mul[0] = 1;
    s_mul[1] = (int)divb[0];
    s_mul[2] = (int)(divb[0] * divb[1]);
    const uint32_t top = s_ok ? (uint32_t)(cells - 1) : 0u;
    s_bits = top ? 32 - __clz((int)top) : 1;
  }
  __syncthreads();
  if (!s_ok) {
    if (t == 0) fw.vinfo[r] = m > 0 ? -1 : 0;
    return;
  }
  auto voxel_of = [&](const float4& p) {
    const int i0 = (int)(floorf(p.x * inv) - (float)s_minb[0]);
    const int i1 = (int)(floorf(p.y * inv) - (float)s_minb[1]);
    const int i2 = (int)(floorf(p.z * inv) - (float)s_minb[2]);
    return (uint32_t)(i0 * s_mul[0] + i1 * s_mul[1] + i2 * s_mul[2]);
  };
  uint64_t* out = fw.vkey + (int64_t)r * kVsortN;
  // (voxel, position) pairs in list order, then the stable sort by voxel
  uint32_t* vk0 = reinterpret_cast<uint32_t*>(smem);
  int32_t* vv0 = reinterpret_cast<int32_t*>(vk0 + kVsortN);
  uint32_t* vk1 = reinterpret_cast<uint32_t*>(vv0 + kVsortN);
  int32_t* vv1 = reinterpret_cast<int32_t*>(vk1 + kVsortN);
  int* vcnt = reinterpret_cast<int*>(vv1 + kVsortN);
#pragma unroll
  for (int k = 0; k < kHeld; ++k)
    if (hq[k] >= 0) {
      vk0[t + k * kPickThreads] = voxel_of(held[k]);
      vv0[t + k * kPickThreads] = hq[k];
    }
  __syncthreads();
  VSTAMP(1);
  radix_sort_pairs_lds<kPickThreads, kHeld>(vk0, vv0, vk1, vv1, m, s_bits, vcnt, rscratch);
  VSTAMP(2);
  for (int i = t; i < m; i += kPickThreads) out[i] = ((uint64_t)vk0[i] << 32) | (uint32_t)vv0[i];
  if (t == 0) fw.vinfo[r] = m;
  VSTAMP(3);
}

// ---- k_fe_pick: grid (6, R), 6 wavefronts: sector j of ring r.  The block
// loads the sector (curvature, columns, flags, reach) and sorts it once:
// std::sort(sp, ep) by smoothness (featureExtraction.cpp:200) as a stable
// block radix sort of (value bits, position) in position order, so ties fall
// to the lower index (the oracle's deterministic choice; values are squares
// >= +0, whose bits order as the floats; entries the reference never
// initialises sort as 0).  Then wavefront v runs the greedy edge / flat picks
// with the sector's v leading points pre-flagged (variant v), on its own
// flags and labels, with register eligibility (a 64-candidate chunk is
// loaded once; a pick clears the candidates inside its reach range; the
// chunk's labels and flags go to LDS before the next chunk reads them).
// MODE kModeLio: LIO-SAM extractFeatures (featureExtraction.cpp:183-296);
// kModeLego: LeGO-LOAM extractFeatures (featureAssociation.cpp:883-1007):
// edges only off the ground (labels 2 for the first 2 = sharp, 1 up to 20),
// flats only on the ground, at most 4 per sector (the 4th does not suppress).
template <int MODE, int SORTN>
__global__ __launch_bounds__(kPickThreads) void k_fe_pick(
    const CloudInfo ci, float* __restrict__ curvature, uint8_t* __restrict__ picked0, int32_t* __restrict__ label,
    const uint8_t* __restrict__ ground, FeatCfg cfg, FeatWork fw) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  static_assert(SORTN >= 64 && SORTN <= 2048 && (SORTN & (SORTN - 1)) == 0, "sort size");
  constexpr int kRadixE = SORTN >= kPickThreads ? SORTN / kPickThreads : 1;
  __shared__ int rscratch[kPickThreads / 64 + 1];
  if (blockIdx.x == 6) {  // the ring's VoxelGrid order (ring_vsort)
    ring_vsort(ci, cfg, fw, smem);
    return;
  }
  const int j = blockIdx.x, r = blockIdx.y;
  const int t = threadIdx.x, lane = t & 63, v = t >> 6;
  const int n = *ci.n_ext;
  const int start = ci.start_ring[r], end = ci.end_ring[r];
  const int base = max(start - 5, 0);
  const int span_end = min(end + 5, n - 1);
  int sp, ep;
  sector_bounds(start, end, j, sp, ep);
  const int cap = cfg.sort_cap, pcap = cfg.sort_cap + kPickPad;
  const int pb = max(sp - 5, base), pe = min(ep + 5, span_end);
  // this block's share of the ring's points [start - 4, end + 5] for the
  // smoothness outputs (sector j's positions; the first / last sector also
  // the ring's 4 / 6 points outside every sector)
  const int wlo = max(j == 0 ? start - 4 : sp, 0), whi = min(j == 5 ? end + 5 : ep, n - 1);
  // LDS index base: pb (a live sector's share starts at or after pb; a ring
  // with fewer than 11 points has no live sector, and its shares may reach
  // back into the previous ring)
  const int lb = min(pb, wlo), hi = max(pe, whi);
  // the sector's sort (SORTN = cap): keys / positions and the radix sort's
  // second buffers and counters; spos: the sector in sort order after it
  uint32_t* rk0 = reinterpret_cast<uint32_t*>(smem);
  int32_t* spos = reinterpret_cast<int32_t*>(rk0 + SORTN);
  uint32_t* rk1 = reinterpret_cast<uint32_t*>(spos + SORTN);
  int32_t* rv1 = reinterpret_cast<int32_t*>(rk1 + SORTN);
  int* rcnt = reinterpret_cast<int*>(rv1 + SORTN);  // 256 x waves
  float* curv = reinterpret_cast<float*>(rcnt + 256 * (kPickThreads / 64));
  int32_t* col = reinterpret_cast<int32_t*>(curv + pcap) + kHalo;  // col[q - pb], q >= pb - kHalo
  float* rng = reinterpret_cast<float*>(col - kHalo + pcap) + kHalo;  // range, as col
  uint8_t* pk0 = reinterpret_cast<uint8_t*>(rng - kHalo + pcap);  // cloudNeighborPicked on entry
  uint8_t* brk = pk0 + pcap;    // column step into position q exceeds 10
  uint8_t* reach = brk + pcap;  // reachL | reachR << 4
  uint8_t* gfl = reach + pcap;  // LeGO: segmentedCloudGroundFlag
  // the wavefront's own flags and labels: written by one lane and read by
  // the others of the wavefront: volatile LDS accesses, in program order
  volatile uint8_t* flag = reinterpret_cast<volatile uint8_t*>(gfl + pcap) + v * 2 * pcap;
  volatile int8_t* lab = reinterpret_cast<volatile int8_t*>(flag + pcap);
  // calculateSmoothness + markOccludedPoints (featureExtraction.cpp:108-176)
  // for [lb, hi] from range / column staged over [lb - 6, hi + 6]
  for (int q = max(lb - kHalo, 0) + t; q <= min(hi + kHalo, n - 1); q += kPickThreads) {
    rng[q - lb] = ci.prange[q];
    col[q - lb] = ci.col_ind[q];
  }
  if (MODE == kModeLego)
    for (int q = pb + t; q <= pe; q += kPickThreads) gfl[q - pb] = ground[q];
  __syncthreads();
  for (int q = lb + t; q <= hi; q += kPickThreads) {
    float c;
    uint8_t pk;
    smooth_at(rng - lb, col - lb, n, q, c, pk);
    curv[q - lb] = c;
    pk0[q - lb] = pk;
  }
  __syncthreads();
  // the block's smoothness outputs: stored here by a dead sector, else by
  // waves 6-7 once they are done with the sort and the reach (a barrier
  // waits for every store issued before it)
  auto store_outputs = [&](int t0, int nt) {
    for (int q = wlo + t0; q <= whi; q += nt) {
      curvature[q] = curv[q - lb];
      picked0[q] = pk0[q - lb];
      label[q] = 0;  // k_fe_ring writes the rings' [start, end]
    }
  };
  if (sp >= ep) {  // `if (sp >= ep) continue;`
    store_outputs(t, kPickThreads);
    if (lane == 0 && v < 6 && (j > 0 || v == 0)) {
      PickVar* pv = fw.var + (r * 6 + j) * 6 + v;
      pv->ncorner = 0;
      pv->nflat = 0;
      pv->fwd_end = -1;
    }
    return;
  }
  FSTAMP(0);
  // the sector's sort: the stable sort of (value bits, position) by value
  // (values >= +0 order as their bits; equal values keep position order)
  const int len = ep - sp;
  if constexpr (SORTN <= 2 * kPickThreads) {  // counting ranks (rank_sort_lds)
    for (int idx = t; idx < ((len + 3) & ~3); idx += kPickThreads) {
      const int k = sp + idx;
      rk0[idx] = idx < len ? __float_as_uint((k >= 5 && k < n - 5) ? curv[k - pb] : 0.0f) : 0xffffffffu;
    }
    __syncthreads();
    rank_sort_lds<kPickThreads, (SORTN + kPickThreads - 1) / kPickThreads>(rk0, len, spos, sp);
  } else {
    for (int idx = t; idx < len; idx += kPickThreads) {
      const int k = sp + idx;
      rk0[idx] = __float_as_uint((k >= 5 && k < n - 5) ? curv[k - pb] : 0.0f);
      spos[idx] = k;
    }
    __syncthreads();
    radix_sort_pairs_lds<kPickThreads, kRadixE>(rk0, spos, rk1, rv1, len, 32, rcnt, rscratch);
  }
  FSTAMP(1);
  // suppression reach (:220-237, 247-262): points ind + l, l = 1..5 (and
  // -1..-5), are flagged while consecutive columns differ by <= 10, so a
  // pick flags the contiguous range [ind - reachL, ind + reachR]
  for (int q = max(pb + 1, sp - 4) + t; q <= pe; q += kPickThreads)
    brk[q - pb] = abs(col[q - pb] - col[q - 1 - pb]) > 10;
  __syncthreads();
  for (int q = sp + t; q <= ep; q += kPickThreads) {
    bool okr = true, okl = true;
    int rr = 0, rl = 0;
#pragma unroll
    for (int l = 1; l <= 5; ++l) {
      okr = okr && q + l <= span_end && !brk[min(q + l, pe) - pb];
      okl = okl && q - l >= base && !brk[q - l + 1 - pb];
      rr += okr;
      rl += okl;
    }
    reach[q - pb] = (uint8_t)(rl | (rr << 4));
  }
  __syncthreads();
  if (v >= 6) {
    store_outputs(t - 6 * 64, kPickThreads - 6 * 64);
    return;
  }
  if (j == 0 && v > 0) return;  // 6 variants; nothing precedes the first sector
  FSTAMP(2);
  const int slot = (r * 6 + j) * 6 + v;
  PickVar* pv = fw.var + slot;
  for (int q = pb + lane; q <= pe; q += 64) {
    flag[q - pb] = pk0[q - pb] | (uint8_t)(q >= sp && q < sp + v);
    lab[q - pb] = 0;
  }
  auto ind_at = [&](int k) -> int { return k == ep ? ep : spos[k - sp]; };
  // edges: k = ep .. sp, at most 20 (:205-238).  [sp, ep) is sorted by
  // curvature, so below the first sorted value <= edgeThreshold nothing is
  // eligible: the scan stops there (k = ep, outside the sort, first).
  int picks = 0;
  bool stop = false;
  for (int top = ep; top >= sp && !stop; top -= 64) {
    const int k = top - lane;
    int ind = 0, lo = 0, hi = -1, myrank = 0;
    bool el = false, tail = false, mine = false;
    if (k >= sp) {
      ind = ind_at(k);
      const int bb = ind - pb;
      const int rc = reach[bb];
      lo = ind - (rc & 15);
      hi = ind + (rc >> 4);
      const float cv = curv[bb];
      el = !flag[bb] && cv > cfg.edge_thr && (MODE == kModeLio || !gfl[bb]);
      tail = k < ep && !(cv > cfg.edge_thr);
    }
    const bool last_chunk = __ballot(tail) != 0;
    uint64_t msk = __ballot(el);
    while (msk) {
      const int l = __ffsll((long long)msk) - 1;
      if (++picks > 20) {
        stop = true;
        break;
      }
      const int lol = __builtin_amdgcn_readlane(lo, l);
      const int hil = __builtin_amdgcn_readlane(hi, l);
      if (lane == l) {
        mine = true;
        myrank = picks;
        pv->corner[picks - 1] = ind;
      }
      el = el && lane > l && !(ind >= lol && ind <= hil);
      msk = __ballot(el);
    }
    if (mine) {
      lab[ind - pb] = (MODE == kModeLego && myrank <= 2) ? 2 : 1;
      for (int q = lo; q <= hi; ++q) flag[q - pb] = 1;
    }
    if (last_chunk) break;
  }
  FSTAMP(3);
  // flats: k = sp .. ep (:239-263).  Ascending curvature: the scan stops
  // after the first sorted value >= surfThreshold; k = ep is examined last.
  bool done_sorted = false;
  int fpicks = 0;
  bool fstop = false;
  for (int bot = sp; bot < ep && !done_sorted && !fstop; bot += 64) {
    const int k = bot + lane;
    int ind = 0, lo = 0, hi = -1;
    bool el = false, tail = false, mine = false, supp = false;
    if (k < ep) {
      ind = ind_at(k);
      const int bb = ind - pb;
      const int rc = reach[bb];
      lo = ind - (rc & 15);
      hi = ind + (rc >> 4);
      const float cv = curv[bb];
      el = !flag[bb] && cv < cfg.surf_thr && (MODE == kModeLio || gfl[bb]);
      tail = !(cv < cfg.surf_thr);
    }
    done_sorted = __ballot(tail) != 0;
    uint64_t msk = __ballot(el);
    while (msk) {
      const int l = __ffsll((long long)msk) - 1;
      ++fpicks;
      if (lane == l) {
        mine = true;
        if (MODE == kModeLego) pv->flat[fpicks - 1] = ind;
      }
      if (MODE == kModeLego && fpicks >= 4) {
        fstop = true;
        break;
      }
      supp |= lane == l;
      const int lol = __builtin_amdgcn_readlane(lo, l);
      const int hil = __builtin_amdgcn_readlane(hi, l);
      el = el && lane > l && !(ind >= lol && ind <= hil);
      msk = __ballot(el);
    }
    if (mine) lab[ind - pb] = -1;
    if (supp)
      for (int q = lo; q <= hi; ++q) flag[q - pb] = 1;
  }
  if (!fstop) {  // k = ep (outside the sorted range)
    const int bb = ep - pb;
    if (!flag[bb] && curv[bb] < cfg.surf_thr && (MODE == kModeLio || gfl[bb])) {
      ++fpicks;
      const int rc = reach[bb];
      const int lol = ep - (rc & 15), hil = ep + (rc >> 4);
      if (lane == 0) {
        lab[bb] = -1;
        if (MODE == kModeLego) pv->flat[fpicks - 1] = ep;
      }
      if (!(MODE == kModeLego && fpicks >= 4) && lane <= hil - lol) flag[lol + lane - pb] = 1;
    }
  }
  FSTAMP(4);
  int8_t* lout = fw.lab + (int64_t)slot * cap;
  for (int q = sp + lane; q <= ep; q += 64) lout[q - sp] = lab[q - pb];
  // marks this sector leaves past its end (a prefix of the next sector)
  const int qf = ep + 1 + lane;
  const bool marked = lane < 5 && qf <= pe && flag[qf - pb] && !pk0[qf - pb];
  const uint64_t mb = __ballot(marked);
  if (lane == 0) {
    pv->ncorner = min(picks, 20);
    pv->nflat = MODE == kModeLego ? min(fpicks, 4) : 0;
    pv->fwd_end = mb ? ep + 64 - __clzll((long long)mb) : -1;
  }
  FSTAMP(5);
}

// The VoxelGrid's output from the surface list in voxel order: keys[q] =
// voxel << 32 | ring position (m entries, in LDS), points from rp.  One
// thread per voxel run start sums the run's points in list order
// (CentroidPoint); voxels go out in ascending index (applyFilter).
template <int NT>
__device__ __forceinline__ void ring_voxels(const uint64_t* keys, float4* vp, const float4* rp, int start, int m,
                                            float4* dst, int* scratch, int32_t* count) {
  const int t = threadIdx.x;
  for (int q = t; q < m; q += NT) vp[q] = rp[(int)(uint32_t)keys[q] - start];
  __syncthreads();
  const int per = (m + NT - 1) / NT;
  const int q0 = t * per, q1 = min(q0 + per, m);
  int starts = 0;
  for (int q = q0; q < q1; ++q) starts += (q == 0) || ((keys[q] >> 32) != (keys[q - 1] >> 32));
  int excl;
  const int nvox = block_exclusive_scan<NT>(starts, scratch, excl);
  int o = excl;
  for (int q = q0; q < q1; ++q) {
    if (!((q == 0) || ((keys[q] >> 32) != (keys[q - 1] >> 32)))) continue;
    const uint32_t id = (uint32_t)(keys[q] >> 32);
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int e = q;
    for (; e < m && (uint32_t)(keys[e] >> 32) == id; ++e) {
      const float4 p = vp[e];
      s0 += p.x;
      s1 += p.y;
      s2 += p.z;
      s3 += p.w;
    }
    const float cnt = (float)(e - q);
    dst[o++] = make_float4(s0 / cnt, s1 / cnt, s2 / cnt, s3 / cnt);
  }
  if (t == 0) *count = nvox;
}

// ---- k_fe_ring: one workgroup per ring.  Variant selection (sector j gets
// the prefix v_j the earlier sectors' marks reach), the ring's labels,
// corners in pick order, surfaceCloudScan (:265-269: sector positions with
// label <= 0, position order), then pcl::VoxelGrid on it: bounding box, leaf
// divisions ("integer indices would overflow" -> output = input), the sort
// of (voxel index, list index) as a stable block radix sort of the voxel
// index over the list order (a voxel's points keep list order), one thread
// per voxel run start, centroid summed in list order (CentroidPoint), voxels
// in ascending index (applyFilter).
template <int MODE, int VOXN>
__global__ __launch_bounds__(kFeatThreads) void k_fe_ring(const CloudInfo ci, FeatCfg cfg,
                                                          FeatOut out, FeatWork fw) {
  static_assert(VOXN >= 64 && VOXN <= 4096 && (VOXN & (VOXN - 1)) == 0, "voxel sort size");
#ifndef SLIO_RING_SORT_W
#define SLIO_RING_SORT_W 16
#endif
  constexpr int kSortW0 = VOXN / 64 < SLIO_RING_SORT_W ? VOXN / 64 : SLIO_RING_SORT_W;
  constexpr int kSortW = kSortW0 < kFeatThreads / 64 ? kSortW0 : kFeatThreads / 64, kSortE = VOXN / (64 * kSortW);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float4* rp = reinterpret_cast<float4*>(smem);                 // ring_cap: the ring's points
  float4* vp = rp + cfg.ring_cap;                               // vox_cap: voxel order
  uint64_t* keys = reinterpret_cast<uint64_t*>(vp + cfg.vox_cap);  // vox_cap
  int32_t* slist = reinterpret_cast<int32_t*>(keys + cfg.vox_cap);  // ring_cap
  int8_t* labr = reinterpret_cast<int8_t*>(slist + cfg.ring_cap);   // ring_cap
  __shared__ int s_sp[6], s_ep[6], s_slot[6], s_cb[7], s_fb[7];
  __shared__ int s_hdr[36][3];  // the ring's variants: ncorner, nflat, fwd_end
  __shared__ int scratch[kFeatThreads / 64 + 1];
  __shared__ float s_min[3], s_max[3];
  __shared__ int s_overflow, s_minb[3], s_mul[3], s_bits;
  const int r = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int start = ci.start_ring[r], end = ci.end_ring[r];
  RGSTAMP(0);
  // the ring's presorted VoxelGrid order (ring_vsort, beside the picks):
  // this thread's share of the entries, loaded with the ring
  const int vm = fw.vinfo ? fw.vinfo[r] : -1;
  constexpr int kVPer = (kVsortN + kFeatThreads - 1) / kFeatThreads;
  uint64_t vk[kVPer];
#pragma unroll
  for (int i = 0; i < kVPer; ++i) {
    const int e = t * kVPer + i;
    vk[i] = (vm > 0 && e < vm) ? fw.vkey[(int64_t)r * kVsortN + e] : 0ull;
  }
  // the ring's points, loaded once (corners, surface list and voxel grid
  // read them from LDS)
  for (int q = start + t; q <= end; q += kFeatThreads) rp[q - start] = ci.xyzi[q];
  if (t < 36) {
    int sp, ep;
    sector_bounds(start, end, t / 6, sp, ep);
    const PickVar& p = fw.var[r * 36 + t];
    const bool live = sp < ep && (t / 6 > 0 || t % 6 == 0);
    s_hdr[t][0] = live ? p.ncorner : 0;
    s_hdr[t][1] = live ? p.nflat : 0;
    s_hdr[t][2] = live ? p.fwd_end : -1;
  }
  __syncthreads();
  if (t == 0) {
    int maxfwd = -1, cb = 0, fb = 0, sharp = 0;
    for (int j = 0; j < 6; ++j) {
      int sp, ep;
      sector_bounds(start, end, j, sp, ep);
      s_sp[j] = sp;
      s_ep[j] = ep;
      s_cb[j] = cb;
      s_fb[j] = fb;
      s_slot[j] = -1;
      if (sp >= ep) continue;
      const int vv = min(max(maxfwd - sp + 1, 0), 5);
      s_slot[j] = (r * 6 + j) * 6 + vv;
      maxfwd = max(maxfwd, s_hdr[j * 6 + vv][2]);
      cb += s_hdr[j * 6 + vv][0];
      fb += s_hdr[j * 6 + vv][1];
      sharp += min(s_hdr[j * 6 + vv][0], 2);
    }
    s_cb[6] = cb;
    s_fb[6] = fb;
    out.corner_count[r] = cb;
    if (MODE == kModeLego) {
      out.sharp_count[r] = sharp;
      out.flat_count[r] = fb;
    }
  }
  __syncthreads();
  RGSTAMP(1);
  auto sector_of = [&](int k) {
    int s = -1;
#pragma unroll
    for (int jj = 0; jj < 6; ++jj)
      if (s_slot[jj] >= 0 && k >= s_sp[jj] && k <= s_ep[jj]) s = jj;
    return s;
  };
  for (int q = start + t; q <= end; q += kFeatThreads) {
    const int s = sector_of(q);
    const int8_t l = s >= 0 ? fw.lab[(int64_t)s_slot[s] * cfg.sort_cap + (q - s_sp[s])] : (int8_t)0;
    labr[q - start] = l;
    out.label[q] = l;
  }
  // corners of this ring (sector order, pick order inside a sector)
  for (int q = t; q < s_cb[6]; q += kFeatThreads) {
    int s = 0;
    while (q >= s_cb[s + 1]) ++s;
    const int p = fw.var[s_slot[s]].corner[q - s_cb[s]];  // a ring position by construction
    out.corner_stage[(int64_t)r * kCornerPerRing + q] = rp[(p >= start && p <= end) ? p - start : 0];
    if (MODE == kModeLego) out.corner_sharp[(int64_t)r * kCornerPerRing + q] = (q - s_cb[s]) < 2;
  }
  if (MODE == kModeLego) {
    for (int q = t; q < s_fb[6]; q += kFeatThreads) {
      int s = 0;
      while (q >= s_fb[s + 1]) ++s;
      const int p = fw.var[s_slot[s]].flat[q - s_fb[s]];
      out.flat_stage[(int64_t)r * kFlatPerRing + q] = rp[(p >= start && p <= end) ? p - start : 0];
    }
  }
  __syncthreads();
  RGSTAMP(2);
  float4* dst = out.surf_stage + (start - 4);  // ring's first extracted index
  if (vm >= 0) {
    // presorted: keep the entries whose label is <= 0 (the surface list, in
    // VoxelGrid order), then the voxels' centroids below
    int cnt = 0;
#pragma unroll
    for (int i = 0; i < kVPer; ++i) {
      const int e = t * kVPer + i;
      cnt += e < vm && labr[(int)(uint32_t)vk[i] - start] <= 0;
    }
    int excl;
    const int mk = block_exclusive_scan<kFeatThreads>(cnt, scratch, excl);
#pragma unroll
    for (int i = 0; i < kVPer; ++i) {
      const int e = t * kVPer + i;
      if (e < vm && labr[(int)(uint32_t)vk[i] - start] <= 0) keys[excl++] = vk[i];
    }
    __syncthreads();
    RGSTAMP(3);
    if (mk == 0) {
      if (t == 0) out.surf_count[r] = 0;
      return;
    }
    ring_voxels<kFeatThreads>(keys, vp, rp, start, mk, dst, scratch, out.surf_count + r);
    RGSTAMP(7);
    return;
  }
  int m;
  {
    const int per = (end - start + 1 + kFeatThreads - 1) / kFeatThreads;
    const int q0 = start + t * per, q1 = min(q0 + per, end + 1);
    int cnt = 0;
    for (int k = q0; k < q1; ++k) cnt += sector_of(k) >= 0 && labr[k - start] <= 0;
    int excl;
    m = block_exclusive_scan<kFeatThreads>(cnt, scratch, excl);
    for (int k = q0; k < q1; ++k)
      if (sector_of(k) >= 0 && labr[k - start] <= 0) slist[excl++] = k;
  }
  __syncthreads();
  RGSTAMP(3);
  if (m == 0) {
    if (t == 0) out.surf_count[r] = 0;
    return;
  }
  {
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int q = t; q < m; q += kFeatThreads) {
      const float4 p = rp[slist[q] - start];
      mn[0] = fminf(mn[0], p.x);
      mn[1] = fminf(mn[1], p.y);
      mn[2] = fminf(mn[2], p.z);
      mx[0] = fmaxf(mx[0], p.x);
      mx[1] = fmaxf(mx[1], p.y);
      mx[2] = fmaxf(mx[2], p.z);
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) {
        mn[a] = fminf(mn[a], __shfl_xor(mn[a], o, 64));
        mx[a] = fmaxf(mx[a], __shfl_xor(mx[a], o, 64));
      }
    }
    __shared__ float wmn[kFeatThreads / 64][3], wmx[kFeatThreads / 64][3];
    if (lane == 0)
      for (int a = 0; a < 3; ++a) {
        wmn[w][a] = mn[a];
        wmx[w][a] = mx[a];
      }
    __syncthreads();
    if (t == 0) {
      for (int a = 0; a < 3; ++a) {
        float a0 = wmn[0][a], a1 = wmx[0][a];
        for (int q = 1; q < kFeatThreads / 64; ++q) {
          a0 = fminf(a0, wmn[q][a]);
          a1 = fmaxf(a1, wmx[q][a]);
        }
        s_min[a] = a0;
        s_max[a] = a1;
      }
      const float inv = 1.0f / cfg.leaf;
      const int64_t dx = (int64_t)((s_max[0] - s_min[0]) * inv) + 1;
      const int64_t dy = (int64_t)((s_max[1] - s_min[1]) * inv) + 1;
      const int64_t dz = (int64_t)((s_max[2] - s_min[2]) * inv) + 1;
      s_overflow = dx * dy * dz > (int64_t)2147483647;
      int divb[3];
      for (int a = 0; a < 3; ++a) {
        s_minb[a] = (int)floorf(s_min[a] * inv);
        divb[a] = (int)floorf(s_max[a] * inv) - s_minb[a] + 1;
      }
      s_mul[0] = 1;
      s_mul[1] = divb[0];
      s_mul[2] = divb[0] * divb[1];
      // voxel indices lie below divb0 * divb1 * divb2: the sort needs only
      // that many low bits
      const uint32_t top = (uint32_t)((int64_t)divb[0] * divb[1] * divb[2] - 1);
      s_bits = top ? 32 - __clz((int)top) : 1;
    }
    __syncthreads();
  }
  RGSTAMP(4);
  if (s_overflow) {  // PCL: "Integer indices would overflow", output = input
    for (int q = t; q < m; q += kFeatThreads) dst[q] = rp[slist[q] - start];
    if (t == 0) out.surf_count[r] = m;
    return;
  }
  const float inv = 1.0f / cfg.leaf;
  // (voxel index, list index) keys: the bitonic sort (sort_keys_lds) is the
  // stable sort of the voxel indices over the list order.  When the voxel
  // index fits 32 - log2(VOXN) bits (the usual ring) the keys are 32-bit --
  // half the cross-lane traffic and one-instruction compares -- and widen to
  // the 64-bit (voxel << 32 | list index) layout after the sort.
  auto voxel_of = [&](int q) {
    const float4 p = rp[slist[q] - start];
    const int i0 = (int)(floorf(p.x * inv) - (float)s_minb[0]);
    const int i1 = (int)(floorf(p.y * inv) - (float)s_minb[1]);
    const int i2 = (int)(floorf(p.z * inv) - (float)s_minb[2]);
    return (uint32_t)(i0 * s_mul[0] + i1 * s_mul[1] + i2 * s_mul[2]);
  };
  constexpr int kQBits = __builtin_ctz(VOXN);
#ifdef SLIO_RING_NO_NARROW
  if (false) {
#else
  if (s_bits + kQBits <= 32) {
#endif
    uint32_t* k32 = reinterpret_cast<uint32_t*>(keys);
    for (int q = t; q < VOXN; q += kFeatThreads) k32[q] = q < m ? (voxel_of(q) << kQBits) | (uint32_t)q : ~0u;
    RGSTAMP(5);
    sort_keys_lds<kSortW, kSortE, uint32_t>(k32);
    constexpr int kHeld = (VOXN + kFeatThreads - 1) / kFeatThreads;
    uint32_t held[kHeld];
#pragma unroll
    for (int i = 0; i < kHeld; ++i) held[i] = t + i * kFeatThreads < VOXN ? k32[t + i * kFeatThreads] : 0u;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kHeld; ++i)
      if (t + i * kFeatThreads < VOXN)
        keys[t + i * kFeatThreads] = ((uint64_t)(held[i] >> kQBits) << 32) | (held[i] & (VOXN - 1));
    __syncthreads();
  } else {
    for (int q = t; q < VOXN; q += kFeatThreads)  // past the list: sorts last
      keys[q] = q < m ? ((uint64_t)voxel_of(q) << 32) | (uint32_t)q : ~0ull;
    RGSTAMP(5);
    sort_keys_lds<kSortW, kSortE>(keys);
  }
  // (the keys' low words become ring positions: the list entries' own)
  for (int q = t; q < m; q += kFeatThreads)
    keys[q] = (keys[q] & 0xFFFFFFFF00000000ull) | (uint32_t)slist[(uint32_t)keys[q]];
  __syncthreads();
  RGSTAMP(6);
  ring_voxels<kFeatThreads>(keys, vp, rp, start, m, dst, scratch, out.surf_count + r);
  RGSTAMP(7);
}

// dynamic LDS of the feature kernels
struct FeatSmem {
  size_t pick, ring;
};
inline FeatSmem feat_smem_sizes(const FeatCfg& fc) {
  const size_t pcap = (size_t)fc.sort_cap + kPickPad;
  // (k_fe_pick's 7th workgroup per ring sorts kVsortN pairs in the same LDS;
  // both sorts: two key / value buffers and 256 counters per wavefront)
  const size_t rcnt = sizeof(int) * 256 * (kPickThreads / 64);
  return FeatSmem{std::max(16 * (size_t)fc.sort_cap + rcnt + (4 + 4 + 4 + 1 + 1 + 1 + 1 + 6 * 2) * pcap,
                           16 * (size_t)kVsortN + rcnt),
                  24 * (size_t)fc.vox_cap + 21 * (size_t)fc.ring_cap};
}
// the sorts' sizes (powers of two; 0: capacity not supported)
inline int sort_items(int sort_cap) {
  return (sort_cap >= 64 && sort_cap <= 2048 && (sort_cap & (sort_cap - 1)) == 0) ? sort_cap : 0;
}
inline int vox_items(int vox_cap) {
  return (vox_cap >= 64 && vox_cap <= 4096 && (vox_cap & (vox_cap - 1)) == 0) ? vox_cap : 0;
}

inline hipError_t feat_work_alloc(FeatWork& fw, int R, const FeatCfg& fc) {
  hipError_t e = hipSuccess;
  auto A = [&](auto*& p, size_t bytes) {
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&p), bytes);
  };
  A(fw.spos, 4 * (size_t)6 * R * fc.sort_cap);
  A(fw.var, sizeof(PickVar) * 36 * (size_t)R);
  A(fw.lab, (size_t)36 * R * fc.sort_cap);
  A(fw.vkey, sizeof(uint64_t) * kVsortN * (size_t)R);
  A(fw.vinfo, sizeof(int32_t) * (size_t)R);
  return e;
}

inline void feat_work_free(FeatWork& fw) {
  void* p[] = {fw.spos, fw.var, fw.lab, fw.vkey, fw.vinfo};
  for (void* q : p)
    if (q) (void)hipFree(q);
  fw = FeatWork{};
}

template <int MODE>
inline const void* ring_kernel(int vn) {
  switch (vn) {
    case 64: return (const void*)k_fe_ring<MODE, 64>;
    case 128: return (const void*)k_fe_ring<MODE, 128>;
    case 256: return (const void*)k_fe_ring<MODE, 256>;
    case 512: return (const void*)k_fe_ring<MODE, 512>;
    case 1024: return (const void*)k_fe_ring<MODE, 1024>;
    case 2048: return (const void*)k_fe_ring<MODE, 2048>;
    default: return (const void*)k_fe_ring<MODE, 4096>;
  }
}

template <int MODE>
inline const void* pick_kernel(int sn) {
  switch (sn) {
    case 64: return (const void*)k_fe_pick<MODE, 64>;
    case 128: return (const void*)k_fe_pick<MODE, 128>;
    case 256: return (const void*)k_fe_pick<MODE, 256>;
    case 512: return (const void*)k_fe_pick<MODE, 512>;
    case 1024: return (const void*)k_fe_pick<MODE, 1024>;
    default: return (const void*)k_fe_pick<MODE, 2048>;
  }
}

// kernels whose LDS may exceed the 64 KB default
template <int MODE>
inline void feat_set_smem(const FeatSmem& s, int sitems, int vitems) {
  if (s.pick > 32 * 1024)
    (void)hipFuncSetAttribute(pick_kernel<MODE>(sitems), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)s.pick);
  if (s.ring > 32 * 1024)
    (void)hipFuncSetAttribute(ring_kernel<MODE>(vitems), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)s.ring);
}

// extractFeatures + per-ring VoxelGrid: 2 launches; ev brackets them (the
// front-end bench's feature-stage timing)
template <int MODE>
inline void launch_features(hipStream_t s, int R, const CloudInfo& ci, float* curv,
                            uint8_t* picked0, const FeatCfg& fc, const FeatOut& fo,
                            const FeatWork& fw, std::pair<hipEvent_t, hipEvent_t> ev) {
  const FeatSmem sm = feat_smem_sizes(fc);
  const dim3 gs(7, R);  // 6 sectors + the ring's VoxelGrid order (ring_vsort)
  const uint32_t ps = (uint32_t)sm.pick;
  const uint8_t* gr = fo.ground;
#define SLIO_PICK(N)                                                                                     \
  case N:                                                                                              \
    hipExtLaunchKernelGGL((k_fe_pick<MODE, N>), gs, dim3(kPickThreads), ps, s, ev.first, nullptr, 0, ci, \
                          curv, picked0, fo.label, gr, fc, fw);                                        \
    break
  switch (sort_items(fc.sort_cap)) {
    SLIO_PICK(64);
    SLIO_PICK(128);
    SLIO_PICK(256);
    SLIO_PICK(512);
    SLIO_PICK(1024);
    default: SLIO_PICK(2048);
  }
#undef SLIO_PICK
  const uint32_t rs = (uint32_t)sm.ring;
#define SLIO_RING(N)                                                                                          \
  case N:                                                                                                   \
    hipExtLaunchKernelGGL((k_fe_ring<MODE, N>), dim3(R), dim3(kFeatThreads), rs, s, nullptr, ev.second, 0, ci, \
                          fc, fo, fw);                                                                      \
    break
  switch (vox_items(fc.vox_cap)) {
    SLIO_RING(64);
    SLIO_RING(128);
    SLIO_RING(256);
    SLIO_RING(512);
    SLIO_RING(1024);
    SLIO_RING(2048);
    default: SLIO_RING(4096);
  }
#undef SLIO_RING
}

// sum of cnt[0 .. r) by one wavefront (lanes take rings lane, lane + 64, ...),
// every lane of the wavefront gets it
__device__ __forceinline__ int wave_prefix_count(const int32_t* cnt, int r) {
  const int lane = threadIdx.x & 63;
  int v = 0;
  for (int q = lane; q < r; q += 64) v += cnt[q];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

constexpr int kConcatThreads = 1024;
__global__ __launch_bounds__(kConcatThreads) void k_lio_concat(int n_scan, const int32_t* start_ring,
                                                               FeatOut f, float4* corner, float4* surface,
                                                               int64_t* counts /* n_corner, n_surface */) {
  __shared__ int s_co, s_so;
  const int r = blockIdx.x, w = threadIdx.x >> 6;
  // ring offsets: wavefront 0 the corners', wavefront 1 the surfaces'
  if (w < 2) {
    const int o = wave_prefix_count(w == 0 ? f.corner_count : f.surf_count, r);
    if ((threadIdx.x & 63) == 0) {
      if (w == 0)
        s_co = o;
      else
        s_so = o;
      if (r == n_scan - 1) counts[w] = o + (w == 0 ? f.corner_count[r] : f.surf_count[r]);
    }
  }
  __syncthreads();
  const int nc = f.corner_count[r], ns = f.surf_count[r];
  for (int q = threadIdx.x; q < nc; q += kConcatThreads)
    corner[s_co + q] = f.corner_stage[(int64_t)r * kCornerPerRing + q];
  const float4* src = f.surf_stage + (start_ring[r] - 4);
  for (int q = threadIdx.x; q < ns; q += kConcatThreads) surface[s_so + q] = src[q];
}

}  // namespace lio
}  // namespace slio

using namespace slio;
using namespace slio::lio;

struct slio_lio {
  bool dev_counted = false;  // counted in slio::dev_users
  slio_lio_params prm{};
  Geo g{};
  hipStream_t own = nullptr, stream = nullptr;
  int64_t cap = 0, cells = 0;
  // input
  float *x = nullptr, *y = nullptr, *z = nullptr, *in = nullptr, *time = nullptr;
  uint16_t* ring = nullptr;
  int64_t n = 0;
  // deskew
  double *it = nullptr, *rx = nullptr, *ry = nullptr, *rz = nullptr;
  int n_imu = 0;
  double t0 = 0.0;
  int deskew = 0;
  int imu_sorted = 0;  // the deskew table's times are non-decreasing
  // projection
  unsigned long long* owner = nullptr;  // cells + 1: (~generation << 32) | point index
  uint32_t gen = 0;                      // scans run (owner generation)
  float* range_mat = nullptr;
  float4* full = nullptr;
  int32_t* row_count = nullptr;     // n_scan * kFillSplit partial counts
  uint32_t* block_first = nullptr;  // per claim block: smallest valid point index
  // cloud_info
  int32_t *start_ring = nullptr, *end_ring = nullptr, *col_ind = nullptr, *n_ext = nullptr;
  float* prange = nullptr;
  float4* xyzi = nullptr;
  // features
  float* curvature = nullptr;
  uint8_t* picked0 = nullptr;
  int32_t* label = nullptr;
  float4* corner_stage = nullptr;
  int32_t* corner_count = nullptr;
  float4* surf_stage = nullptr;
  int32_t* surf_count = nullptr;
  float4* corner = nullptr;
  float4* surface = nullptr;
  int64_t* counts = nullptr;  // device: n_corner, n_surface
  int64_t* h_counts = nullptr;  // pinned: n_ext, n_corner, n_surface
  FeatCfg fc{};
  FeatWork fw{};
  bool ran = false;
  // feature-stage timing
  bool prof = false;
  bool prof_scan = false;  // SLIO_LIO_PROFILE_SCAN: the events span the whole scan
  double prof_ms = 0.0;
  int64_t prof_n = 0;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending, pool;
};

namespace {

void lio_prof_drain(slio_lio* h) {
  for (auto& p : h->pending) {
    float ms = 0.f;
    if (hipEventSynchronize(p.second) == hipSuccess &&
        hipEventElapsedTime(&ms, p.first, p.second) == hipSuccess) {
      h->prof_ms += ms;
      h->prof_n += 1;
    }
    h->pool.push_back(p);
  }
  h->pending.clear();
}

void lio_free(slio_lio* h) {
  lio_prof_drain(h);
  for (auto& p : h->pool) {
    (void)hipEventDestroy(p.first);
    (void)hipEventDestroy(p.second);
  }
  void* dev[] = {h->x, h->y, h->z, h->in, h->time, h->ring, h->it, h->rx, h->ry, h->rz,
                 h->owner, h->range_mat, h->full, h->row_count, h->block_first,
                 h->start_ring, h->end_ring,
                 h->col_ind, h->n_ext, h->prange, h->xyzi, h->curvature, h->picked0, h->label,
                 h->corner_stage, h->corner_count, h->surf_stage, h->surf_count, h->corner,
                 h->surface, h->counts};
  for (void* p : dev)
    if (p) (void)hipFree(p);
  feat_work_free(h->fw);
  if (h->h_counts) (void)hipHostFree(h->h_counts);
  if (h->own) (void)hipStreamDestroy(h->own);
}

#define LIO_CHECK_H(h)                    \
  do {                                    \
    if (!(h)) {                           \
      set_error("null slio_lio handle");  \
      return SLIO_EINVAL;                 \
    }                                     \
    LIO_HIP(hipSetDevice((h)->prm.device)); \
  } while (0)

}  // namespace

extern "C" {

#ifdef SLIO_FE_STAMP
int slio_dbg_fe_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fstamp), sizeof(g_fstamp)) == hipSuccess ? 0 : -1;
}
int slio_dbg_ring_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rstamp), sizeof(g_rstamp)) == hipSuccess ? 0 : -1;
}
#endif

int slio_lio_params_default(slio_lio_params* p) {
  if (!p) return SLIO_EINVAL;
  std::memset(p, 0, sizeof(*p));
  p->n_scan = 16;
  p->horizon_scan = 1800;
  p->downsample_rate = 1;
  p->lidar_min_range = 1.0f;
  p->lidar_max_range = 1000.0f;
  p->edge_threshold = 1.0f;
  p->surf_threshold = 0.1f;
  p->surf_leaf_size = 0.4f;
  return SLIO_OK;
}

int slio_lio_create(slio_lio_handle* out, const slio_lio_params* p) {
  if (!out || !p) {
    set_error("slio_lio_create: null argument");
    return SLIO_EINVAL;
  }
  *out = nullptr;
  if (p->n_scan <= 0 || p->horizon_scan <= 0 || p->horizon_scan > 65536 || p->downsample_rate <= 0 ||
      !(p->surf_leaf_size > 0.0f) || p->max_points < 0 || p->n_scan > 65535) {
    set_error("slio_lio_create: bad n_scan / horizon_scan / downsample_rate / leaf / max_points");
    return SLIO_EINVAL;
  }
  int ndev = 0;
  LIO_HIP(hipGetDeviceCount(&ndev));
  if (p->device < 0 || p->device >= ndev) {
    set_error("slio_lio_create: no such HIP device");
    return SLIO_EDEVICE;
  }
  LIO_HIP(hipSetDevice(p->device));
  auto* h = new slio_lio();
  h->prm = *p;
  h->cells = (int64_t)p->n_scan * p->horizon_scan;
  h->cap = p->max_points > 0 ? p->max_points : h->cells;
  h->g = Geo{p->n_scan, p->horizon_scan, p->downsample_rate, p->lidar_min_range,
             p->lidar_max_range, (float)(360.0 / float(p->horizon_scan)), h->cells};
  const int64_t C = h->cells, N = h->cap;
  hipError_t e = hipStreamCreateWithFlags(&h->own, hipStreamNonBlocking);
  h->stream = h->own;
#define A(ptr, bytes) \
  if (!e) e = hipMalloc(reinterpret_cast<void**>(&(ptr)), (bytes))
  A(h->x, 4 * N);
  A(h->y, 4 * N);
  A(h->z, 4 * N);
  A(h->in, 4 * N);
  A(h->time, 4 * N);
  A(h->ring, 2 * N);
  A(h->it, 8 * kMaxImu);
  A(h->rx, 8 * kMaxImu);
  A(h->ry, 8 * kMaxImu);
  A(h->rz, 8 * kMaxImu);
  A(h->owner, 8 * (C + 1));
  A(h->range_mat, 4 * C);
  A(h->full, 16 * C);
  A(h->row_count, 4 * p->n_scan * kFillSplit);
  A(h->block_first, 4 * ((N + 255) / 256 + 1));
  A(h->start_ring, 4 * p->n_scan);
  A(h->end_ring, 4 * p->n_scan);
  A(h->col_ind, 4 * C);
  A(h->n_ext, 4);
  A(h->prange, 4 * C);
  A(h->xyzi, 16 * C);
  A(h->curvature, 4 * C);
  A(h->picked0, C);
  A(h->label, 4 * C);
  A(h->corner_stage, 16 * (int64_t)p->n_scan * kCornerPerRing);
  A(h->corner_count, 4 * p->n_scan);
  A(h->surf_stage, 16 * C);
  A(h->surf_count, 4 * p->n_scan);
  A(h->corner, 16 * (int64_t)p->n_scan * kCornerPerRing);
  A(h->surface, 16 * C);
  A(h->counts, 16);
#undef A
  if (!e) e = hipHostMalloc(reinterpret_cast<void**>(&h->h_counts), 3 * sizeof(int64_t));
  if (e) {
    set_error(std::string("slio_lio_create: ") + hipGetErrorString(e));
    lio_free(h);
    delete h;
    return SLIO_ENOMEM;
  }
  const int H = p->horizon_scan;
  h->fc.edge_thr = p->edge_threshold;
  h->fc.surf_thr = p->surf_threshold;
  h->fc.leaf = p->surf_leaf_size;
  h->fc.sort_cap = 64;
  while (h->fc.sort_cap < H / 6 + 2) h->fc.sort_cap <<= 1;
  h->fc.vox_cap = 64;
  while (h->fc.vox_cap < H) h->fc.vox_cap <<= 1;
  h->fc.ring_cap = H + 16;
  const FeatSmem fsm = feat_smem_sizes(h->fc);
  if (std::max(fsm.pick, fsm.ring) > 96 * 1024 || !sort_items(h->fc.sort_cap) ||
      !vox_items(h->fc.vox_cap)) {
    set_error("slio_lio_create: horizon_scan too large for the feature kernels' LDS layout");
    lio_free(h);
    delete h;
    return SLIO_EINVAL;
  }
  e = feat_work_alloc(h->fw, p->n_scan, h->fc);
  if (e) {
    set_error(std::string("slio_lio_create: ") + hipGetErrorString(e));
    lio_free(h);
    delete h;
    return SLIO_ENOMEM;
  }
  feat_set_smem<kModeLio>(fsm, sort_items(h->fc.sort_cap), vox_items(h->fc.vox_cap));
  h->dev_counted = true;
  slio::dev_users(h->prm.device, +1);
  *out = h;
  return SLIO_OK;
}

int slio_lio_destroy(slio_lio_handle h) {
  if (!h) return SLIO_OK;
  (void)hipSetDevice(h->prm.device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  lio_free(h);
  if (h->dev_counted) slio::dev_users(h->prm.device, -1);
  delete h;
  return SLIO_OK;
}

int slio_lio_set_stream(slio_lio_handle h, void* stream) {
  LIO_CHECK_H(h);
  h->stream = stream ? (hipStream_t)stream : h->own;
  return SLIO_OK;
}

int slio_lio_set_deskew(slio_lio_handle h, const double* imu_time, const double* rot_x,
                        const double* rot_y, const double* rot_z, int32_t n_imu,
                        double time_scan_cur, int32_t enabled) {
  LIO_CHECK_H(h);
  if (enabled && (n_imu < 1 || n_imu > kMaxImu || !imu_time || !rot_x || !rot_y || !rot_z)) {
    set_error("slio_lio_set_deskew: need 1 <= n_imu <= 2000 and all four tables");
    return SLIO_EINVAL;
  }
  h->deskew = enabled ? 1 : 0;
  h->n_imu = enabled ? n_imu : 0;
  h->t0 = time_scan_cur;
  h->imu_sorted = 1;
  for (int k = 1; enabled && k < n_imu; ++k)
    if (!(imu_time[k - 1] <= imu_time[k])) h->imu_sorted = 0;
  if (enabled) {
    LIO_HIP(hipMemcpyAsync(h->it, imu_time, 8 * n_imu, hipMemcpyHostToDevice, h->stream));
    LIO_HIP(hipMemcpyAsync(h->rx, rot_x, 8 * n_imu, hipMemcpyHostToDevice, h->stream));
    LIO_HIP(hipMemcpyAsync(h->ry, rot_y, 8 * n_imu, hipMemcpyHostToDevice, h->stream));
    LIO_HIP(hipMemcpyAsync(h->rz, rot_z, 8 * n_imu, hipMemcpyHostToDevice, h->stream));
    LIO_HIP(hipStreamSynchronize(h->stream));  // host tables may be freed on return
  }
  return SLIO_OK;
}

int slio_lio_upload(slio_lio_handle h, const float* x, const float* y, const float* z,
                    const float* intensity, const uint16_t* ring, const float* time, int64_t n) {
  LIO_CHECK_H(h);
  if (n < 0 || (n > 0 && (!x || !y || !z || !intensity || !ring || !time))) {
    set_error("slio_lio_upload: bad arguments");
    return SLIO_EINVAL;
  }
  if (n > h->cap || n >= (int64_t)kNone) {
    set_error("slio_lio_upload: scan exceeds max_points");
    return SLIO_ECAPACITY;
  }
  h->n = n;
  if (n > 0) {
    LIO_HIP(hipMemcpyAsync(h->x, x, 4 * n, hipMemcpyHostToDevice, h->stream));
    LIO_HIP(hipMemcpyAsync(h->y, y, 4 * n, hipMemcpyHostToDevice, h->stream));
    LIO_HIP(hipMemcpyAsync(h->z, z, 4 * n, hipMemcpyHostToDevice, h->stream));
    LIO_HIP(hipMemcpyAsync(h->in, intensity, 4 * n, hipMemcpyHostToDevice, h->stream));
    LIO_HIP(hipMemcpyAsync(h->ring, ring, 2 * n, hipMemcpyHostToDevice, h->stream));
    LIO_HIP(hipMemcpyAsync(h->time, time, 4 * n, hipMemcpyHostToDevice, h->stream));
    LIO_HIP(hipStreamSynchronize(h->stream));
  }
  h->ran = false;
  return SLIO_OK;
}

int slio_lio_run_async(slio_lio_handle h) {
  LIO_CHECK_H(h);
  const Geo& g = h->g;
  const int R = g.n_scan;
  if (h->gen == 0 || h->gen == 0xFFFFFFFEu) {  // first scan, or the generation wraps
    LIO_HIP(hipMemsetAsync(h->owner, 0xff, 8 * g.cells, h->stream));
    h->gen = 0;
  }
  const uint32_t hi = ~(++h->gen);
  const In in{h->x, h->y, h->z, h->in, h->ring, h->time, h->n};
  const int nclaim = (int)((h->n + 255) / 256);
  std::pair<hipEvent_t, hipEvent_t> ev{nullptr, nullptr};
  if (h->prof) {
    if (h->pending.size() > 256) lio_prof_drain(h);
    if (!h->pool.empty()) {
      ev = h->pool.back();
      h->pool.pop_back();
    } else {
      LIO_HIP(hipEventCreate(&ev.first));
      LIO_HIP(hipEventCreate(&ev.second));
    }
    h->pending.push_back(ev);
  }
  // the events: in the first and last launches' dispatch packets (the whole
  // scan), or around the feature stage
  const hipEvent_t e0 = h->prof_scan ? ev.first : nullptr, e1 = h->prof_scan ? ev.second : nullptr;
  if (h->n > 0)
    hipExtLaunchKernelGGL(k_lio_claim, dim3(nclaim), dim3(256), 0, h->stream, e0, nullptr, 0, in, g, h->owner, hi,
                          h->block_first);
  const Deskew d{h->it, h->rx, h->ry, h->rz, h->n_imu - 1, h->t0, h->deskew, h->imu_sorted};
  hipExtLaunchKernelGGL(k_lio_fill, dim3(R, kFillSplit), dim3(kFillThreads), 0, h->stream,
                        h->n > 0 ? nullptr : e0, nullptr, 0, in, g, h->owner, hi, h->block_first, nclaim, d,
                        h->range_mat, h->full, h->row_count);
  const CloudInfo ci{h->start_ring, h->end_ring, h->col_ind, h->prange, h->xyzi, h->n_ext};
  k_lio_extract<<<R, kRowThreads, 0, h->stream>>>(g, h->range_mat, h->full, h->row_count, ci);
  const FeatOut fo{h->label, h->corner_stage, h->corner_count, h->surf_stage, h->surf_count,
                   nullptr, nullptr, nullptr, nullptr, nullptr};
  launch_features<kModeLio>(h->stream, R, ci, h->curvature, h->picked0, h->fc, fo, h->fw,
                            h->prof_scan ? std::pair<hipEvent_t, hipEvent_t>{nullptr, nullptr} : ev);
  hipExtLaunchKernelGGL(k_lio_concat, dim3(R), dim3(kConcatThreads), 0, h->stream, nullptr, e1, 0, R,
                        h->start_ring, fo, h->corner, h->surface, h->counts);
  LIO_HIP(hipGetLastError());
  h->ran = true;
  return SLIO_OK;
}

int slio_lio_profile(slio_lio_handle h, int enable) {
  LIO_CHECK_H(h);
  const bool keep = (enable & SLIO_LIO_PROFILE_KEEP) != 0;
  h->prof = (enable & ~SLIO_LIO_PROFILE_KEEP) != 0;
  h->prof_scan = (enable & SLIO_LIO_PROFILE_SCAN) != 0;
  if (!keep) {  // pausing / resuming never waits; a reset drains first
    lio_prof_drain(h);
    h->prof_ms = 0.0;
    h->prof_n = 0;
  }
  return SLIO_OK;
}

int slio_lio_profile_read(slio_lio_handle h, double* ms, int64_t* launches) {
  LIO_CHECK_H(h);
  LIO_HIP(hipStreamSynchronize(h->stream));
  lio_prof_drain(h);
  if (ms) *ms = h->prof_ms;
  if (launches) *launches = h->prof_n;
  return SLIO_OK;
}

int slio_lio_get_counts(slio_lio_handle h, slio_lio_counts* c) {
  LIO_CHECK_H(h);
  if (!h->ran) {
    set_error("slio_lio: no scan processed");
    return SLIO_ESTATE;
  }
  int32_t ne = 0;
  LIO_HIP(hipMemcpyAsync(h->h_counts + 1, h->counts, 16, hipMemcpyDeviceToHost, h->stream));
  LIO_HIP(hipMemcpyAsync(&ne, h->n_ext, 4, hipMemcpyDeviceToHost, h->stream));
  LIO_HIP(hipStreamSynchronize(h->stream));
  h->h_counts[0] = ne;
  if (c) {
    c->n_extracted = h->h_counts[0];
    c->n_corner = h->h_counts[1];
    c->n_surface = h->h_counts[2];
  }
  return SLIO_OK;
}

int slio_lio_run(slio_lio_handle h, slio_lio_counts* c) {
  const int rc = slio_lio_run_async(h);
  if (rc) return rc;
  return slio_lio_get_counts(h, c);
}

int slio_lio_get_range_image(slio_lio_handle h, float* range_mat, int32_t* cell_point) {
  LIO_CHECK_H(h);
  if (!h->ran) {
    set_error("slio_lio: no scan processed");
    return SLIO_ESTATE;
  }
  if (range_mat)
    LIO_HIP(hipMemcpyAsync(range_mat, h->range_mat, 4 * h->cells, hipMemcpyDeviceToHost, h->stream));
  std::vector<unsigned long long> own(cell_point ? (size_t)h->cells : 0);
  if (cell_point)
    LIO_HIP(hipMemcpyAsync(own.data(), h->owner, 8 * h->cells, hipMemcpyDeviceToHost, h->stream));
  LIO_HIP(hipStreamSynchronize(h->stream));
  const uint32_t hi = ~h->gen;
  for (size_t c = 0; c < own.size(); ++c)  // a cell of an older scan is empty: -1
    cell_point[c] = (uint32_t)(own[c] >> 32) == hi ? (int32_t)(uint32_t)own[c] : -1;
  return SLIO_OK;
}

int slio_lio_get_cloud_info(slio_lio_handle h, int32_t* start_ring, int32_t* end_ring,
                            int32_t* col_ind, float* point_range, float* xyzi) {
  slio_lio_counts c;
  const int rc = slio_lio_get_counts(h, &c);
  if (rc) return rc;
  const int64_t n = c.n_extracted, R = h->g.n_scan;
  if (start_ring) LIO_HIP(hipMemcpyAsync(start_ring, h->start_ring, 4 * R, hipMemcpyDeviceToHost, h->stream));
  if (end_ring) LIO_HIP(hipMemcpyAsync(end_ring, h->end_ring, 4 * R, hipMemcpyDeviceToHost, h->stream));
  if (n > 0) {
    if (col_ind) LIO_HIP(hipMemcpyAsync(col_ind, h->col_ind, 4 * n, hipMemcpyDeviceToHost, h->stream));
    if (point_range) LIO_HIP(hipMemcpyAsync(point_range, h->prange, 4 * n, hipMemcpyDeviceToHost, h->stream));
    if (xyzi) LIO_HIP(hipMemcpyAsync(xyzi, h->xyzi, 16 * n, hipMemcpyDeviceToHost, h->stream));
  }
  LIO_HIP(hipStreamSynchronize(h->stream));
  return SLIO_OK;
}

int slio_lio_get_features(slio_lio_handle h, float* curvature, uint8_t* picked, int32_t* label) {
  slio_lio_counts c;
  const int rc = slio_lio_get_counts(h, &c);
  if (rc) return rc;
  const int64_t n = c.n_extracted;
  if (n > 0) {
    if (curvature) LIO_HIP(hipMemcpyAsync(curvature, h->curvature, 4 * n, hipMemcpyDeviceToHost, h->stream));
    if (picked) LIO_HIP(hipMemcpyAsync(picked, h->picked0, n, hipMemcpyDeviceToHost, h->stream));
    if (label) LIO_HIP(hipMemcpyAsync(label, h->label, 4 * n, hipMemcpyDeviceToHost, h->stream));
  }
  LIO_HIP(hipStreamSynchronize(h->stream));
  return SLIO_OK;
}

int slio_lio_get_clouds(slio_lio_handle h, float* corner_xyzi, float* surface_xyzi) {
  slio_lio_counts c;
  const int rc = slio_lio_get_counts(h, &c);
  if (rc) return rc;
  if (corner_xyzi && c.n_corner > 0)
    LIO_HIP(hipMemcpyAsync(corner_xyzi, h->corner, 16 * c.n_corner, hipMemcpyDeviceToHost, h->stream));
  if (surface_xyzi && c.n_surface > 0)
    LIO_HIP(hipMemcpyAsync(surface_xyzi, h->surface, 16 * c.n_surface, hipMemcpyDeviceToHost, h->stream));
  LIO_HIP(hipStreamSynchronize(h->stream));
  return SLIO_OK;
}

}  // extern "C"


// ======================================================================
// LeGO-LOAM.  One scan = 14 launches:
//   memsets (cell owners, ground, component stats)
//   k_lego_claim     per point   projectPointCloud: row from the vertical
//                                angle, the LAST point wins (atomicMax, :177-213)
//   k_lego_fill      per cell    rangeMat / fullCloud (intensity row + col/1e4)
//   k_lego_ground    per column  groundRemoval, sequential over the ground rows
//                                as the reference loop (:216-262), labelMat -1
//   k_lego_union     per cell    labelComponents as connected components: the
//                                BFS edge test (:355-372) is symmetric, so BFS
//                                visits exactly a component; lock-free
//                                union-find linking to the smaller index, so a
//                                root is the component's first row-major cell
//   k_lego_compress  per cell    roots, component size, rows of its pushed cells
//   k_lego_rowcount  per ring    feasible roots / segmented / outlier counts
//   k_lego_extract   per ring    labelCount order of feasible roots, cloud_info,
//                                segmented + outlier clouds (:268-330)
//   k_lego_label     per cell    labelMat (label, 999999 or -1)
//   k_lego_half      per point   adjustDistortion's halfPassed switch point
//   k_lego_deskew    per point   adjustDistortion (:617-805)
//   k_fe_pick<kModeLego>  calculateSmoothness + markOccludedPoints +
//                         extractFeatures (:883-1007); VoxelGrid order
//   k_fe_ring<kModeLego>  variant chain, labels, VoxelGrid 0.2
//   k_lego_concat    per ring    sharp / less sharp / flat / less flat clouds
// ======================================================================
namespace slio {
namespace lego {
using namespace slio::lio;

struct LGeo {
  int N, H, gsi, vpn, vln;
  float res_x, res_y, bottom, mount, theta;
  float sX, cX, sY, cY;  // sin / cos of segmentAlphaX / segmentAlphaY
  int64_t cells;
};

__device__ __forceinline__ bool lego_row(const LGeo& g, float x, float y, float z, int& row) {
  // verticalAngle; rowIdn is a size_t: the quotient truncates toward zero,
  // (-1, 0) -> 0, <= -1 or NaN wraps out of range (imageProjection.cpp:180-182)
  const float va = (float)((double)(fatan2(z, sqrtf(x * x + y * y)) * 180.0f) / M_PI);
  const float q = (va + g.bottom) / g.res_y;
  if (!(q > -1.0f) || !(q < (float)g.N)) return false;
  row = (int)q;
  return row < g.N;
}

__device__ __forceinline__ bool lego_col(const LGeo& g, float x, float y, int& col) {
  const float ha = (float)((double)(fatan2(x, y) * 180.0f) / M_PI);
  int64_t c = (int64_t)(-round(((double)ha - 90.0) / (double)g.res_x) + (double)(g.H / 2));
  if (c >= g.H) c -= g.H;
  if (c < 0 || c >= g.H) return false;
  col = (int)c;
  return true;
}

__global__ __launch_bounds__(256) void k_lego_claim(const float* __restrict__ x,
                                                    const float* __restrict__ y,
                                                    const float* __restrict__ z, int64_t n, LGeo g,
                                                    int32_t* owner) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  int row, col;
  if (!lego_row(g, x[i], y[i], z[i], row) || !lego_col(g, x[i], y[i], col)) return;
  atomicMax(&owner[col + (int64_t)row * g.H], (int32_t)i);
}

__global__ __launch_bounds__(256) void k_lego_fill(const float* __restrict__ x,
                                                   const float* __restrict__ y,
                                                   const float* __restrict__ z, LGeo g,
                                                   const int32_t* owner, float* range_mat,
                                                   float4* full, int8_t* ground) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= g.cells) return;
  ground[c] = 0;  // k_lego_ground sets the ground rows' flags
  const int o = owner[c];
  if (o < 0) {
    range_mat[c] = FLT_MAX;
    full[c] = make_float4(0.f, 0.f, 0.f, -1.0f);  // nanPoint's intensity (:65-68)
    return;
  }
  const float px = x[o], py = y[o], pz = z[o];
  const int row = (int)(c / g.H), col = (int)(c - (int64_t)row * g.H);
  range_mat[c] = sqrtf(px * px + py * py + pz * pz);
  full[c] = make_float4(px, py, pz, (float)((double)(float)row + (double)(float)col / 10000.0));
}

// groundRemoval per column (:216-262): the ground rows' cells and points are
// read up front (one round trip instead of one per row: the loop's flag
// stores could alias the loads), the flags formed in registers in the
// reference's row order, then stored.  init_parent: the union-find roots of
// the global labelComponents kernels (k_lego_cc sets its own).
constexpr int kLegoGroundRows = 16;
__global__ __launch_bounds__(256) void k_lego_ground(LGeo g, const int32_t* __restrict__ owner,
                                                     const float4* __restrict__ full, int8_t* __restrict__ ground,
                                                     int32_t* __restrict__ parent, bool init_parent) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= g.H) return;
  auto ground_test = [&](const float4& a, const float4& b) {
    const float dx = b.x - a.x, dy = b.y - a.y, dz = b.z - a.z;
    const float angle = (float)((double)(fatan2(dz, sqrtf(dx * dx + dy * dy)) * 180.0f) / M_PI);
    return fabsf(angle - g.mount) <= 10;
  };
  if (g.gsi < kLegoGroundRows) {
    int own[kLegoGroundRows + 1];
    float4 f[kLegoGroundRows + 1];
    int8_t gr[kLegoGroundRows + 1];
#pragma unroll
    for (int i = 0; i <= kLegoGroundRows; ++i) {
      own[i] = i <= g.gsi ? owner[j + (int64_t)i * g.H] : -1;
      gr[i] = 0;
    }
#pragma unroll
    for (int i = 0; i <= kLegoGroundRows; ++i)
      f[i] = (i <= g.gsi && own[i] >= 0) ? full[j + (int64_t)i * g.H] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < kLegoGroundRows; ++i) {
      if (i < g.gsi) {
        if (own[i] < 0 || own[i + 1] < 0) {
          gr[i] = -1;
        } else if (ground_test(f[i], f[i + 1])) {
          gr[i] = 1;
          gr[i + 1] = 1;
        }
      }
    }
#pragma unroll
    for (int i = 0; i <= kLegoGroundRows; ++i)
      if (i <= g.gsi && gr[i] != 0) ground[j + (int64_t)i * g.H] = gr[i];
  } else {
    for (int i = 0; i < g.gsi; ++i) {
      const int64_t lo = j + (int64_t)i * g.H, up = lo + g.H;
      if (owner[lo] < 0 || owner[up] < 0) {
        ground[lo] = -1;
        continue;
      }
      if (ground_test(full[lo], full[up])) {
        ground[lo] = 1;
        ground[up] = 1;
      }
    }
  }
  if (!init_parent) return;
  // labelMat = -1 for ground and empty cells (:247-254); the rest start as
  // their own union-find roots
  for (int i = 0; i < g.N; ++i) {
    const int64_t c = j + (int64_t)i * g.H;
    parent[c] = (ground[c] == 1 || owner[c] < 0) ? -1 : (int32_t)c;
  }
}

__device__ __forceinline__ int32_t ld_parent(const int32_t* p, int64_t i) {
  return __hip_atomic_load(p + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// parent pointers only ever move to smaller indices, so every chain ends
__device__ __forceinline__ int32_t uf_find(const int32_t* parent, int32_t x) {
  while (true) {
    const int32_t p = ld_parent(parent, x);
    if (p == x) return x;
    x = p;
  }
}

__device__ void uf_unite(int32_t* parent, int32_t a, int32_t b) {
  while (true) {
    a = uf_find(parent, a);
    b = uf_find(parent, b);
    if (a == b) return;
    if (a > b) {
      const int32_t t = a;
      a = b;
      b = t;
    }
    const int32_t old = atomicCAS(&parent[b], b, a);  // link the larger root below the smaller
    if (old == b) return;
    b = old;
  }
}

__device__ __forceinline__ bool lego_edge(const LGeo& g, float ra, float rb, bool horiz) {
  const float d1 = fmaxf(ra, rb), d2 = fminf(ra, rb);
  const float s = horiz ? g.sX : g.sY, c = horiz ? g.cX : g.cY;
  return fatan2(d2 * s, (d1 - d2 * c)) > g.theta;  // :358-362
}

__global__ __launch_bounds__(256) void k_lego_union(LGeo g, const float* __restrict__ range_mat,
                                                    int32_t* parent) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= g.cells || ld_parent(parent, c) < 0) return;
  const int row = (int)(c / g.H), col = (int)(c - (int64_t)row * g.H);
  const float rc = range_mat[c];
  // right neighbour (column wrap) and the one below; the reverse directions
  // are the same undirected edges seen from the other cell
  const int64_t cr = (col + 1 < g.H ? col + 1 : 0) + (int64_t)row * g.H;
  if (cr != c && ld_parent(parent, cr) >= 0 && lego_edge(g, rc, range_mat[cr], true))
    uf_unite(parent, (int32_t)c, (int32_t)cr);
  if (row + 1 < g.N) {
    const int64_t cd = c + g.H;
    if (ld_parent(parent, cd) >= 0 && lego_edge(g, rc, range_mat[cd], false))
      uf_unite(parent, (int32_t)c, (int32_t)cd);
  }
}

__global__ __launch_bounds__(256) void k_lego_compress(LGeo g, int32_t* parent, int32_t* csize,
                                                       unsigned long long* rows) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= g.cells || ld_parent(parent, c) < 0) return;
  const int32_t r = uf_find(parent, (int32_t)c);
  // path compression: any ancestor is a valid value for concurrent readers
  __hip_atomic_store(parent + c, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  atomicAdd(&csize[r], 1);
  // lineCountFlag is set for every pushed cell, not for the seed (:373)
  if (r != c) {
    const int row = (int)(c / g.H);
    atomicOr(&rows[2 * (int64_t)r + (row >> 6)], 1ull << (row & 63));
  }
}

// ---- labelComponents in one workgroup's LDS (images of <= kLegoCcCells
// cells, e.g. VLP-16's 16 x 1800): the union-find of k_lego_union /
// k_lego_compress ran on global atomics with chains as long as a row's runs
// (~70 us a sweep).  k_lego_edges (per cell) forms the two edge tests of the
// BFS (:355-372) and zeroes the per-root statistics; k_lego_cc links every
// horizontal run to its first cell with a wavefront prefix max (one
// wavefront per row), unites the vertical and the column-wrap edges with LDS
// atomics (linking the larger root below the smaller, path halving), then
// counts the component sizes in the roots' own entries and sets the row bits
// of the components under 30 cells (the only ones lego_feasible reads them
// for).  Same roots (each component's first row-major cell), sizes and row
// sets as the global kernels, so every later kernel is unchanged.
#ifdef SLIO_FE_STAMP
__device__ unsigned long long g_ccstamp[8];
#define CCSTAMP(k)                                                             \
  do {                                                                         \
    if (threadIdx.x == 0) g_ccstamp[k] = __builtin_amdgcn_s_memrealtime();     \
  } while (0)
__device__ unsigned long long g_bstamp[64][8];  // k_lego_cc_band: per band
__device__ unsigned long long g_mstamp[8];      // k_lego_cc_band: the merge
#define BSTAMP(k)                                                                          \
  do {                                                                                     \
    if (threadIdx.x == 0 && blockIdx.x < 64) g_bstamp[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define MSTAMP(k)                                                              \
  do {                                                                         \
    if (threadIdx.x == 0) g_mstamp[k] = __builtin_amdgcn_s_memrealtime();      \
  } while (0)
#else
#define BSTAMP(k) \
  do {            \
  } while (0)
#define MSTAMP(k) \
  do {            \
  } while (0)
#define CCSTAMP(k) \
  do {             \
  } while (0)
#endif
constexpr int kLegoCcThreads = 1024;
constexpr int kLegoCcSeg = 32;           // row cells per lane held in registers (rows <= 2048 cells)
constexpr int kLegoCcCells = 31 * 1024;  // 5 B of LDS a cell: 155 KB
__global__ __launch_bounds__(256) void k_lego_edges(LGeo g, const int32_t* __restrict__ owner,
                                                    const int8_t* __restrict__ ground,
                                                    const float* __restrict__ range_mat,
                                                    uint8_t* __restrict__ edges, int32_t* __restrict__ csize,
                                                    unsigned long long* __restrict__ rows) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= g.cells) return;
  csize[c] = 0;
  rows[2 * c] = 0ull;
  rows[2 * c + 1] = 0ull;
  auto valid = [&](int64_t k) { return owner[k] >= 0 && ground[k] != 1; };
  uint8_t e = 0;
  if (valid(c)) {
    e = 4;
    const int row = (int)(c / g.H), col = (int)(c - (int64_t)row * g.H);
    const float rc = range_mat[c];
    const int64_t cr = (col + 1 < g.H ? col + 1 : 0) + (int64_t)row * g.H;
    if (cr != c && valid(cr) && lego_edge(g, rc, range_mat[cr], true)) e |= 1;
    if (row + 1 < g.N && valid(c + g.H) && lego_edge(g, rc, range_mat[c + g.H], false)) e |= 2;
  }
  edges[c] = e;
}

__device__ __forceinline__ int lds_ld(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ int cc_find(int* par, int x) {
  int p = lds_ld(par + x);
  while (p != x) {
    const int gp = lds_ld(par + p);
    if (gp != p) __hip_atomic_store(par + x, gp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);  // halving
    x = p;
    p = gp;
  }
  return x;
}
__device__ __forceinline__ void cc_unite(int* par, int a, int b) {
  while (true) {
    a = cc_find(par, a);
    b = cc_find(par, b);
    if (a == b) return;
    if (a > b) {
      const int t = a;
      a = b;
      b = t;
    }
    const int old = atomicCAS(par + b, b, a);  // link the larger root below the smaller
    if (old == b) return;
    b = old;
  }
}

__global__ __launch_bounds__(kLegoCcThreads) void k_lego_cc(LGeo g, const uint8_t* __restrict__ edges,
                                                            int32_t* __restrict__ parent,
                                                            int32_t* __restrict__ csize,
                                                            unsigned long long* __restrict__ rows) {
  extern __shared__ int par[];  // cells, then the edge flags (cells bytes)
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int C = (int)g.cells;
  uint8_t* edg = reinterpret_cast<uint8_t*>(par + C);
  CCSTAMP(0);
  constexpr int kPer = (kLegoCcCells + kLegoCcThreads - 1) / kLegoCcThreads;
  // the edge flags into LDS first, every load in flight at once (the phases
  // below read them in dependent loops: from global memory each step paid
  // a round trip, ~50 us a sweep)
  {
    uint8_t ev[kPer];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int c = t + i * kLegoCcThreads;
      ev[i] = c < C ? edges[c] : 0;
    }
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int c = t + i * kLegoCcThreads;
      if (c < C) edg[c] = ev[i];
    }
  }
  __syncthreads();
  CCSTAMP(1);
  // horizontal runs: a valid cell with no edge from its left neighbour
  // starts a run; every cell of a run points at the run's first cell.  A
  // wavefront per row, each lane a contiguous segment of it: the segment's
  // last run start, a prefix max over the lanes, then the segment's cells
  // (a 64-cell chunk per step with a cross-lane carry was a chain of ~8
  // dependent shuffles per step: 12 us)
  for (int r = w; r < g.N; r += kLegoCcThreads / 64) {
    const int rb = r * g.H;
    const int seg = (g.H + 63) / 64;
    const int c0 = min(lane * seg, g.H), c1 = min(c0 + seg, g.H);
    // (rows hold <= 2048 cells: slio_lego_create refuses wider images for
    // the feature kernels' LDS layout, so a segment is <= kLegoCcSeg cells)
    {
      // the segment's flags (and its left neighbour's) in registers, every
      // LDS read in flight at once
      uint8_t eb[kLegoCcSeg + 1];
#pragma unroll
      for (int k = 0; k <= kLegoCcSeg; ++k) {
        const int col = c0 - 1 + k;
        eb[k] = (col >= 0 && col < c1) ? edg[rb + col] : 0;
      }
      int last = -1;
#pragma unroll
      for (int k = 1; k <= kLegoCcSeg; ++k)
        if ((eb[k] & 4) && !(eb[k - 1] & 1)) last = rb + c0 - 1 + k;
      int v = last;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(v, o, 64);
        if (lane >= o) v = max(v, u);
      }
      int cur = __shfl_up(v, 1, 64);  // the last run start before this segment
      if (lane == 0) cur = -1;
#pragma unroll
      for (int k = 1; k <= kLegoCcSeg; ++k) {
        const int col = c0 - 1 + k;
        if ((eb[k] & 4) && !(eb[k - 1] & 1)) cur = rb + col;
        if (col < c1) par[rb + col] = (eb[k] & 4) ? cur : -1;
      }
    }
  }
  __syncthreads();
  CCSTAMP(2);
  // vertical edges and the column wrap (col H - 1 -> 0).  A vertical edge
  // whose left neighbours are linked the same way (both cells continue a run
  // and the edge to the left exists) adds nothing: only the first of each
  // stretch of parallel edges is united.
  // (the thread's cells' tests first, every LDS read in flight, then the
  // unions: each one a chain of dependent LDS reads)
  {
    uint64_t need = 0;  // bit 2i: vertical union of cell i, 2i + 1: wrap union
    int col = t % g.H;
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int c = t + i * kLegoCcThreads;
      if (c < C) {
        const int e = edg[c];
        const bool vert = (e & 2) && !(col > 0 && (edg[c - 1] & 3) == 3 && (edg[c + g.H - 1] & 1));
        const bool wrap = (e & 1) && col == g.H - 1;
        need |= (vert ? 1ull : 0ull) << (2 * i);
        need |= (wrap ? 2ull : 0ull) << (2 * i);
      }
      col += kLegoCcThreads;
      while (col >= g.H) col -= g.H;
    }
    static_assert(2 * kPer <= 64, "need bits");
    for (uint64_t m = need; m; m &= m - 1) {
      const int b = __ffsll((unsigned long long)m) - 1, i = b >> 1;
      const int c = t + i * kLegoCcThreads;
      if (b & 1)
        cc_unite(par, c, c - (g.H - 1));
      else
        cc_unite(par, c, c + g.H);
    }
  }
  __syncthreads();
  CCSTAMP(3);
  // roots of every cell (registers: the entries are rewritten below)
  int root[kPer];
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int c = t + i * kLegoCcThreads;
    root[i] = (c < C && lds_ld(par + c) >= 0) ? cc_find(par, c) : -1;
  }
  __syncthreads();
  CCSTAMP(4);
  // sizes: a root's entry becomes -(size + 1) (<= -2; -1 stays "no label"):
  // it starts at -1 and every cell of the component subtracts 1, one atomic
  // per stretch of lanes (consecutive cells) with the same root
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int c = t + i * kLegoCcThreads;
    if (c < C) {
      parent[c] = root[i];
      if (root[i] == c) par[c] = -1;
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int r = root[i];
    const int prev = __shfl_up(r, 1, 64);
    const uint64_t heads = __ballot(lane == 0 || prev != r);
    if (r >= 0 && (lane == 0 || prev != r)) {
      const uint64_t after = heads & ~((2ull << lane) - 1ull);  // (lane 63: 2 << 63 wraps to 0)
      const int end = after ? __ffsll((unsigned long long)after) - 1 : 64;
      atomicSub(par + r, end - lane);
    }
  }
  __syncthreads();
  CCSTAMP(5);
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int c = t + i * kLegoCcThreads;
    if (c >= C || root[i] < 0) continue;
    const int sz = -lds_ld(par + root[i]) - 1;
    if (root[i] == c) csize[c] = sz;
    // lineCountFlag: every pushed cell's row (not the seed's, :373)
    if (root[i] != c && sz < 30) {
      const int row = c / g.H;
      atomicOr(&rows[2 * (int64_t)root[i] + (row >> 6)], 1ull << (row & 63));
    }
  }
  CCSTAMP(6);
}

// ---- labelComponents in column bands (round 5): the one-workgroup kernel
// above runs the whole image on one CU (~34 us a VLP-16 sweep).  Here band b
// (64 columns, all rows; one workgroup per band, grid ceil(H / 64)) forms its
// cells' edge bits (k_lego_edges' tests), links its row runs (a prefix max
// over the band's lanes), unites its vertical edges in LDS (union by the
// smaller cell index, path halving) and counts each band-local component's
// cells and row bits.  A band-local root is its component's smallest cell in
// the band; parent[] of every cell points at it (a global cell index).  The
// components a horizontal edge joins across a band seam (and across the
// column wrap H - 1 -> 0) are merged by the LAST band workgroup to arrive: the
// seam cells' local roots, sizes and row bits are handed over as records
// (write-through stores, drained, one arrival add; the last arriver loads
// them write-through, MI355X_MICROARCH.md inter-workgroup visibility), united
// in an LDS hash table by the smaller cell index, and each absorbed local root
// is linked below its component's root (parent[lr] = root, a smaller index:
// uf_find in the later kernels follows it), whose size and row bits become the
// component's.  The root of a component is its smallest cell index overall --
// the reference's label order (first row-major cell) -- and sizes and row
// sets (every cell's row but the seed's, :373) are the one-workgroup kernel's,
// so every later kernel is unchanged.  Rows <= 64.
constexpr int kLegoBandW = 64;
constexpr int kLegoBandThreads = 256;
constexpr int kLegoBandMaxRows = 64;
struct LegoSeamRec {
  int32_t root;   // the seam cell's band-local root (global cell index), -1: no cell
  int32_t size;   // that local component's cells
  uint64_t rows;  // its cells' rows, the local root's own row excluded
};
// the band kernel's limits: rows <= 64, the merge's hash at most half full
inline bool lego_band_ok(const LGeo& g) {
  const int64_t nb = (g.H + kLegoBandW - 1) / kLegoBandW;
  return g.N >= 1 && g.N <= kLegoBandMaxRows && g.H >= 2 && 4 * nb * g.N <= (int64_t)kLegoBandMaxRows * kLegoBandW;
}
__device__ __forceinline__ bool lego_valid(const int32_t* owner, const int8_t* ground, int64_t c) {
  return owner[c] >= 0 && ground[c] != 1;
}

__global__ __launch_bounds__(kLegoBandThreads) void k_lego_cc_band(
    LGeo g, const int32_t* __restrict__ owner, const int8_t* __restrict__ ground,
    const float* __restrict__ range_mat, int32_t* __restrict__ parent, int32_t* __restrict__ csize,
    unsigned long long* __restrict__ rows, LegoSeamRec* __restrict__ seam, uint32_t* __restrict__ arrive_ctr) {
  constexpr int W = kLegoBandW;
  constexpr int kRowsPerWave = kLegoBandMaxRows / (kLegoBandThreads / 64);
  __shared__ int lpar[kLegoBandMaxRows * W];
  __shared__ int lcnt[kLegoBandMaxRows * W];
  __shared__ unsigned long long lrow[kLegoBandMaxRows * W];
  __shared__ uint8_t le[kLegoBandMaxRows * W];
  __shared__ int s_last;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int N = g.N, H = g.H;
  const int nb = (H + W - 1) / W;
  const int band = blockIdx.x;
  const int col = band * W + lane;
  const bool incol = col < H;
  BSTAMP(0);
  // 1. the band's cells and the next column (its right neighbours, the
  // column wrap for the last band) staged in LDS: validity and range, every
  // global load of the thread in flight at once (a row-by-row loop with
  // branches on validity was a chain of dependent round trips: ~20 us)
  {
    constexpr int kSW = W + 1;
    constexpr int kPer = (kLegoBandMaxRows * kSW + kLegoBandThreads - 1) / kLegoBandThreads;
    const int width = min(W, H - band * W);  // the band's columns; column `width` is the next one
    int32_t ov[kPer];
    int8_t gv[kPer];
    float rv[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int q = t + u * kLegoBandThreads;
      const int r = q / kSW, j = q - r * kSW;
      const bool in = r < N && j <= width;
      int cj = band * W + j;
      if (cj >= H) cj -= H;
      const int64_t c = in ? (int64_t)r * H + cj : 0;
      ov[u] = in ? owner[c] : -1;
      gv[u] = in ? ground[c] : (int8_t)1;
      rv[u] = in ? range_mat[c] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int q = t + u * kLegoBandThreads;
      if (q < kLegoBandMaxRows * kSW) {
        reinterpret_cast<float*>(lrow)[q] = rv[u];                       // (lrow: free until step 4)
        reinterpret_cast<uint8_t*>(lcnt)[q] = ov[u] >= 0 && gv[u] != 1;  // (lcnt: likewise)
      }
    }
    __syncthreads();
    BSTAMP(1);
    const float* srng = reinterpret_cast<const float*>(lrow);
    const uint8_t* sval = reinterpret_cast<const uint8_t*>(lcnt);
    // edge bits: 4 valid, 1 right neighbour (column wrap), 2 below
    uint8_t ev[kLegoBandMaxRows / (kLegoBandThreads / 64)];
#pragma unroll
    for (int k = 0; k < kLegoBandMaxRows / (kLegoBandThreads / 64); ++k) {
      const int r = w + k * (kLegoBandThreads / 64);
      uint8_t e = 0;
      if (r < N && lane < width && sval[r * kSW + lane]) {
        e = 4;
        const float rc = srng[r * kSW + lane];
        // (one column: the right neighbour is the cell itself, no edge)
        if (H > 1 && sval[r * kSW + lane + 1] && lego_edge(g, rc, srng[r * kSW + lane + 1], true)) e |= 1;
        if (r + 1 < N && sval[(r + 1) * kSW + lane] && lego_edge(g, rc, srng[(r + 1) * kSW + lane], false))
          e |= 2;
      }
      ev[k] = e;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kLegoBandMaxRows / (kLegoBandThreads / 64); ++k) {
      const int r = w + k * (kLegoBandThreads / 64);
      if (r < N) {
        le[r * W + lane] = ev[k];
        lcnt[r * W + lane] = 0;
        lrow[r * W + lane] = 0ull;
      }
    }
  }
  __syncthreads();
  BSTAMP(2);
  // 2. row runs inside the band: every cell of a run points at its first cell
  for (int r = w; r < N; r += kLegoBandThreads / 64) {
    const int i = r * W + lane;
    const int e = le[i];
    const bool st = (e & 4) && !(lane > 0 && (le[i - 1] & 1));
    int v = st ? lane : -1;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(v, o, 64);
      if (lane >= o) v = max(v, u);
    }
    lpar[i] = (e & 4) ? r * W + v : -1;
  }
  __syncthreads();
  BSTAMP(3);
  // 3. vertical edges (only the first of a stretch of parallel ones)
  for (int r = w; r < N; r += kLegoBandThreads / 64) {
    const int i = r * W + lane;
    const int e = le[i];
    const bool vert = (e & 2) && !(lane > 0 && (le[i - 1] & 3) == 3 && (le[i - 1 + W] & 1));
    if (vert) cc_unite(lpar, i, i + W);
  }
  __syncthreads();
  BSTAMP(4);
  // 4. band-local roots, sizes and row bits (the root's own row excluded)
  int root[kRowsPerWave];
#pragma unroll
  for (int k = 0; k < kRowsPerWave; ++k) {
    const int r = w + k * (kLegoBandThreads / 64);
    const int i = r * W + lane;
    root[k] = (r < N && lds_ld(lpar + i) >= 0) ? cc_find(lpar, i) : -1;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kRowsPerWave; ++k) {
    const int r = w + k * (kLegoBandThreads / 64);
    const int i = r * W + lane;
    if (root[k] >= 0) {
      atomicAdd(&lcnt[root[k]], 1);
      if (root[k] != i) atomicOr(&lrow[root[k]], 1ull << r);
    }
  }
  __syncthreads();
  auto gidx = [&](int li) { return (int32_t)((li / W) * H + band * W + (li % W)); };
#pragma unroll
  for (int k = 0; k < kRowsPerWave; ++k) {
    const int r = w + k * (kLegoBandThreads / 64);
    if (r >= N || !incol) continue;
    const int i = r * W + lane;
    const int64_t c = (int64_t)r * H + col;
    parent[c] = root[k] >= 0 ? gidx(root[k]) : -1;
    if (root[k] == i) {
      csize[c] = lcnt[i];
      rows[2 * c] = lrow[i];
      rows[2 * c + 1] = 0ull;
    }
    // the seam records: the band's first (side 0) and last (side 1) column,
    // per row (a one-column band writes both)
    const int last = min(W, H - band * W) - 1;
    LegoSeamRec rec{-1, 0, 0ull};
    if (root[k] >= 0) rec = LegoSeamRec{gidx(root[k]), lcnt[root[k]], lrow[root[k]]};
#pragma unroll
    for (int side = 0; side < 2; ++side) {
      if (lane != (side == 0 ? 0 : last)) continue;
      LegoSeamRec* dst = seam + ((int64_t)band * 2 + side) * N + r;
      __hip_atomic_store(&dst->root, rec.root, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&dst->size, rec.size, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&dst->rows, rec.rows, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  BSTAMP(5);
  // 5. arrival (after every wave's stores have completed); the last band merges.
  // The band's parent / csize / rows lines are written back from this XCD's L2
  // (agent-scope release: buffer_wbl2) before the arrival: the merging band,
  // possibly on another XCD, overwrites some of the same words with plain
  // stores, and two L2s holding the same dirty words write them back at the
  // kernel's end in any order -- the band's stale copy could win.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __syncthreads();
  if (t == 0)
    s_last = __hip_atomic_fetch_add(arrive_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (uint32_t)nb - 1;
  __syncthreads();
  BSTAMP(6);
  if (!s_last) return;
  MSTAMP(0);
  if (t == 0) __hip_atomic_store(arrive_ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
  // merge: an LDS hash of the seam records' roots (key: cell index), union by
  // the smaller key across the horizontal seam edges, then each absorbed local
  // root below its component's root.  (The band arrays are reused.)
  constexpr int kHash = kLegoBandMaxRows * W;  // >= 2 x N seam records per band for nb <= 32 bands
  int* hkey = lcnt;                            // key or -1
  int* hpar = lpar;                            // union-find over slots
  unsigned long long* hrow = lrow;             // the slot's record rows; then the component's
  __shared__ int hsize[kHash];
  __shared__ int hacc[kHash];
  const int nrec = nb * 2 * N;
  for (int s = t; s < kHash; s += kLegoBandThreads) {
    hkey[s] = -1;
    hacc[s] = 0;
  }
  __syncthreads();
  auto slot_of = [&](int32_t key, bool insert) {
    uint32_t hsh = ((uint32_t)key * 2654435761u) & (kHash - 1);
    while (true) {
      const int k = lds_ld(hkey + hsh);
      if (k == key) return (int)hsh;
      if (k == -1) {
        if (!insert) return -1;
        const int old = atomicCAS(hkey + hsh, -1, key);
        if (old == -1 || old == key) return (int)hsh;
      }
      hsh = (hsh + 1) & (kHash - 1);
    }
  };
  MSTAMP(1);
  // (the thread's records first, every load in flight, then the inserts)
  constexpr int kRecPer = kHash / 2 / kLegoBandThreads;  // nrec <= kHash / 2 (lego_band_ok)
  {
    int32_t rk[kRecPer], rsz[kRecPer];
    uint64_t rrw[kRecPer];
#pragma unroll
    for (int u = 0; u < kRecPer; ++u) {
      const int q = t + u * kLegoBandThreads;
      const LegoSeamRec* src = seam + (q < nrec ? q : 0);
      rk[u] = __hip_atomic_load(&src->root, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      rsz[u] = __hip_atomic_load(&src->size, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      rrw[u] = __hip_atomic_load(&src->rows, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (q >= nrec) rk[u] = -1;
    }
#pragma unroll
    for (int u = 0; u < kRecPer; ++u) {
      if (rk[u] < 0) continue;
      const int s = slot_of(rk[u], true);
      hsize[s] = rsz[u];
      hrow[s] = rrw[u];
      hpar[s] = s;
    }
  }
  __syncthreads();
  // union-find over slots, the root slot keeps the smallest key
  auto sfind = [&](int s) {
    int p = lds_ld(hpar + s);
    while (p != s) {
      const int gp = lds_ld(hpar + p);
      if (gp != p) __hip_atomic_store(hpar + s, gp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      s = p;
      p = gp;
    }
    return s;
  };
  MSTAMP(2);
  // seam k: band k's last column -> band (k + 1) % nb's first column, every
  // row (a seam cell's edge to the right is a band's own test: the seam
  // cells' loads, all in flight, then the unions)
  constexpr int kSeamPer = kHash / 4 / kLegoBandThreads;  // nb * N <= kHash / 4 (lego_band_ok)
  bool sedge[kSeamPer];
  int32_t skl[kSeamPer], skr[kSeamPer];
  {
    int32_t oL[kSeamPer], oR[kSeamPer];
    int8_t gL[kSeamPer], gR[kSeamPer];
    float rL[kSeamPer], rR[kSeamPer];
#pragma unroll
    for (int u = 0; u < kSeamPer; ++u) {
      const int q = t + u * kLegoBandThreads;
      const bool in = q < nb * N;
      const int k = in ? q / N : 0, r = in ? q - k * N : 0;
      const int k2 = k + 1 < nb ? k + 1 : 0;
      const int colL = min((k + 1) * W, H) - 1, colR = k2 * W;
      const int64_t cL = (int64_t)r * H + colL, cR = (int64_t)r * H + colR;
      oL[u] = owner[cL];
      oR[u] = owner[cR];
      gL[u] = ground[cL];
      gR[u] = ground[cR];
      rL[u] = range_mat[cL];
      rR[u] = range_mat[cR];
      skl[u] = __hip_atomic_load(&seam[((int64_t)k * 2 + 1) * N + r].root, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
      skr[u] = __hip_atomic_load(&seam[((int64_t)k2 * 2) * N + r].root, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
      sedge[u] = in && cL != cR;
    }
#pragma unroll
    for (int u = 0; u < kSeamPer; ++u)
      sedge[u] = sedge[u] && oL[u] >= 0 && gL[u] != 1 && oR[u] >= 0 && gR[u] != 1 &&
                 lego_edge(g, rL[u], rR[u], true);
  }
#pragma unroll
  for (int u = 0; u < kSeamPer; ++u) {
    if (!sedge[u]) continue;
    int a = slot_of(skl[u], false), b = slot_of(skr[u], false);
    while (true) {
      a = sfind(a);
      b = sfind(b);
      if (a == b) break;
      if (hkey[a] > hkey[b]) {
        const int tmp = a;
        a = b;
        b = tmp;
      }
      const int old = atomicCAS(hpar + b, b, a);  // the larger key's root below the smaller's
      if (old == b) break;
      b = old;
    }
  }
  __syncthreads();
  MSTAMP(3);
  // each slot into its component's root: sizes, row bits (an absorbed local
  // root's own row counts: it is not the component's seed), parent links
  int rs[kHash / kLegoBandThreads];
#pragma unroll
  for (int u = 0; u < kHash / kLegoBandThreads; ++u) {
    const int s = t + u * kLegoBandThreads;
    rs[u] = hkey[s] >= 0 ? sfind(s) : -1;
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kHash / kLegoBandThreads; ++u) {
    const int s = t + u * kLegoBandThreads;
    if (rs[u] < 0 || rs[u] == s) continue;
    const int32_t key = hkey[s], rk = hkey[rs[u]];
    atomicAdd(&hacc[rs[u]], hsize[s]);
    atomicOr(&hrow[rs[u]], hrow[s] | (1ull << (key / H)));
    parent[key] = rk;
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kHash / kLegoBandThreads; ++u) {
    const int s = t + u * kLegoBandThreads;
    if (rs[u] == s && hacc[s] > 0) {
      const int32_t key = hkey[s];
      csize[key] = hsize[s] + hacc[s];
      rows[2 * (int64_t)key] = hrow[s];
    }
  }
  MSTAMP(4);
}

__device__ __forceinline__ bool lego_feasible(const LGeo& g, const int32_t* csize,
                                              const unsigned long long* rows, int32_t r) {
  const int sz = csize[r];
  if (sz >= 30) return true;
  if (sz < g.vpn) return false;
  const int lc = __popcll(rows[2 * (int64_t)r]) + __popcll(rows[2 * (int64_t)r + 1]);
  return lc >= g.vln;
}

// per cell of ring r: 0 feasible root, 1 segmented point, 2 outlier point
__device__ __forceinline__ void lego_cell_class(const LGeo& g, int r, int j, const int8_t* ground,
                                                const int32_t* parent, const int32_t* csize,
                                                const unsigned long long* rows, bool& root,
                                                bool& seg, bool& outl) {
  const int64_t c = j + (int64_t)r * g.H;
  const int32_t p = parent[c];
  const bool gnd = ground[c] == 1;
  root = seg = outl = false;
  bool positive = false, rejected = false;
  if (p >= 0) {
    const int32_t rt = uf_find(parent, p);
    const bool feas = lego_feasible(g, csize, rows, rt);
    root = feas && rt == c;
    positive = feas;
    rejected = !feas;
  }
  if (!(positive || rejected || gnd)) return;  // label -1 and not ground
  if (rejected) {  // 999999 (:286-293)
    outl = r > g.gsi && j % 5 == 0;
    return;
  }
  if (gnd && j % 5 != 0 && j > 5 && j < g.H - 5) return;  // ground decimation (:295-297)
  seg = true;
}

constexpr int kLegoRowThreads = 1024;

__global__ __launch_bounds__(kLegoRowThreads) void k_lego_rowcount(LGeo g, const int8_t* ground,
                                                                   const int32_t* parent,
                                                                   const int32_t* csize,
                                                                   const unsigned long long* rows,
                                                                   int32_t* cnt /* [N][3] */) {
  __shared__ int scratch[kLegoRowThreads / 64 + 1];
  const int r = blockIdx.x, t = threadIdx.x;
  int a = 0, b = 0, d = 0;
  for (int j = t; j < g.H; j += kLegoRowThreads) {
    bool root, seg, outl;
    lego_cell_class(g, r, j, ground, parent, csize, rows, root, seg, outl);
    a += root;
    b += seg;
    d += outl;
  }
  int e;
  a = block_exclusive_scan<kLegoRowThreads>(a, scratch, e);
  b = block_exclusive_scan<kLegoRowThreads>(b, scratch, e);
  d = block_exclusive_scan<kLegoRowThreads>(d, scratch, e);
  if (t == 0) {
    cnt[3 * r] = a;
    cnt[3 * r + 1] = b;
    cnt[3 * r + 2] = d;
  }
}

struct LegoSeg {
  int32_t *start_ring, *end_ring, *col_ind;
  uint8_t* ground_flag;
  float* range;
  float4* xyzi;
  float4* outlier;
  int32_t* n;  // n_segmented, n_outlier
};

__global__ __launch_bounds__(kLegoRowThreads) void k_lego_extract(
    LGeo g, const int8_t* ground, const int32_t* parent, const int32_t* csize,
    const unsigned long long* rows, const int32_t* cnt, const float* range_mat, const float4* full,
    int32_t* rootlab, LegoSeg sg) {
  __shared__ int scratch[kLegoRowThreads / 64 + 1];
  const int r = blockIdx.x, t = threadIdx.x;
  int pa = 0, pb = 0, pd = 0;
  for (int q = t; q < r; q += kLegoRowThreads) {
    pa += cnt[3 * q];
    pb += cnt[3 * q + 1];
    pd += cnt[3 * q + 2];
  }
  int e;
  const int oa = block_exclusive_scan<kLegoRowThreads>(pa, scratch, e);
  const int ob = block_exclusive_scan<kLegoRowThreads>(pb, scratch, e);
  const int od = block_exclusive_scan<kLegoRowThreads>(pd, scratch, e);
  if (t == 0) {
    sg.start_ring[r] = ob - 1 + 5;
    sg.end_ring[r] = ob + cnt[3 * r + 1] - 1 - 5;
    if (r == g.N - 1) {
      sg.n[0] = ob + cnt[3 * r + 1];
      sg.n[1] = od + cnt[3 * r + 2];
    }
  }
  // thread t owns the contiguous columns [t * per, (t + 1) * per)
  const int per = (g.H + kLegoRowThreads - 1) / kLegoRowThreads;
  const int j0 = t * per, j1 = min(j0 + per, g.H);
  int a = 0, b = 0, d = 0;
  for (int j = j0; j < j1; ++j) {
    bool root, seg, outl;
    lego_cell_class(g, r, j, ground, parent, csize, rows, root, seg, outl);
    a += root;
    b += seg;
    d += outl;
  }
  int ea, eb, ed;
  block_exclusive_scan<kLegoRowThreads>(a, scratch, ea);
  block_exclusive_scan<kLegoRowThreads>(b, scratch, eb);
  block_exclusive_scan<kLegoRowThreads>(d, scratch, ed);
  int ka = oa + ea, kb = ob + eb, kd = od + ed;
  for (int j = j0; j < j1; ++j) {
    bool root, seg, outl;
    lego_cell_class(g, r, j, ground, parent, csize, rows, root, seg, outl);
    const int64_t c = j + (int64_t)r * g.H;
    if (root) rootlab[c] = 1 + ka++;  // labelCount order (:390)
    if (seg) {
      sg.ground_flag[kb] = ground[c] == 1;
      sg.col_ind[kb] = j;
      sg.range[kb] = range_mat[c];
      sg.xyzi[kb] = full[c];
      ++kb;
    }
    if (outl) sg.outlier[kd++] = full[c];
  }
}

__global__ __launch_bounds__(256) void k_lego_label(LGeo g, const int32_t* parent, const int32_t* csize,
                                                    const unsigned long long* rows,
                                                    const int32_t* rootlab, int32_t* label, int32_t* clear) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= g.cells) return;
  clear[c] = -1;  // the other owner table, for the next sweep
  const int32_t p = parent[c];
  if (p < 0) {
    label[c] = -1;
    return;
  }
  const int32_t rt = uf_find(parent, p);
  label[c] = lego_feasible(g, csize, rows, rt) ? rootlab[rt] : 999999;
}

struct LegoImuDev {
  const double* time;
  const float *roll, *pitch, *yaw, *vx, *vy, *vz, *ax, *ay, *az;
  int last, last_it, Q;
  double t0;
  float ang_last[3];
  int on;
  int seg;  // entries on the ring from last_it to last; > 0: their times are non-decreasing
};

struct LegoImuOutDev {
  float rpy_start[3], rpy_cur[3], velo_from_start[3], angular_from_start[3], ang_last[3];
};

// adjustDistortion's per-point orientation before the halfPassed switch
__device__ __forceinline__ float ori_a(float so, float px, float pz, bool& passes) {
  float ori = -fatan2(px, pz);
  if (ori < so - M_PI / 2)
    ori = (float)((double)ori + 2 * M_PI);
  else if (ori > so + M_PI * 3 / 2)
    ori = (float)((double)ori - 2 * M_PI);
  passes = ori - so > M_PI;
  return ori;
}

__global__ __launch_bounds__(256) void k_lego_half(const float4* seg, const int32_t* nseg, float so,
                                                   uint32_t* slot, LegoImuOutDev* io, float al0,
                                                   float al1, float al2) {
  __shared__ uint32_t wmin[4];
  const int n = *nseg;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i == 0) {  // the state adjustDistortion leaves when it writes nothing
    *io = LegoImuOutDev{};
    io->ang_last[0] = al0;
    io->ang_last[1] = al1;
    io->ang_last[2] = al2;
  }
  bool f = false;
  if (i < n) {
    const float4 p = seg[i];
    ori_a(so, p.y, p.x, f);  // point.x = y, point.z = x
  }
  uint32_t v = f ? (uint32_t)i : kNone;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, 64));
  if ((threadIdx.x & 63) == 0) wmin[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) slot[blockIdx.x] = min(min(wmin[0], wmin[1]), min(wmin[2], wmin[3]));
}

// k_lego_rowcount + k_lego_extract + k_lego_label + k_lego_half in ONE
// launch of kLegoRowsSplit workgroups per ring (block b = r S + s takes the
// ring's s-th column range; all N S <= 1024 blocks resident at once): each
// block classifies its cells once (root / segmented / outlier, kept in
// registers), publishes its three counts, waits for the blocks before it (in
// row-major order) to publish theirs -- a decoupled look-back over blocks
// dispatched earlier -- and writes its part of the segmented cloud, the
// outliers and its roots' labelCount numbers (write-through); after a second
// publication it labels its cells once the earlier blocks' numbers are out (a
// component's root is its first row-major cell: in this block or an earlier
// one).  halfPassed's first switch point per block goes to slot[b]
// (k_lego_deskew takes the minimum).  Flags carry the sweep's sequence number
// (no reset); a wait gives up after ~0.5 s and marks the sweep failed
// (n_segmented = -1) instead of hanging.
// (8 blocks of 256 per ring measured slower: 26.9 vs 21.8 us a VLP-16 sweep --
// the look-back over 8x the blocks and the phases' round trips dominate)
constexpr int kLegoRowsSplit = 1;    // blocks per ring
constexpr int kLegoRowsThreads = 1024;
constexpr int kLegoRowsPer = 8;      // cells per thread: rings of <= 8192 columns
__device__ __forceinline__ bool lego_wait_blocks(const uint32_t* flag, int b, uint32_t seq) {
  bool ok = true;
  const unsigned long long t0 = wall_clock64();
  for (int q = threadIdx.x; q < b && ok; q += kLegoRowsThreads)
    while (__hip_atomic_load(flag + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != seq) {
      if (wall_clock64() - t0 > 50000000ull) {  // 100 MHz: 0.5 s
        ok = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return __syncthreads_and(ok);
}
__global__ __launch_bounds__(kLegoRowsThreads) void k_lego_rows(
    LGeo g, const int8_t* ground, const int32_t* parent, const int32_t* csize, const unsigned long long* rows,
    const float* range_mat, const float4* full, int32_t* rootlab, LegoSeg sg, int32_t* label, int32_t* clear,
    uint32_t* rsync /* [B] ready, [B] done, [3 B] counts */, uint32_t seq, float so, uint32_t* slot,
    LegoImuOutDev* io, float al0, float al1, float al2) {
  __shared__ int scratch[kLegoRowsThreads / 64 + 1];
  __shared__ uint32_t wmin[kLegoRowsThreads / 64];
  const int b = blockIdx.x, t = threadIdx.x, B = g.N * kLegoRowsSplit;
  const int r = b / kLegoRowsSplit, sp = b % kLegoRowsSplit;
  uint32_t* ready = rsync;
  uint32_t* done = rsync + B;
  uint32_t* cnt = rsync + 2 * B;
  if (b == 0 && t == 0) {  // the state adjustDistortion leaves when it writes nothing
    *io = LegoImuOutDev{};
    io->ang_last[0] = al0;
    io->ang_last[1] = al1;
    io->ang_last[2] = al2;
  }
  const int c0 = (int)((int64_t)g.H * sp / kLegoRowsSplit), c1 = (int)((int64_t)g.H * (sp + 1) / kLegoRowsSplit);
  const int per = (c1 - c0 + kLegoRowsThreads - 1) / kLegoRowsThreads;
  const int j0 = c0 + t * per, j1 = min(j0 + per, c1);
  int32_t rt[kLegoRowsPer];
  uint8_t cls[kLegoRowsPer];  // 1 root, 2 segmented, 4 outlier, 8 feasible root, 16 has a parent
  int a = 0, bb = 0, d = 0;
#pragma unroll
  for (int k = 0; k < kLegoRowsPer; ++k) {
    const int j = j0 + k;
    rt[k] = -1;
    cls[k] = 0;
    if (j >= j1) continue;
    const int64_t c = j + (int64_t)r * g.H;
    const int32_t p = parent[c];
    const bool gnd = ground[c] == 1;
    bool positive = false, rejected = false;
    uint8_t f = 0;
    if (p >= 0) {
      rt[k] = uf_find(parent, p);
      const bool feas = lego_feasible(g, csize, rows, rt[k]);
      positive = feas;
      rejected = !feas;
      f |= 16 | (feas ? 8 : 0) | (feas && rt[k] == c ? 1 : 0);
    }
    // lego_cell_class
    if (positive || rejected || gnd) {
      if (rejected) {
        if (r > g.gsi && j % 5 == 0) f |= 4;
      } else if (!(gnd && j % 5 != 0 && j > 5 && j < g.H - 5)) {
        f |= 2;
      }
    }
    cls[k] = f;
    a += f & 1;
    bb += (f >> 1) & 1;
    d += (f >> 2) & 1;
  }
  int ea, eb, ed;
  const int ta = block_exclusive_scan<kLegoRowsThreads>(a, scratch, ea);
  const int tb = block_exclusive_scan<kLegoRowsThreads>(bb, scratch, eb);
  const int td = block_exclusive_scan<kLegoRowsThreads>(d, scratch, ed);
  if (t == 0) {
    __hip_atomic_store(cnt + 3 * b, (uint32_t)ta, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(cnt + 3 * b + 1, (uint32_t)tb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(cnt + 3 * b + 2, (uint32_t)td, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(ready + b, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
  bool ok = lego_wait_blocks(ready, b, seq);
  int pa = 0, pb = 0, pd = 0;
  for (int q = t; q < b; q += kLegoRowsThreads) {
    pa += (int)__hip_atomic_load(cnt + 3 * q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    pb += (int)__hip_atomic_load(cnt + 3 * q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    pd += (int)__hip_atomic_load(cnt + 3 * q + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  int e;
  const int oa = block_exclusive_scan<kLegoRowsThreads>(pa, scratch, e);
  const int ob = block_exclusive_scan<kLegoRowsThreads>(pb, scratch, e);
  const int od = block_exclusive_scan<kLegoRowsThreads>(pd, scratch, e);
  if (t == 0) {
    if (sp == 0) sg.start_ring[r] = ob - 1 + 5;
    if (sp == kLegoRowsSplit - 1) sg.end_ring[r] = ob + tb - 1 - 5;
    if (b == B - 1) {
      sg.n[0] = ok ? ob + tb : -1;
      sg.n[1] = od + td;
    }
  }
  int ka = oa + ea, kb = ob + eb, kd = od + ed;
  uint32_t sw = kNone;  // halfPassed: the block's first segmented point past the switch
#pragma unroll
  for (int k = 0; k < kLegoRowsPer; ++k) {
    const int j = j0 + k;
    if (j >= j1) continue;
    const int64_t c = j + (int64_t)r * g.H;
    const uint8_t f = cls[k];
    if (f & 1) __hip_atomic_store(rootlab + c, 1 + ka++, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (f & 2) {
      const float4 q = full[c];
      sg.ground_flag[kb] = ground[c] == 1;
      sg.col_ind[kb] = j;
      sg.range[kb] = range_mat[c];
      sg.xyzi[kb] = q;
      bool pass;
      ori_a(so, q.y, q.x, pass);  // point.x = y, point.z = x
      if (pass) sw = min(sw, (uint32_t)kb);
      ++kb;
    }
    if (f & 4) sg.outlier[kd++] = full[c];
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) sw = min(sw, (uint32_t)__shfl_xor((int)sw, o, 64));
  if ((t & 63) == 0) wmin[t >> 6] = sw;
  // every wave's root numbers out (write-through, drained) before "done"
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __syncthreads();
  if (t == 0) {
    uint32_t m = wmin[0];
    for (int q = 1; q < kLegoRowsThreads / 64; ++q) m = min(m, wmin[q]);
    slot[b] = m;
    __hip_atomic_store(done + b, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
  ok = lego_wait_blocks(done, b, seq) && ok;
  if (!ok && t == 0) sg.n[0] = -1;
#pragma unroll
  for (int k = 0; k < kLegoRowsPer; ++k) {
    const int j = j0 + k;
    if (j >= j1) continue;
    const int64_t c = j + (int64_t)r * g.H;
    clear[c] = -1;  // the other owner table, for the next sweep
    const uint8_t f = cls[k];
    label[c] = !(f & 16) ? -1
                         : (f & 8) ? (int32_t)__hip_atomic_load(rootlab + rt[k], __ATOMIC_RELAXED,
                                                                 __HIP_MEMORY_SCOPE_AGENT)
                                   : 999999;
  }
}

struct ImuCur {
  float r, p, y, vx, vy, vz;
  bool after;
  int f, b;
  float rf, rb;
};

// :652-719 interpolation of the IMU ring at timeScanCur + pointTime
__device__ ImuCur imu_at(const LegoImuDev& m, float pointTime) {
  ImuCur c;
  const double tq = m.t0 + pointTime;
  int f = m.last_it;
  if (m.seg > 0) {
    // the first of the ring entries last_it, ... before last whose time
    // exceeds tq, else last: over non-decreasing times the reference's walk
    // ends where this binary search does (a NaN tq: at last in both)
    int lo = 0, n = m.seg - 1;
    while (n > 0) {
      const int h = n >> 1;
      const int q = m.last_it + lo + h;
      if (!(tq < m.time[q >= m.Q ? q - m.Q : q])) {
        lo += h + 1;
        n -= h + 1;
      } else {
        n = h;
      }
    }
    f = m.last_it + lo;
    if (f >= m.Q) f -= m.Q;
  } else {
    while (f != m.last) {
      if (tq < m.time[f]) break;
      f = f + 1 == m.Q ? 0 : f + 1;  // (f + 1) % Q without the division
    }
  }
  c.f = f;
  c.b = f == 0 ? m.Q - 1 : f - 1;
  c.after = tq > m.time[f];
  c.rf = c.rb = 0.f;
  if (c.after) {
    c.r = m.roll[f];
    c.p = m.pitch[f];
    c.y = m.yaw[f];
    c.vx = m.vx[f];
    c.vy = m.vy[f];
    c.vz = m.vz[f];
  } else {
    const int b = c.b;
    c.rf = (float)((tq - m.time[b]) / (m.time[f] - m.time[b]));
    c.rb = (float)((m.time[f] - tq) / (m.time[f] - m.time[b]));
    c.r = m.roll[f] * c.rf + m.roll[b] * c.rb;
    c.p = m.pitch[f] * c.rf + m.pitch[b] * c.rb;
    if (m.yaw[f] - m.yaw[b] > M_PI)
      c.y = (float)(m.yaw[f] * c.rf + ((double)m.yaw[b] + 2 * M_PI) * c.rb);
    else if (m.yaw[f] - m.yaw[b] < -M_PI)
      c.y = (float)(m.yaw[f] * c.rf + ((double)m.yaw[b] - 2 * M_PI) * c.rb);
    else
      c.y = m.yaw[f] * c.rf + m.yaw[b] * c.rb;
    c.vx = m.vx[f] * c.rf + m.vx[b] * c.rb;
    c.vy = m.vy[f] * c.rf + m.vy[b] * c.rb;
    c.vz = m.vz[f] * c.rf + m.vz[b] * c.rb;
  }
  return c;
}

constexpr int kImuQueLds = 512;

__global__ __launch_bounds__(256) void k_lego_deskew(const float4* seg, const int32_t* nseg,
                                                     const uint32_t* slot, int nslot, float so,
                                                     float eo, float od, float scan_period,
                                                     LegoImuDev m, float4* out,
                                                     LegoImuOutDev* io) {
  __shared__ uint32_t wmin[4];
  __shared__ double s_time[kImuQueLds];
  __shared__ float s_arr[9][kImuQueLds];
  __shared__ float st[12];  // rs ps ys vxs vys vzs cR cP cY sR sP sY
  const int n = *nseg;
  const int t = threadIdx.x;
  const int i = blockIdx.x * 256 + t;
  // the halfPassed switch point: the first point whose pre-switch orientation passes
  uint32_t v = kNone;
  for (int q = t; q < nslot; q += 256) v = min(v, slot[q]);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, 64));
  if ((t & 63) == 0) wmin[t >> 6] = v;
  const bool imu = m.on && m.last >= 0;
  if (imu && m.Q <= kImuQueLds) {
    for (int q = t; q < m.Q; q += 256) {
      s_time[q] = m.time[q];
      s_arr[0][q] = m.roll[q];
      s_arr[1][q] = m.pitch[q];
      s_arr[2][q] = m.yaw[q];
      s_arr[3][q] = m.vx[q];
      s_arr[4][q] = m.vy[q];
      s_arr[5][q] = m.vz[q];
      s_arr[6][q] = m.ax[q];
      s_arr[7][q] = m.ay[q];
      s_arr[8][q] = m.az[q];
    }
  }
  __syncthreads();
  if (imu && m.Q <= kImuQueLds) {
    m.time = s_time;
    m.roll = s_arr[0];
    m.pitch = s_arr[1];
    m.yaw = s_arr[2];
    m.vx = s_arr[3];
    m.vy = s_arr[4];
    m.vz = s_arr[5];
    m.ax = s_arr[6];
    m.ay = s_arr[7];
    m.az = s_arr[8];
  }
  const uint32_t half = min(min(wmin[0], wmin[1]), min(wmin[2], wmin[3]));
  // start state from point 0 (i == 0 branch, :721-781)
  if (imu && t == 0 && n > 0) {
    const float4 p0 = seg[0];
    bool f0;
    const float o0 = ori_a(so, p0.y, p0.x, f0);
    const float rel0 = (o0 - so) / od;
    const ImuCur c0 = imu_at(m, rel0 * scan_period);
    st[0] = c0.r;
    st[1] = c0.p;
    st[2] = c0.y;
    st[3] = c0.vx;
    st[4] = c0.vy;
    st[5] = c0.vz;
    fsincos(c0.r, st[9], st[6]);
    fsincos(c0.p, st[10], st[7]);
    fsincos(c0.y, st[11], st[8]);
    if (blockIdx.x == 0) {
      float a[3];
      if (c0.after) {
        a[0] = m.ax[c0.f];
        a[1] = m.ay[c0.f];
        a[2] = m.az[c0.f];
      } else {
        a[0] = m.ax[c0.f] * c0.rf + m.ax[c0.b] * c0.rb;
        a[1] = m.ay[c0.f] * c0.rf + m.ay[c0.b] * c0.rb;
        a[2] = m.az[c0.f] * c0.rf + m.az[c0.b] * c0.rb;
      }
      for (int k = 0; k < 3; ++k) {
        io->angular_from_start[k] = a[k] - m.ang_last[k];
        io->ang_last[k] = a[k];
      }
      io->rpy_start[0] = c0.r;
      io->rpy_start[1] = c0.p;
      io->rpy_start[2] = c0.y;
    }
  }
  __syncthreads();
  if (i >= n) return;
  const float4 s4 = seg[i];
  float px = s4.y, py = s4.z, pz = s4.x;
  float ori;
  if ((uint32_t)i <= half) {
    bool f;
    ori = ori_a(so, px, pz, f);
  } else {
    ori = -fatan2(px, pz);
    ori = (float)((double)ori + 2 * M_PI);
    if (ori < eo - M_PI * 3 / 2)
      ori = (float)((double)ori + 2 * M_PI);
    else if (ori > eo + M_PI / 2)
      ori = (float)((double)ori - 2 * M_PI);
  }
  const float relTime = (ori - so) / od;
  const float inten = int(s4.w) + scan_period * relTime;
  if (imu) {
    const ImuCur c = imu_at(m, relTime * scan_period);
    if (i == n - 1) {
      io->rpy_cur[0] = c.r;
      io->rpy_cur[1] = c.p;
      io->rpy_cur[2] = c.y;
    }
    if (i > 0) {
      const float cRs = st[6], cPs = st[7], cYs = st[8], sRs = st[9], sPs = st[10], sYs = st[11];
      if (i == n - 1) {  // VeloToStartIMU (:392-427) of the last point
        const float vx = c.vx - st[3], vy = c.vy - st[4], vz = c.vz - st[5];
        const float x1 = cYs * vx - sYs * vz, y1 = vy, z1 = sYs * vx + cYs * vz;
        const float x2 = x1, y2 = cPs * y1 + sPs * z1, z2 = -sPs * y1 + cPs * z1;
        io->velo_from_start[0] = cRs * x2 + sRs * y2;
        io->velo_from_start[1] = -sRs * x2 + cRs * y2;
        io->velo_from_start[2] = z2;
      }
      // TransformToStartIMU (:429-458); imuShiftFromStartCur is 0.  One
      // double sincos per angle (six separate sin / cos calls were most of
      // the kernel's time)
      float sr, cr, sp_, cp, sy, cy;
      fsincos(c.r, sr, cr);
      fsincos(c.p, sp_, cp);
      fsincos(c.y, sy, cy);
      const float x1 = cr * px - sr * py;
      const float y1 = sr * px + cr * py;
      const float z1 = pz;
      const float x2 = x1;
      const float y2 = cp * y1 - sp_ * z1;
      const float z2 = sp_ * y1 + cp * z1;
      const float x3 = cy * x2 + sy * z2;
      const float y3 = y2;
      const float z3 = -sy * x2 + cy * z2;
      const float x4 = cYs * x3 - sYs * z3;
      const float y4 = y3;
      const float z4 = sYs * x3 + cYs * z3;
      const float x5 = x4;
      const float y5 = cPs * y4 + sPs * z4;
      const float z5 = -sPs * y4 + cPs * z4;
      px = cRs * x5 + sRs * y5 + 0.0f;
      py = -sRs * x5 + cRs * y5 + 0.0f;
      pz = z5 + 0.0f;
    }
  }
  out[i] = make_float4(px, py, pz, inten);
}

__global__ __launch_bounds__(kConcatThreads) void k_lego_concat(int n_scan, const int32_t* start_ring,
                                                                FeatOut f, float4* sharp, float4* less_sharp,
                                                                float4* flat, float4* less_flat,
                                                                int64_t* counts) {
  __shared__ int s_o[4];
  const int r = blockIdx.x, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // ring offsets: wavefront k of the first four sums the earlier rings' counts
  // of output k (sharp, less sharp, flat, less flat)
  if (w < 4) {
    const int32_t* cnt = w == 0 ? f.sharp_count : w == 1 ? f.corner_count : w == 2 ? f.flat_count : f.surf_count;
    const int o = wave_prefix_count(cnt, r);
    if (lane == 0) {
      s_o[w] = o;
      if (r == n_scan - 1) counts[w] = o + cnt[r];
    }
  }
  __syncthreads();
  const int nc = f.corner_count[r];
  if (w == 0) {
    // cornerPointsSharp: the label-2 picks in pick order (ballot compaction)
    int k = s_o[0];
    for (int q0 = 0; q0 < nc; q0 += 64) {
      const int q = q0 + lane;
      const bool sh = q < nc && f.corner_sharp[(int64_t)r * kCornerPerRing + q];
      const uint64_t b = __ballot(sh);
      if (sh) sharp[k + __popcll(b & ((1ull << lane) - 1))] = f.corner_stage[(int64_t)r * kCornerPerRing + q];
      k += __popcll(b);
    }
  }
  for (int q = threadIdx.x; q < nc; q += kConcatThreads)
    less_sharp[s_o[1] + q] = f.corner_stage[(int64_t)r * kCornerPerRing + q];
  for (int q = threadIdx.x; q < f.flat_count[r]; q += kConcatThreads)
    flat[s_o[2] + q] = f.flat_stage[(int64_t)r * kFlatPerRing + q];
  const float4* src = f.surf_stage + (start_ring[r] - 4);
  for (int q = threadIdx.x; q < f.surf_count[r]; q += kConcatThreads) less_flat[s_o[3] + q] = src[q];
}

}  // namespace lego
}  // namespace slio

using namespace slio::lego;

#ifdef SLIO_FE_STAMP
extern "C" int slio_dbg_vsort_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(slio::lio::g_vstamp), sizeof(slio::lio::g_vstamp)) == hipSuccess ? 0 : -1;
}
extern "C" int slio_dbg_band_stamps(unsigned long long* band, unsigned long long* merge) {
  return hipMemcpyFromSymbol(band, HIP_SYMBOL(g_bstamp), sizeof(g_bstamp)) == hipSuccess &&
                 hipMemcpyFromSymbol(merge, HIP_SYMBOL(g_mstamp), sizeof(g_mstamp)) == hipSuccess
             ? 0
             : -1;
}
extern "C" int slio_dbg_cc_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ccstamp), sizeof(g_ccstamp)) == hipSuccess ? 0 : -1;
}
#endif

struct slio_lego {
  bool dev_counted = false;  // counted in slio::dev_users
  slio_lego_params prm{};
  LGeo g{};
  hipStream_t own = nullptr, stream = nullptr;
  int64_t cap = 0, cells = 0;
  float *x = nullptr, *y = nullptr, *z = nullptr;
  int64_t n = 0;
  float orient[3] = {0.f, 0.f, 0.f};
  // IMU ring (device) + state
  double* itime = nullptr;
  float* iarr = nullptr;  // 12 arrays of que_len
  int que = 0;
  LegoImuDev imu{};
  int imu_last_host = 0;
  bool cc_global = false;  // labelComponents by k_lego_union / k_lego_compress
  bool cc_lds1 = false;    // labelComponents by the one-workgroup k_lego_cc (SLIO_LEGO_CC_LDS1)
  LegoSeamRec* seam = nullptr;  // k_lego_cc_band's seam records
  uint32_t* cc_arrive = nullptr;
  // image / segmentation
  int32_t* owner = nullptr;      // this sweep's cell owners (0xFFFFFFFF: none)
  int32_t* owner_alt = nullptr;  // the other table: the last sweep's, cleared by this sweep's
                                 // k_lego_label for the next one (no memset per sweep)
  bool swept = false;
  float* range_mat = nullptr;
  float4* full = nullptr;
  int8_t* ground = nullptr;
  int32_t* parent = nullptr;
  uint8_t* edges = nullptr;
  int32_t* csize = nullptr;
  unsigned long long* rows = nullptr;
  int32_t* cnt = nullptr;
  uint32_t* rsync = nullptr;  // k_lego_rows' flags and counts per block ([B] ready, [B] done, [3 B])
  uint32_t sweep_seq = 0;
  bool rows_split = false;    // SLIO_LEGO_ROWS_SPLIT=1: the four-launch row stage (A/B)
  int32_t* rootlab = nullptr;
  int32_t* label = nullptr;
  int32_t *start_ring = nullptr, *end_ring = nullptr, *col_ind = nullptr, *nseg = nullptr;
  uint8_t* gflag = nullptr;
  float* srange = nullptr;
  float4 *sxyzi = nullptr, *outlier = nullptr;
  // features
  uint32_t* slot = nullptr;
  float4* desk = nullptr;
  LegoImuOutDev* io = nullptr;
  float* curvature = nullptr;
  uint8_t* picked0 = nullptr;
  int32_t* flabel = nullptr;
  float4* corner_stage = nullptr;
  int8_t* corner_sharp = nullptr;
  int32_t *corner_count = nullptr, *sharp_count = nullptr, *flat_count = nullptr, *surf_count = nullptr;
  float4 *flat_stage = nullptr, *surf_stage = nullptr;
  float4 *c_sharp = nullptr, *c_less_sharp = nullptr, *c_flat = nullptr, *c_less_flat = nullptr;
  int64_t* counts = nullptr;
  FeatCfg fc{};
  FeatWork fw{};
  bool ran = false;
  bool prof = false;
  bool prof_scan = false;  // SLIO_LIO_PROFILE_SCAN: the events span the whole scan
  double prof_ms = 0.0;
  int64_t prof_n = 0;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending, pool;
};

namespace {

void lego_prof_drain(slio_lego* h) {
  for (auto& p : h->pending) {
    float ms = 0.f;
    if (hipEventSynchronize(p.second) == hipSuccess &&
        hipEventElapsedTime(&ms, p.first, p.second) == hipSuccess) {
      h->prof_ms += ms;
      h->prof_n += 1;
    }
    h->pool.push_back(p);
  }
  h->pending.clear();
}

void lego_free(slio_lego* h) {
  lego_prof_drain(h);
  for (auto& p : h->pool) {
    (void)hipEventDestroy(p.first);
    (void)hipEventDestroy(p.second);
  }
  void* dev[] = {h->x, h->y, h->z, h->itime, h->iarr, h->owner, h->owner_alt, h->range_mat, h->full, h->ground,
                 h->parent, h->edges, h->csize, h->rows, h->cnt, h->rootlab, h->label, h->start_ring,
                 h->end_ring, h->col_ind, h->nseg, h->gflag, h->srange, h->sxyzi, h->outlier,
                 h->slot, h->desk, h->io, h->curvature, h->picked0, h->flabel, h->corner_stage,
                 h->corner_sharp, h->corner_count, h->sharp_count, h->flat_count, h->surf_count,
                 h->flat_stage, h->surf_stage, h->c_sharp, h->c_less_sharp, h->c_flat,
                 h->c_less_flat, h->counts, h->seam, h->cc_arrive, h->rsync};
  for (void* p : dev)
    if (p) (void)hipFree(p);
  feat_work_free(h->fw);
  if (h->own) (void)hipStreamDestroy(h->own);
}

#define LEGO_CHECK_H(h)                    \
  do {                                     \
    if (!(h)) {                            \
      set_error("null slio_lego handle");  \
      return SLIO_EINVAL;                  \
    }                                      \
    LIO_HIP(hipSetDevice((h)->prm.device)); \
  } while (0)

inline float hfatan2(float y, float x) { return (float)std::atan2((double)y, (double)x); }

}  // namespace

extern "C" {

int slio_lego_params_default(slio_lego_params* p) {
  if (!p) return SLIO_EINVAL;
  std::memset(p, 0, sizeof(*p));
  p->n_scan = 16;
  p->horizon_scan = 1800;
  p->ground_scan_ind = 7;
  p->segment_valid_point_num = 5;
  p->segment_valid_line_num = 3;
  p->ang_res_x = 0.2f;
  p->ang_res_y = 2.0f;
  p->ang_bottom = 15.0f + 0.1f;
  p->sensor_mount_angle = 0.0f;
  p->segment_theta = 1.0472f;
  p->edge_threshold = 0.1f;
  p->surf_threshold = 0.1f;
  p->leaf_size = 0.2f;
  p->scan_period = 0.1f;
  return SLIO_OK;
}

int slio_lego_create(slio_lego_handle* out, const slio_lego_params* p) {
  if (!out || !p) {
    set_error("slio_lego_create: null argument");
    return SLIO_EINVAL;
  }
  *out = nullptr;
  if (p->n_scan <= 1 || p->n_scan > 128 || p->horizon_scan <= 0 || p->horizon_scan > 8192 ||
      p->ground_scan_ind < 0 || p->ground_scan_ind >= p->n_scan || !(p->leaf_size > 0.0f) ||
      !(p->ang_res_x > 0.0f) || !(p->ang_res_y > 0.0f) || p->max_points < 0) {
    set_error("slio_lego_create: bad n_scan (2..128) / horizon_scan / ground_scan_ind / resolution / leaf");
    return SLIO_EINVAL;
  }
  int ndev = 0;
  LIO_HIP(hipGetDeviceCount(&ndev));
  if (p->device < 0 || p->device >= ndev) {
    set_error("slio_lego_create: no such HIP device");
    return SLIO_EDEVICE;
  }
  LIO_HIP(hipSetDevice(p->device));
  auto* h = new slio_lego();
  h->prm = *p;
  h->cells = (int64_t)p->n_scan * p->horizon_scan;
  h->cap = p->max_points > 0 ? p->max_points : 4 * h->cells;
  const float ax = (float)((double)p->ang_res_x / 180.0 * M_PI);
  const float ay = (float)((double)p->ang_res_y / 180.0 * M_PI);
  h->g = LGeo{p->n_scan, p->horizon_scan, p->ground_scan_ind, p->segment_valid_point_num,
              p->segment_valid_line_num, p->ang_res_x, p->ang_res_y, p->ang_bottom,
              p->sensor_mount_angle, p->segment_theta,
              (float)std::sin((double)ax), (float)std::cos((double)ax),
              (float)std::sin((double)ay), (float)std::cos((double)ay), h->cells};
  const int64_t C = h->cells, N = h->cap, R = p->n_scan;
  hipError_t e = hipStreamCreateWithFlags(&h->own, hipStreamNonBlocking);
  h->stream = h->own;
#define A(ptr, bytes) \
  if (!e) e = hipMalloc(reinterpret_cast<void**>(&(ptr)), (bytes))
  A(h->x, 4 * N);
  A(h->y, 4 * N);
  A(h->z, 4 * N);
  A(h->owner, 4 * C);
  A(h->owner_alt, 4 * C);
  if (!e) e = hipMemsetAsync(h->owner, 0xff, 4 * C, h->own);
  if (!e) e = hipMemsetAsync(h->owner_alt, 0xff, 4 * C, h->own);
  if (!e) e = hipStreamSynchronize(h->own);
  A(h->range_mat, 4 * C);
  A(h->full, 16 * C);
  A(h->ground, C);
  A(h->parent, 4 * C);
  A(h->edges, C);
  A(h->csize, 4 * C);
  A(h->rows, 16 * C);
  A(h->cnt, 12 * R);
  A(h->rsync, 20 * R * kLegoRowsSplit);
  A(h->rootlab, 4 * C);
  A(h->label, 4 * C);
  A(h->start_ring, 4 * R);
  A(h->end_ring, 4 * R);
  A(h->col_ind, 4 * C);
  A(h->nseg, 8);
  A(h->gflag, C);
  A(h->srange, 4 * C);
  A(h->sxyzi, 16 * C);
  A(h->outlier, 16 * C);
  A(h->slot, 4 * std::max<int64_t>((C + 255) / 256 + 1, R * kLegoRowsSplit));
  A(h->desk, 16 * C);
  A(h->io, sizeof(LegoImuOutDev));
  A(h->curvature, 4 * C);
  A(h->picked0, C);
  A(h->flabel, 4 * C);
  A(h->corner_stage, 16 * R * kCornerPerRing);
  A(h->corner_sharp, R * kCornerPerRing);
  A(h->corner_count, 4 * R);
  A(h->sharp_count, 4 * R);
  A(h->flat_count, 4 * R);
  A(h->surf_count, 4 * R);
  A(h->flat_stage, 16 * R * kFlatPerRing);
  A(h->surf_stage, 16 * C);
  A(h->c_sharp, 16 * R * kCornerPerRing);
  A(h->c_less_sharp, 16 * R * kCornerPerRing);
  A(h->c_flat, 16 * R * kFlatPerRing);
  A(h->c_less_flat, 16 * C);
  A(h->counts, 32);
#undef A
  if (!e) e = hipMemset(h->io, 0, sizeof(LegoImuOutDev));
  if (!e) e = hipMemset(h->rsync, 0, 20 * R * kLegoRowsSplit);
  if (e) {
    set_error(std::string("slio_lego_create: ") + hipGetErrorString(e));
    lego_free(h);
    delete h;
    return SLIO_ENOMEM;
  }
  const int H = p->horizon_scan;
  h->fc.edge_thr = p->edge_threshold;
  h->fc.surf_thr = p->surf_threshold;
  h->fc.leaf = p->leaf_size;
  h->fc.sort_cap = 64;
  while (h->fc.sort_cap < H / 6 + 2) h->fc.sort_cap <<= 1;
  h->fc.vox_cap = 64;
  while (h->fc.vox_cap < H) h->fc.vox_cap <<= 1;
  h->fc.ring_cap = H + 16;
  const FeatSmem fsm = feat_smem_sizes(h->fc);
  if (std::max(fsm.pick, fsm.ring) > 96 * 1024 || !sort_items(h->fc.sort_cap) ||
      !vox_items(h->fc.vox_cap)) {
    set_error("slio_lego_create: horizon_scan too large for the feature kernels' LDS layout");
    lego_free(h);
    delete h;
    return SLIO_EINVAL;
  }
  if (feat_work_alloc(h->fw, p->n_scan, h->fc) != hipSuccess) {
    set_error("slio_lego_create: out of device memory");
    lego_free(h);
    delete h;
    return SLIO_ENOMEM;
  }
  feat_set_smem<kModeLego>(fsm, sort_items(h->fc.sort_cap), vox_items(h->fc.vox_cap));
  // labelComponents in LDS when the image fits (SLIO_LEGO_CC_GLOBAL=1: the
  // global-atomic kernels, for A/B and tests)
  {
    const char* cg = std::getenv("SLIO_LEGO_CC_GLOBAL");
    h->cc_global = cg && cg[0] && cg[0] != '0';
    const char* c1 = std::getenv("SLIO_LEGO_CC_LDS1");
    h->cc_lds1 = c1 && c1[0] && c1[0] != '0';
    const char* rs = std::getenv("SLIO_LEGO_ROWS_SPLIT");
    h->rows_split = rs && rs[0] && rs[0] != '0';
  }
  if (lego_band_ok(h->g)) {
    const int nb = (h->g.H + kLegoBandW - 1) / kLegoBandW;
    if (hipMalloc(&h->seam, sizeof(LegoSeamRec) * 2 * (size_t)nb * h->g.N) != hipSuccess ||
        hipMalloc(&h->cc_arrive, sizeof(uint32_t)) != hipSuccess ||
        hipMemset(h->cc_arrive, 0, sizeof(uint32_t)) != hipSuccess) {
      set_error("slio_lego_create: out of device memory");
      lego_free(h);
      delete h;
      return SLIO_ENOMEM;
    }
  }
  if (h->cells <= kLegoCcCells) {
    // the attribute is the kernel's, for the whole process: set once to the
    // largest image the kernel takes, not to this handle's size
    static const hipError_t cc_attr = hipFuncSetAttribute(
        reinterpret_cast<const void*>(k_lego_cc), hipFuncAttributeMaxDynamicSharedMemorySize, 5 * kLegoCcCells);
    if (cc_attr != hipSuccess) {
      set_error(std::string("slio_lego_create: k_lego_cc LDS attribute: ") + hipGetErrorString(cc_attr));
      lego_free(h);
      delete h;
      return SLIO_EDEVICE;
    }
  }
  h->dev_counted = true;
  slio::dev_users(h->prm.device, +1);
  *out = h;
  return SLIO_OK;
}

int slio_lego_destroy(slio_lego_handle h) {
  if (!h) return SLIO_OK;
  (void)hipSetDevice(h->prm.device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  lego_free(h);
  if (h->dev_counted) slio::dev_users(h->prm.device, -1);
  delete h;
  return SLIO_OK;
}

int slio_lego_set_stream(slio_lego_handle h, void* stream) {
  LEGO_CHECK_H(h);
  h->stream = stream ? (hipStream_t)stream : h->own;
  return SLIO_OK;
}

int slio_lego_set_imu(slio_lego_handle h, const slio_lego_imu* m) {
  LEGO_CHECK_H(h);
  h->imu.on = 0;
  if (!m || m->pointer_last < 0) {
    h->imu.last = -1;
    h->imu_last_host = m ? m->pointer_last : 0;
    for (int a = 0; a < 3; ++a) h->imu.ang_last[a] = m ? m->ang_last[a] : 0.0f;
    return SLIO_OK;
  }
  if (m->que_len <= 0 || m->que_len > 65536 || m->pointer_last >= m->que_len ||
      m->pointer_last_iteration < 0 || m->pointer_last_iteration >= m->que_len || !m->time) {
    set_error("slio_lego_set_imu: bad que_len / pointers");
    return SLIO_EINVAL;
  }
  const int Q = m->que_len;
  if (Q > h->que) {
    if (h->itime) (void)hipFree(h->itime);
    if (h->iarr) (void)hipFree(h->iarr);
    h->itime = nullptr;
    h->iarr = nullptr;
    LIO_HIP(hipMalloc(&h->itime, 8 * Q));
    LIO_HIP(hipMalloc(&h->iarr, 4 * 12 * (size_t)Q));
    h->que = Q;
  }
  const float* arr[12] = {m->roll, m->pitch, m->yaw, m->velo_x, m->velo_y, m->velo_z,
                          m->shift_x, m->shift_y, m->shift_z, m->ang_x, m->ang_y, m->ang_z};
  for (int k = 0; k < 12; ++k)
    if (!arr[k]) {
      set_error("slio_lego_set_imu: null IMU array");
      return SLIO_EINVAL;
    }
  LIO_HIP(hipMemcpyAsync(h->itime, m->time, 8 * Q, hipMemcpyHostToDevice, h->stream));
  for (int k = 0; k < 12; ++k)
    LIO_HIP(hipMemcpyAsync(h->iarr + (size_t)k * Q, arr[k], 4 * Q, hipMemcpyHostToDevice, h->stream));
  LIO_HIP(hipStreamSynchronize(h->stream));
  float* a = h->iarr;
  h->imu = LegoImuDev{h->itime, a, a + Q, a + 2 * Q, a + 3 * Q, a + 4 * Q, a + 5 * Q,
                      a + 9 * Q, a + 10 * Q, a + 11 * Q, m->pointer_last,
                      m->pointer_last_iteration, Q, m->time_scan_cur,
                      {m->ang_last[0], m->ang_last[1], m->ang_last[2]}, 1, 0};
  {
    // the entries imu_at walks (last_it .. last on the ring): a binary search
    // when their times do not decrease
    const int L = (m->pointer_last - m->pointer_last_iteration + Q) % Q + 1;
    bool mono = true;
    for (int k = 1; k < L && mono; ++k) {
      const int a0 = (m->pointer_last_iteration + k - 1) % Q, a1 = (m->pointer_last_iteration + k) % Q;
      mono = m->time[a0] <= m->time[a1];
    }
    h->imu.seg = mono ? L : 0;
  }
  h->imu_last_host = m->pointer_last;
  return SLIO_OK;
}

int slio_lego_upload(slio_lego_handle h, const float* x, const float* y, const float* z, int64_t n) {
  LEGO_CHECK_H(h);
  if (n < 0 || (n > 0 && (!x || !y || !z))) {
    set_error("slio_lego_upload: bad arguments");
    return SLIO_EINVAL;
  }
  if (n > h->cap || n > INT32_MAX) {
    set_error("slio_lego_upload: scan exceeds max_points");
    return SLIO_ECAPACITY;
  }
  h->n = n;
  // findStartEndAngle (imageProjection.cpp:160-175)
  if (n >= 2) {
    const float so = -hfatan2(y[0], x[0]);
    float eo = (float)(-(double)hfatan2(y[n - 1], x[n - 2]) + 2 * M_PI);
    if (eo - so > 3 * M_PI)
      eo = (float)((double)eo - 2 * M_PI);
    else if (eo - so < M_PI)
      eo = (float)((double)eo + 2 * M_PI);
    h->orient[0] = so;
    h->orient[1] = eo;
    h->orient[2] = eo - so;
  } else {
    h->orient[0] = h->orient[1] = h->orient[2] = 0.0f;
  }
  if (n > 0) {
    LIO_HIP(hipMemcpyAsync(h->x, x, 4 * n, hipMemcpyHostToDevice, h->stream));
    LIO_HIP(hipMemcpyAsync(h->y, y, 4 * n, hipMemcpyHostToDevice, h->stream));
    LIO_HIP(hipMemcpyAsync(h->z, z, 4 * n, hipMemcpyHostToDevice, h->stream));
    LIO_HIP(hipStreamSynchronize(h->stream));
  }
  h->ran = false;
  return SLIO_OK;
}

int slio_lego_run_async(slio_lego_handle h) {
  LEGO_CHECK_H(h);
  const LGeo& g = h->g;
  const int R = g.N;
  const unsigned cb = (unsigned)((g.cells + 255) / 256);
  // labelComponents: column bands (default), one workgroup's LDS, or global
  // atomics (SLIO_LEGO_CC_LDS1 / SLIO_LEGO_CC_GLOBAL; all give the same labels)
  const bool cc_band = h->seam && !h->cc_global && !h->cc_lds1;
  const bool cc_lds = !cc_band && g.cells <= kLegoCcCells && !h->cc_global;
  // this sweep's owner table: the one the last sweep cleared; the swap is
  // committed only once k_lego_label (which clears the other table for the
  // next sweep) is enqueued, and a failed enqueue re-clears both tables
  int32_t* own = h->swept ? h->owner_alt : h->owner;
  int32_t* idle = h->swept ? h->owner : h->owner_alt;
  auto fail = [&](hipError_t e) {
    (void)hipGetLastError();
    (void)hipMemsetAsync(h->owner, 0xff, 4 * g.cells, h->stream);
    (void)hipMemsetAsync(h->owner_alt, 0xff, 4 * g.cells, h->stream);
    (void)hipStreamSynchronize(h->stream);
    h->swept = false;
    set_error(std::string("slio_lego_run_async: ") + hipGetErrorString(e));
    return SLIO_EDEVICE;
  };
  if (!cc_lds && !cc_band) {
    hipError_t e = hipMemsetAsync(h->csize, 0, 4 * g.cells, h->stream);
    if (!e) e = hipMemsetAsync(h->rows, 0, 16 * g.cells, h->stream);
    if (e) return fail(e);
  }
  std::pair<hipEvent_t, hipEvent_t> ev{nullptr, nullptr};
  if (h->prof) {
    if (h->pending.size() > 256) lego_prof_drain(h);
    if (!h->pool.empty()) {
      ev = h->pool.back();
      h->pool.pop_back();
    } else {
      LIO_HIP(hipEventCreate(&ev.first));
      LIO_HIP(hipEventCreate(&ev.second));
    }
    h->pending.push_back(ev);
  }
  // the events: in the first and last launches' dispatch packets (the whole
  // sweep), or around the feature stage
  const hipEvent_t e0 = h->prof_scan ? ev.first : nullptr, e1 = h->prof_scan ? ev.second : nullptr;
  if (h->n > 0)
    hipExtLaunchKernelGGL(k_lego_claim, dim3((unsigned)((h->n + 255) / 256)), dim3(256), 0, h->stream, e0, nullptr,
                          0, h->x, h->y, h->z, h->n, g, own);
  hipExtLaunchKernelGGL(k_lego_fill, dim3(cb), dim3(256), 0, h->stream, h->n > 0 ? nullptr : e0, nullptr, 0, h->x,
                        h->y, h->z, g, own, h->range_mat, h->full, h->ground);
  k_lego_ground<<<(g.H + 255) / 256, 256, 0, h->stream>>>(g, own, h->full, h->ground, h->parent,
                                                           !cc_lds && !cc_band);
  if (cc_band) {
    k_lego_cc_band<<<(g.H + kLegoBandW - 1) / kLegoBandW, kLegoBandThreads, 0, h->stream>>>(
        g, own, h->ground, h->range_mat, h->parent, h->csize, h->rows, h->seam, h->cc_arrive);
  } else if (cc_lds) {
    k_lego_edges<<<cb, 256, 0, h->stream>>>(g, own, h->ground, h->range_mat, h->edges, h->csize, h->rows);
    k_lego_cc<<<1, kLegoCcThreads, 5 * g.cells, h->stream>>>(g, h->edges, h->parent, h->csize, h->rows);
  } else {
    k_lego_union<<<cb, 256, 0, h->stream>>>(g, h->range_mat, h->parent);
    k_lego_compress<<<cb, 256, 0, h->stream>>>(g, h->parent, h->csize, h->rows);
  }
  const LegoSeg sg{h->start_ring, h->end_ring, h->col_ind, h->gflag, h->srange, h->sxyzi,
                   h->outlier, h->nseg};
  int nslot = (int)cb;
  if (!h->rows_split) {
    if (++h->sweep_seq == 0) h->sweep_seq = 1;
    k_lego_rows<<<R * kLegoRowsSplit, kLegoRowsThreads, 0, h->stream>>>(g, h->ground, h->parent, h->csize, h->rows, h->range_mat,
                                                      h->full, h->rootlab, sg, h->label, idle, h->rsync,
                                                      h->sweep_seq, h->orient[0], h->slot, h->io,
                                                      h->imu.ang_last[0], h->imu.ang_last[1], h->imu.ang_last[2]);
    nslot = R * kLegoRowsSplit;
  } else {
    k_lego_rowcount<<<R, kLegoRowThreads, 0, h->stream>>>(g, h->ground, h->parent, h->csize, h->rows,
                                                          h->cnt);
    k_lego_extract<<<R, kLegoRowThreads, 0, h->stream>>>(g, h->ground, h->parent, h->csize, h->rows,
                                                         h->cnt, h->range_mat, h->full, h->rootlab, sg);
    k_lego_label<<<cb, 256, 0, h->stream>>>(g, h->parent, h->csize, h->rows, h->rootlab, h->label, idle);
  }
  if (const hipError_t e = hipGetLastError()) return fail(e);
  h->owner = own;
  h->owner_alt = idle;
  h->swept = true;
  // adjustDistortion
  if (h->rows_split)
    k_lego_half<<<cb, 256, 0, h->stream>>>(h->sxyzi, h->nseg, h->orient[0], h->slot, h->io,
                                            h->imu.ang_last[0], h->imu.ang_last[1], h->imu.ang_last[2]);
  k_lego_deskew<<<cb, 256, 0, h->stream>>>(h->sxyzi, h->nseg, h->slot, nslot, h->orient[0],
                                            h->orient[1], h->orient[2], h->prm.scan_period, h->imu,
                                            h->desk, h->io);
  const CloudInfo ci{h->start_ring, h->end_ring, h->col_ind, h->srange, h->desk, h->nseg};
  const FeatOut fo{h->flabel, h->corner_stage, h->corner_count, h->surf_stage, h->surf_count,
                   h->corner_sharp, h->sharp_count, h->flat_stage, h->flat_count, h->gflag};
  launch_features<kModeLego>(h->stream, R, ci, h->curvature, h->picked0, h->fc, fo, h->fw,
                             h->prof_scan ? std::pair<hipEvent_t, hipEvent_t>{nullptr, nullptr} : ev);
  hipExtLaunchKernelGGL(k_lego_concat, dim3(R), dim3(kConcatThreads), 0, h->stream, nullptr, e1, 0, R,
                        h->start_ring, fo, h->c_sharp, h->c_less_sharp, h->c_flat, h->c_less_flat, h->counts);
  LIO_HIP(hipGetLastError());
  h->ran = true;
  return SLIO_OK;
}

int slio_lego_get_counts(slio_lego_handle h, slio_lego_counts* c) {
  LEGO_CHECK_H(h);
  if (!h->ran) {
    set_error("slio_lego: no scan processed");
    return SLIO_ESTATE;
  }
  int32_t ns[2];
  int64_t k[4];
  LIO_HIP(hipMemcpyAsync(ns, h->nseg, 8, hipMemcpyDeviceToHost, h->stream));
  LIO_HIP(hipMemcpyAsync(k, h->counts, 32, hipMemcpyDeviceToHost, h->stream));
  LIO_HIP(hipStreamSynchronize(h->stream));
  if (ns[0] < 0) {
    // k_lego_rows gave up waiting for an earlier ring's counts (~0.5 s): the
    // sweep's outputs are void; the next sweep's flags carry a new sequence
    set_error("slio_lego: the row stage's wait for an earlier ring gave up; this sweep's outputs are void");
    return SLIO_ETIMEOUT;
  }
  if (c) {
    c->n_segmented = ns[0];
    c->n_outlier = ns[1];
    c->n_sharp = k[0];
    c->n_less_sharp = k[1];
    c->n_flat = k[2];
    c->n_less_flat = k[3];
    for (int a = 0; a < 3; ++a) c->orientation[a] = h->orient[a];
  }
  return SLIO_OK;
}

int slio_lego_run(slio_lego_handle h, slio_lego_counts* c) {
  const int rc = slio_lego_run_async(h);
  if (rc) return rc;
  return slio_lego_get_counts(h, c);
}

int slio_lego_get_image(slio_lego_handle h, float* range_mat, int32_t* cell_point, int8_t* ground,
                        int32_t* label) {
  slio_lego_counts c;
  const int rc = slio_lego_get_counts(h, &c);
  if (rc) return rc;
  const int64_t C = h->cells;
  if (range_mat) LIO_HIP(hipMemcpyAsync(range_mat, h->range_mat, 4 * C, hipMemcpyDeviceToHost, h->stream));
  if (cell_point) LIO_HIP(hipMemcpyAsync(cell_point, h->owner, 4 * C, hipMemcpyDeviceToHost, h->stream));
  if (ground) LIO_HIP(hipMemcpyAsync(ground, h->ground, C, hipMemcpyDeviceToHost, h->stream));
  if (label) LIO_HIP(hipMemcpyAsync(label, h->label, 4 * C, hipMemcpyDeviceToHost, h->stream));
  LIO_HIP(hipStreamSynchronize(h->stream));
  return SLIO_OK;
}

int slio_lego_get_seg_info(slio_lego_handle h, int32_t* start_ring, int32_t* end_ring,
                           uint8_t* ground_flag, int32_t* col_ind, float* range, float* seg_xyzi,
                           float* outlier_xyzi) {
  slio_lego_counts c;
  const int rc = slio_lego_get_counts(h, &c);
  if (rc) return rc;
  const int64_t R = h->g.N, n = c.n_segmented, no = c.n_outlier;
  if (start_ring) LIO_HIP(hipMemcpyAsync(start_ring, h->start_ring, 4 * R, hipMemcpyDeviceToHost, h->stream));
  if (end_ring) LIO_HIP(hipMemcpyAsync(end_ring, h->end_ring, 4 * R, hipMemcpyDeviceToHost, h->stream));
  if (n > 0) {
    if (ground_flag) LIO_HIP(hipMemcpyAsync(ground_flag, h->gflag, n, hipMemcpyDeviceToHost, h->stream));
    if (col_ind) LIO_HIP(hipMemcpyAsync(col_ind, h->col_ind, 4 * n, hipMemcpyDeviceToHost, h->stream));
    if (range) LIO_HIP(hipMemcpyAsync(range, h->srange, 4 * n, hipMemcpyDeviceToHost, h->stream));
    if (seg_xyzi) LIO_HIP(hipMemcpyAsync(seg_xyzi, h->sxyzi, 16 * n, hipMemcpyDeviceToHost, h->stream));
  }
  if (outlier_xyzi && no > 0)
    LIO_HIP(hipMemcpyAsync(outlier_xyzi, h->outlier, 16 * no, hipMemcpyDeviceToHost, h->stream));
  LIO_HIP(hipStreamSynchronize(h->stream));
  return SLIO_OK;
}

int slio_lego_get_features(slio_lego_handle h, float* deskewed, float* curvature, uint8_t* picked,
                           int32_t* label, slio_lego_imu_out* imu_out) {
  slio_lego_counts c;
  const int rc = slio_lego_get_counts(h, &c);
  if (rc) return rc;
  const int64_t n = c.n_segmented;
  if (n > 0) {
    if (deskewed) LIO_HIP(hipMemcpyAsync(deskewed, h->desk, 16 * n, hipMemcpyDeviceToHost, h->stream));
    if (curvature) LIO_HIP(hipMemcpyAsync(curvature, h->curvature, 4 * n, hipMemcpyDeviceToHost, h->stream));
    if (picked) LIO_HIP(hipMemcpyAsync(picked, h->picked0, n, hipMemcpyDeviceToHost, h->stream));
    if (label) LIO_HIP(hipMemcpyAsync(label, h->flabel, 4 * n, hipMemcpyDeviceToHost, h->stream));
  }
  LegoImuOutDev io;
  LIO_HIP(hipMemcpyAsync(&io, h->io, sizeof(io), hipMemcpyDeviceToHost, h->stream));
  LIO_HIP(hipStreamSynchronize(h->stream));
  if (imu_out) {
    std::memcpy(imu_out->rpy_start, io.rpy_start, sizeof(io.rpy_start));
    std::memcpy(imu_out->rpy_cur, io.rpy_cur, sizeof(io.rpy_cur));
    std::memcpy(imu_out->velo_from_start, io.velo_from_start, sizeof(io.velo_from_start));
    std::memcpy(imu_out->angular_from_start, io.angular_from_start, sizeof(io.angular_from_start));
    std::memcpy(imu_out->ang_last, io.ang_last, sizeof(io.ang_last));
    imu_out->pointer_last_iteration = h->imu_last_host;  // :804
  }
  return SLIO_OK;
}

int slio_lego_get_clouds(slio_lego_handle h, float* sharp, float* less_sharp, float* flat,
                         float* less_flat) {
  slio_lego_counts c;
  const int rc = slio_lego_get_counts(h, &c);
  if (rc) return rc;
  if (sharp && c.n_sharp > 0)
    LIO_HIP(hipMemcpyAsync(sharp, h->c_sharp, 16 * c.n_sharp, hipMemcpyDeviceToHost, h->stream));
  if (less_sharp && c.n_less_sharp > 0)
    LIO_HIP(hipMemcpyAsync(less_sharp, h->c_less_sharp, 16 * c.n_less_sharp, hipMemcpyDeviceToHost, h->stream));
  if (flat && c.n_flat > 0)
    LIO_HIP(hipMemcpyAsync(flat, h->c_flat, 16 * c.n_flat, hipMemcpyDeviceToHost, h->stream));
  if (less_flat && c.n_less_flat > 0)
    LIO_HIP(hipMemcpyAsync(less_flat, h->c_less_flat, 16 * c.n_less_flat, hipMemcpyDeviceToHost, h->stream));
  LIO_HIP(hipStreamSynchronize(h->stream));
  return SLIO_OK;
}

int slio_lego_profile(slio_lego_handle h, int enable) {
  LEGO_CHECK_H(h);
  const bool keep = (enable & SLIO_LIO_PROFILE_KEEP) != 0;
  h->prof = (enable & ~SLIO_LIO_PROFILE_KEEP) != 0;
  h->prof_scan = (enable & SLIO_LIO_PROFILE_SCAN) != 0;
  if (!keep) {
    lego_prof_drain(h);
    h->prof_ms = 0.0;
    h->prof_n = 0;
  }
  return SLIO_OK;
}

int slio_lego_profile_read(slio_lego_handle h, double* ms, int64_t* launches) {
  LEGO_CHECK_H(h);
  LIO_HIP(hipStreamSynchronize(h->stream));
  lego_prof_drain(h);
  if (ms) *ms = h->prof_ms;
  if (launches) *launches = h->prof_n;
  return SLIO_OK;
}

}  // extern "C"
