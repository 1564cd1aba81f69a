// slio_device.hip — MI355X (gfx950) device runtime of the IKF scan-matching core.
//
// Replaces, for one scan against a static map snapshot:
//   * KD_TREE::Build / Nearest_Search (ikd_Tree.cpp:355-402, Search :960-1101)
//     -> a dense uniform-grid index in HBM (points sorted by cell, float4
//        {x, y, z, map index}) and an exact 5-NN search that walks x-runs of
//        cells with 8 lanes per query and merges per-lane top-5 lists with
//        wave shuffles;
//   * esekf::h_share_model (esekfom.hpp:106-227) -> one fused kernel per pass:
//        body->world transform, kNN gate, esti_plane, residual gate, Jacobian
//        row, and the H^T H / H^T h products (esekfom.hpp:306-319) reduced in
//        fp64 per 128-point chunk in a fixed order;
//   * the reduction tree -> chunk partials -> 8 super-chunk sums (fixed order)
//     so 1/2/4/8 GPUs give bitwise-identical sums.
// Built with -ffp-contract=off: every float/double expression is evaluated
// exactly as written (the reference's x86-64 build has no FMA either).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "slio_common.hpp"
#include "slio_plane.hpp"

namespace slio {

static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }

#define SLIO_HIP(call)                                                          \
  do {                                                                          \
    hipError_t e_ = (call);                                                     \
    if (e_ != hipSuccess) {                                                     \
      set_error(std::string(#call) + ": " + hipGetErrorString(e_));             \
      return SLIO_EDEVICE;                                                      \
    }                                                                           \
  } while (0)

constexpr int kLPQ = 8;                          // lanes per query
constexpr int kBlock = 256;                      // threads per search workgroup
constexpr int kQPP = kBlock / kLPQ;              // queries per pass (32)
constexpr int kPasses = SLIO_CHUNK / kQPP;       // passes per chunk (4)
constexpr uint64_t kInfKey = ~0ull;

static_assert(SLIO_CHUNK % kQPP == 0, "chunk must be a multiple of queries/pass");

__constant__ uint8_t c_pa[SLIO_NPROD];
__constant__ uint8_t c_pb[SLIO_NPROD];

// ---------------------------------------------------------------- map index
struct GridGeom {
  float ox, oy, oz;   // origin = bbox min
  float h, inv_h;     // cell edge and its reciprocal
  float tol;          // conservative slack on cell-boundary coordinates
  int dx, dy, dz;     // dims
};

struct MapDev {
  GridGeom g;
  int64_t n = 0;
  int64_t ncells = 0;
  float4* pts = nullptr;          // sorted by cell: x, y, z, bits(map index)
  uint32_t* start = nullptr;      // ncells + 1 prefix offsets
  int device = 0;
  ~MapDev() {
    if (pts) (void)hipFree(pts);
    if (start) (void)hipFree(start);
  }
};

// trivially-copyable kernel argument view of a MapDev
struct MapView {
  GridGeom g;
  int64_t n;
  const float4* pts;
  const uint32_t* start;
};

__device__ __host__ __forceinline__ int cell_coord(float p, float o, float inv_h) {
  float t = floorf((p - o) * inv_h);
  t = fminf(fmaxf(t, -1.0e8f), 1.0e8f);
  return (int)t;
}

__global__ void k_cell_keys(const float* __restrict__ x, const float* __restrict__ y,
                            const float* __restrict__ z, int64_t n, GridGeom g,
                            uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int cx = min(max(cell_coord(x[i], g.ox, g.inv_h), 0), g.dx - 1);
  int cy = min(max(cell_coord(y[i], g.oy, g.inv_h), 0), g.dy - 1);
  int cz = min(max(cell_coord(z[i], g.oz, g.inv_h), 0), g.dz - 1);
  keys[i] = ((uint32_t)cz * (uint32_t)g.dy + (uint32_t)cy) * (uint32_t)g.dx + (uint32_t)cx;
  vals[i] = (uint32_t)i;
}

__global__ void k_cell_hist(const uint32_t* __restrict__ keys, int64_t n,
                            uint32_t* __restrict__ counts) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  atomicAdd(&counts[keys[i]], 1u);
}

__global__ void k_gather_sorted(const float* __restrict__ x, const float* __restrict__ y,
                                const float* __restrict__ z, const uint32_t* __restrict__ order,
                                int64_t n, float4* __restrict__ pts) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t o = order[i];
  pts[i] = make_float4(x[o], y[o], z[o], __uint_as_float(o));
}

// ---------------------------------------------------------------- math helpers
struct PoseDev {
  double rq[4], pos[3], lq[4], tli[3];  // quaternions (w, x, y, z)
  double R[9];                          // rot.matrix(), row-major
  double RL[9];                         // offset_R_L_I.matrix(), row-major
};

// Sophus::SO3::operator*(Vector3d) = Eigen QuaternionBase::_transformVector:
// uv = q.vec() x v; uv += uv; return v + q.w() * uv + q.vec() x uv;
__device__ __forceinline__ void qrot(const double (&q)[4], const double (&v)[3], double (&o)[3]) {
  double ux = q[2] * v[2] - q[3] * v[1];
  double uy = q[3] * v[0] - q[1] * v[2];
  double uz = q[1] * v[1] - q[2] * v[0];
  ux = ux + ux;
  uy = uy + uy;
  uz = uz + uz;
  const double cx = q[2] * uz - q[3] * uy;
  const double cy = q[3] * ux - q[1] * uz;
  const double cz = q[1] * uy - q[2] * ux;
  o[0] = (v[0] + q[0] * ux) + cx;
  o[1] = (v[1] + q[0] * uy) + cy;
  o[2] = (v[2] + q[0] * uz) + cz;
}

// 3-term dot in Eigen's unrolled order for a fixed 3-vector: a0b0 + (a1b1 + a2b2)
__device__ __forceinline__ double dot3(double a0, double a1, double a2, double b0, double b1,
                                       double b2) {
  return a0 * b0 + (a1 * b1 + a2 * b2);
}

// Jacobian row of esekfom.hpp:197-226 for one effective point.
__device__ __forceinline__ void jacobian_row(const PoseDev& P, float bx, float by, float bz,
                                             float nx, float ny, float nz, bool extrinsic,
                                             double (&row)[12]) {
  const double pb[3] = {(double)bx, (double)by, (double)bz};
  double pI[3];
  qrot(P.lq, pb, pI);
  pI[0] = pI[0] + P.tli[0];
  pI[1] = pI[1] + P.tli[1];
  pI[2] = pI[2] + P.tli[2];
  const double n0 = nx, n1 = ny, n2 = nz;
  // C = rot.matrix()^T * n
  const double C0 = dot3(P.R[0], P.R[3], P.R[6], n0, n1, n2);
  const double C1 = dot3(P.R[1], P.R[4], P.R[7], n0, n1, n2);
  const double C2 = dot3(P.R[2], P.R[5], P.R[8], n0, n1, n2);
  // A = [pI]x * C with SKEW_SYM_MATRX rows (0,-v2,v1), (v2,0,-v0), (-v1,v0,0)
  const double A0 = dot3(0.0, -pI[2], pI[1], C0, C1, C2);
  const double A1 = dot3(pI[2], 0.0, -pI[0], C0, C1, C2);
  const double A2 = dot3(-pI[1], pI[0], 0.0, C0, C1, C2);
  double B0 = 0.0, B1 = 0.0, B2 = 0.0;
  if (extrinsic) {
    // B = ([p_b]x * R_LI^T) * C
    const double S[9] = {0.0, -pb[2], pb[1], pb[2], 0.0, -pb[0], -pb[1], pb[0], 0.0};
    double M[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j)  // (R_LI^T)(k, j) = RL[j*3+k]
        M[i * 3 + j] = dot3(S[i * 3 + 0], S[i * 3 + 1], S[i * 3 + 2], P.RL[j * 3 + 0],
                            P.RL[j * 3 + 1], P.RL[j * 3 + 2]);
    B0 = dot3(M[0], M[1], M[2], C0, C1, C2);
    B1 = dot3(M[3], M[4], M[5], C0, C1, C2);
    B2 = dot3(M[6], M[7], M[8], C0, C1, C2);
  }
  row[0] = n0;
  row[1] = n1;
  row[2] = n2;
  row[3] = A0;
  row[4] = A1;
  row[5] = A2;
  row[6] = B0;
  row[7] = B1;
  row[8] = B2;
  row[9] = C0;
  row[10] = C1;
  row[11] = C2;
}

// body -> world in double, rounded to the float query (esekfom.hpp:128-132)
__device__ __forceinline__ void body_to_world(const PoseDev& P, float bx, float by, float bz,
                                              float& wx, float& wy, float& wz) {
  const double pb[3] = {(double)bx, (double)by, (double)bz};
  double a[3];
  qrot(P.lq, pb, a);
  a[0] = a[0] + P.tli[0];
  a[1] = a[1] + P.tli[1];
  a[2] = a[2] + P.tli[2];
  double w[3];
  qrot(P.rq, a, w);
  wx = (float)(w[0] + P.pos[0]);
  wy = (float)(w[1] + P.pos[1]);
  wz = (float)(w[2] + P.pos[2]);
}

// residual + range gate of esekfom.hpp:159-164; returns s > 0.9
__device__ __forceinline__ bool residual_gate(const float (&abcd)[4], float wx, float wy,
                                              float wz, float bx, float by, float bz,
                                              float& pd2) {
  pd2 = ((abcd[0] * wx + abcd[1] * wy) + abcd[2] * wz) + abcd[3];
  const double X = bx, Y = by, Z = bz;
  const double nrm = sqrt((X * X + Y * Y) + Z * Z);
  const float s = (float)(1.0 - (0.9 * (double)fabsf(pd2)) / sqrt(nrm));
  return (double)s > 0.9;
}

// ---------------------------------------------------------------- top-5
__device__ __forceinline__ void insert5(uint64_t key, uint32_t pos, uint64_t (&k)[5],
                                        uint32_t (&p)[5]) {
  if (key < k[4]) {
    k[4] = key;
    p[4] = pos;
#pragma unroll
    for (int j = 4; j > 0; --j) {
      const bool sw = k[j] < k[j - 1];
      const uint64_t ka = k[j - 1], kb = k[j];
      const uint32_t pa = p[j - 1], pb = p[j];
      k[j - 1] = sw ? kb : ka;
      k[j] = sw ? ka : kb;
      p[j - 1] = sw ? pb : pa;
      p[j] = sw ? pa : pb;
    }
  }
}

__device__ __forceinline__ void consider(const float4 c, uint32_t pos, float qx, float qy,
                                         float qz, uint64_t (&k)[5], uint32_t (&p)[5]) {
  const float ddx = qx - c.x, ddy = qy - c.y, ddz = qz - c.z;
  const float d = (ddx * ddx + ddy * ddy) + ddz * ddz;
  const uint64_t key = ((uint64_t)__float_as_uint(d) << 32) | (uint64_t)__float_as_uint(c.w);
  insert5(key, pos, k, p);
}

// butterfly merge of the kLPQ per-lane lists of a query group
__device__ __forceinline__ void group_merge(uint64_t (&k)[5], uint32_t (&p)[5]) {
#pragma unroll
  for (int m = 1; m < kLPQ; m <<= 1) {
    uint64_t ok[5];
    uint32_t op[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      ok[j] = __shfl_xor(k[j], m);
      op[j] = __shfl_xor(p[j], m);
    }
#pragma unroll
    for (int j = 0; j < 5; ++j) insert5(ok[j], op[j], k, p);
  }
}

// Scan all candidates of cube [c-r, c+r]^3 minus cube [c-rin, c+rin]^3
// (rin < 0: nothing excluded), clamped to the grid; lanes stride over runs.
__device__ void scan_region(const float4* __restrict__ pts,
                            const uint32_t* __restrict__ start, const GridGeom& g, int cx,
                            int cy, int cz, int r, int rin, int sub, float qx, float qy,
                            float qz, uint64_t (&k)[5], uint32_t (&p)[5]) {
  const int z0 = max(cz - r, 0), z1 = min(cz + r, g.dz - 1);
  const int y0 = max(cy - r, 0), y1 = min(cy + r, g.dy - 1);
  const int xlo = max(cx - r, 0), xhi = min(cx + r, g.dx - 1);
  if (xlo > xhi) return;
  for (int zz = z0; zz <= z1; ++zz) {
    for (int yy = y0; yy <= y1; ++yy) {
      const bool inner_row = rin >= 0 && abs(zz - cz) <= rin && abs(yy - cy) <= rin;
      const uint32_t rowbase = ((uint32_t)zz * (uint32_t)g.dy + (uint32_t)yy) * (uint32_t)g.dx;
      // up to two x segments
      int sa0, sa1, sb0, sb1;
      if (!inner_row) {
        sa0 = xlo;
        sa1 = xhi;
        sb0 = 1;
        sb1 = 0;
      } else {
        sa0 = xlo;
        sa1 = min(cx - rin - 1, xhi);
        sb0 = max(cx + rin + 1, xlo);
        sb1 = xhi;
      }
#pragma unroll
      for (int seg = 0; seg < 2; ++seg) {
        const int a0 = seg ? sb0 : sa0, a1 = seg ? sb1 : sa1;
        if (a0 > a1) continue;
        const uint32_t s = start[rowbase + a0];
        const uint32_t e = start[rowbase + a1 + 1];
        for (uint32_t j = s + sub; j < e; j += kLPQ) consider(pts[j], j, qx, qy, qz, k, p);
      }
    }
  }
}

// Exactness bound: every map point outside cube [c-r, c+r] lies at least this
// far from q (minus float slack); +inf when the cube covers the grid.
__device__ __forceinline__ float outside_bound(const GridGeom& g, int cx, int cy, int cz, int r,
                                               float qx, float qy, float qz, bool& covers) {
  const float INF = __int_as_float(0x7f800000);
  float b = INF;
  covers = true;
  auto axis = [&](int c, int d, float o, float q) {
    if (c - r > 0) {
      covers = false;
      const float face = o + (float)(c - r) * g.h + g.tol;
      b = fminf(b, q - face);
    }
    if (c + r < d - 1) {
      covers = false;
      const float face = o + (float)(c + r + 1) * g.h - g.tol;
      b = fminf(b, face - q);
    }
  };
  axis(cx, g.dx, g.ox, qx);
  axis(cy, g.dy, g.oy, qy);
  axis(cz, g.dz, g.oz, qz);
  return b;
}

// ---------------------------------------------------------------- kernels
struct ScanDev {
  const float* bx;
  const float* by;
  const float* bz;
  int64_t n;
};

struct PassOut {
  int32_t* nbr_idx;  // n * 5
  float* nbr_sqd;    // n * 5
  float4* plane;     // n
  uint8_t* sel;      // n
  float* resid;      // n
  double* chunk_part;  // C * NPROD (global chunk index)
};

struct PassCfg {
  float plane_thr;
  float max_sqd;
  int extrinsic;
  int64_t c_begin, c_end;  // global chunk range of this rank
};

__device__ __forceinline__ int64_t xcd_chunk(int64_t c_begin, int64_t nblk) {
  // blocks b and b+8 share an XCD: give each XCD group a contiguous chunk range
  const int64_t b = blockIdx.x;
  const int64_t xcd = b & 7, q = nblk >> 3, rr = nblk & 7;
  const int64_t base = xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q;
  return c_begin + base + (b >> 3);
}

// fixed-order product phase: rows[SLIO_CHUNK][kRow] in LDS -> chunk partial
template <int NT>
__device__ __forceinline__ void chunk_products(const double (*rows)[kRow], double (*part)[SLIO_NPROD],
                                               double* __restrict__ out) {
  constexpr int kSplit = NT / 128;                 // row halves handled in parallel
  constexpr int kRowsPer = SLIO_CHUNK / kSplit;
  const int t = threadIdx.x;
  const int half = t >> 7, kk = t & 127;
  if (kk < SLIO_NPROD && half < kSplit) {
    const int a = c_pa[kk], b = c_pb[kk];
    double s = 0.0;
    const int r0 = half * kRowsPer;
    for (int r = r0; r < r0 + kRowsPer; ++r) s = s + rows[r][a] * rows[r][b];
    part[half][kk] = s;
  }
  __syncthreads();
  if (t < SLIO_NPROD) {
    double s = part[0][t];
#pragma unroll
    for (int h = 1; h < kSplit; ++h) s = s + part[h][t];
    out[t] = s;
  }
}

__global__ __launch_bounds__(kBlock) void k_search_pass(const MapView map, const ScanDev scan,
                                                        const PoseDev pose, const PassCfg cfg,
                                                        const PassOut out) {
  __shared__ double rows[SLIO_CHUNK][kRow];
  __shared__ double part[kBlock / 128][SLIO_NPROD];
  const int64_t chunk = xcd_chunk(cfg.c_begin, cfg.c_end - cfg.c_begin);
  const int tid = threadIdx.x;
  const int sub = tid & (kLPQ - 1);
  const int grp = tid / kLPQ;
  const GridGeom g = map.g;
  const float4* __restrict__ pts = map.pts;
  const uint32_t* __restrict__ start = map.start;

  for (int pass = 0; pass < kPasses; ++pass) {
    const int slot = pass * kQPP + grp;
    const int64_t i = chunk * SLIO_CHUNK + slot;
    double row[kRow];
#pragma unroll
    for (int j = 0; j < kRow; ++j) row[j] = 0.0;
    if (i < scan.n) {
      const float bx = scan.bx[i], by = scan.by[i], bz = scan.bz[i];
      float qx, qy, qz;
      body_to_world(pose, bx, by, bz, qx, qy, qz);

      uint64_t k[5];
      uint32_t p[5];
#pragma unroll
      for (int j = 0; j < 5; ++j) {
        k[j] = kInfKey;
        p[j] = 0;
      }
      const bool finite = isfinite(qx) && isfinite(qy) && isfinite(qz) && map.n > 0;
      if (finite) {
        const int cx = cell_coord(qx, g.ox, g.inv_h);
        const int cy = cell_coord(qy, g.oy, g.inv_h);
        const int cz = cell_coord(qz, g.oz, g.inv_h);
        const int ex = max(max(-cx, cx - (g.dx - 1)), 0);
        const int ey = max(max(-cy, cy - (g.dy - 1)), 0);
        const int ez = max(max(-cz, cz - (g.dz - 1)), 0);
        int r = max(1, max(ex, max(ey, ez)));
        int rin = -1;
        if (r == 1) {
          // fast path: 3x3x3 block = 9 x-runs; issue the 18 run bounds first
          uint32_t rs[9], rl[9];
          const int xlo = max(cx - 1, 0), xhi = min(cx + 1, g.dx - 1);
#pragma unroll
          for (int q = 0; q < 9; ++q) {
            const int yy = cy - 1 + (q % 3), zz = cz - 1 + (q / 3);
            const bool ok = yy >= 0 && yy < g.dy && zz >= 0 && zz < g.dz && xlo <= xhi;
            const uint32_t rb = ok ? ((uint32_t)zz * (uint32_t)g.dy + (uint32_t)yy) * (uint32_t)g.dx : 0u;
            const uint32_t s = ok ? start[rb + xlo] : 0u;
            const uint32_t e = ok ? start[rb + xhi + 1] : 0u;
            rs[q] = s;
            rl[q] = e - s;
          }
          uint32_t pre[10];
          pre[0] = 0;
#pragma unroll
          for (int q = 0; q < 9; ++q) pre[q + 1] = pre[q] + rl[q];
          const uint32_t T = pre[9];
          for (uint32_t t0 = sub; t0 < T; t0 += 2 * kLPQ) {
            const uint32_t t1 = t0 + kLPQ;
            uint32_t a0 = 0, a1 = 0;
#pragma unroll
            for (int q = 0; q < 9; ++q) {
              if (t0 >= pre[q]) a0 = rs[q] + (t0 - pre[q]);
              if (t1 >= pre[q]) a1 = rs[q] + (t1 - pre[q]);
            }
            const float4 c0 = pts[a0];
            float4 c1 = make_float4(0.f, 0.f, 0.f, 0.f);
            if (t1 < T) c1 = pts[a1];
            consider(c0, a0, qx, qy, qz, k, p);
            if (t1 < T) consider(c1, a1, qx, qy, qz, k, p);
          }
          group_merge(k, p);
          rin = 1;
          r = 2;
          bool covers;
          const float b = outside_bound(g, cx, cy, cz, 1, qx, qy, qz, covers);
          const float d5 = __uint_as_float((uint32_t)(k[4] >> 32));
          const bool done = covers || (k[4] != kInfKey && b > 0.0f && d5 < (b * b) * 0.99999f);
          if (!done && sub != 0) {
#pragma unroll
            for (int j = 0; j < 5; ++j) k[j] = kInfKey;
          }
          if (done) r = -1;
        }
        // general rings (rare): expand until the 5th distance is provably final
        while (r > 0) {
          scan_region(pts, start, g, cx, cy, cz, r, rin, sub, qx, qy, qz, k, p);
          group_merge(k, p);
          bool covers;
          const float b = outside_bound(g, cx, cy, cz, r, qx, qy, qz, covers);
          const float d5 = __uint_as_float((uint32_t)(k[4] >> 32));
          const bool done = covers || (k[4] != kInfKey && b > 0.0f && d5 < (b * b) * 0.99999f);
          if (done) break;
          if (sub != 0) {
#pragma unroll
            for (int j = 0; j < 5; ++j) k[j] = kInfKey;
          }
          rin = r;
          ++r;
        }
      }

      // Nearest_Points / pointSearchSqDis for this point
      if (sub < 5) {
        uint64_t mk = k[0];
#pragma unroll
        for (int j = 1; j < 5; ++j) mk = (sub == j) ? k[j] : mk;
        out.nbr_idx[i * 5 + sub] = (mk == kInfKey) ? -1 : (int32_t)(uint32_t)mk;
        out.nbr_sqd[i * 5 + sub] =
            (mk == kInfKey) ? __int_as_float(0x7f800000) : __uint_as_float((uint32_t)(mk >> 32));
      }
      // kNN gate (esekfom.hpp:144-147)
      const float d5 = __uint_as_float((uint32_t)(k[4] >> 32));
      bool sel = (k[4] != kInfKey) && !(d5 > cfg.max_sqd);
      float abcd[4] = {__int_as_float(0x7fc00000), __int_as_float(0x7fc00000),
                       __int_as_float(0x7fc00000), __int_as_float(0x7fc00000)};
      float pd2 = __int_as_float(0x7fc00000);
      if (sel) {
        float nb[5][3];
#pragma unroll
        for (int j = 0; j < 5; ++j) {
          const float4 c = pts[p[j]];
          nb[j][0] = c.x;
          nb[j][1] = c.y;
          nb[j][2] = c.z;
        }
        float pl[4];
        sel = esti_plane_dev(nb, cfg.plane_thr, pl);
        if (sel) {
#pragma unroll
          for (int j = 0; j < 4; ++j) abcd[j] = pl[j];
          sel = residual_gate(abcd, qx, qy, qz, bx, by, bz, pd2);
        }
      }
      if (sub == 0) {
        out.plane[i] = make_float4(abcd[0], abcd[1], abcd[2], abcd[3]);
        out.sel[i] = sel ? 1 : 0;
        out.resid[i] = sel ? pd2 : __int_as_float(0x7fc00000);
      }
      if (sel) {
        double h[12];
        jacobian_row(pose, bx, by, bz, abcd[0], abcd[1], abcd[2], cfg.extrinsic != 0, h);
#pragma unroll
        for (int j = 0; j < 12; ++j) row[j] = h[j];
        row[12] = -(double)pd2;
        row[13] = 1.0;
      }
    }
    // lanes of the group write the row cooperatively
#pragma unroll
    for (int j = 0; j < kRow; ++j)
      if ((j & (kLPQ - 1)) == sub) rows[slot][j] = row[j];
  }
  __syncthreads();
  chunk_products<kBlock>(rows, part, out.chunk_part + chunk * SLIO_NPROD);
}

// Non-search pass: reuse neighbours/plane/selection (esekfom.hpp:138-150 with
// converge == false), one lane per point.
__global__ __launch_bounds__(SLIO_CHUNK) void k_reuse_pass(const ScanDev scan, const PoseDev pose,
                                                           const PassCfg cfg, const PassOut out) {
  __shared__ double rows[SLIO_CHUNK][kRow];
  __shared__ double part[1][SLIO_NPROD];
  const int64_t chunk = xcd_chunk(cfg.c_begin, cfg.c_end - cfg.c_begin);
  const int t = threadIdx.x;
  const int64_t i = chunk * SLIO_CHUNK + t;
  double row[kRow];
#pragma unroll
  for (int j = 0; j < kRow; ++j) row[j] = 0.0;
  if (i < scan.n) {
    bool sel = out.sel[i] != 0;
    float pd2 = __int_as_float(0x7fc00000);
    if (sel) {
      const float bx = scan.bx[i], by = scan.by[i], bz = scan.bz[i];
      float qx, qy, qz;
      body_to_world(pose, bx, by, bz, qx, qy, qz);
      const float4 pl = out.plane[i];
      const float abcd[4] = {pl.x, pl.y, pl.z, pl.w};
      sel = residual_gate(abcd, qx, qy, qz, bx, by, bz, pd2);
      if (sel) {
        double h[12];
        jacobian_row(pose, bx, by, bz, abcd[0], abcd[1], abcd[2], cfg.extrinsic != 0, h);
#pragma unroll
        for (int j = 0; j < 12; ++j) row[j] = h[j];
        row[12] = -(double)pd2;
        row[13] = 1.0;
      }
      out.sel[i] = sel ? 1 : 0;
    }
    out.resid[i] = sel ? pd2 : __int_as_float(0x7fc00000);
  }
#pragma unroll
  for (int j = 0; j < kRow; ++j) rows[t][j] = row[j];
  __syncthreads();
  chunk_products<SLIO_CHUNK>(rows, part, out.chunk_part + chunk * SLIO_NPROD);
}

// super-chunk sums in fixed chunk order; rows of super-chunks this rank does
// not own are written as zeros.
__global__ __launch_bounds__(128) void k_super_sums(const double* __restrict__ chunk_part,
                                                    int64_t C, int s_begin, int s_end,
                                                    double* __restrict__ super_out) {
  const int s = blockIdx.x;
  const int t = threadIdx.x;
  if (t >= SLIO_NPROD) return;
  double acc = 0.0;
  if (s >= s_begin && s < s_end) {
    const int64_t c0 = super_lo(C, s), c1 = super_lo(C, s + 1);
    for (int64_t c = c0; c < c1; ++c) acc = acc + chunk_part[c * SLIO_NPROD + t];
  }
  super_out[s * SLIO_NPROD + t] = acc;
}

// ---------------------------------------------------------------- context
struct Ctx {
  slio_params prm{};
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  std::shared_ptr<MapDev> map;
  // scan
  int64_t n = 0;
  float* bx = nullptr;
  float* by = nullptr;
  float* bz = nullptr;
  int32_t* nbr_idx = nullptr;
  float* nbr_sqd = nullptr;
  float4* plane = nullptr;
  uint8_t* sel = nullptr;
  float* resid = nullptr;
  double* chunk_part = nullptr;
  double* d_super = nullptr;
  double* d_super_own = nullptr;
  double* h_super = nullptr;  // pinned
  bool searched = false;
  // profiling: event pairs pending per kind, accumulated time
  bool prof = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending[3];
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pool;
  double prof_ms[3] = {0, 0, 0};
  int64_t prof_n[3] = {0, 0, 0};
};

static std::pair<hipEvent_t, hipEvent_t> prof_pair(Ctx& c) {
  if (!c.pool.empty()) {
    auto p = c.pool.back();
    c.pool.pop_back();
    return p;
  }
  std::pair<hipEvent_t, hipEvent_t> p{nullptr, nullptr};
  (void)hipEventCreate(&p.first);
  (void)hipEventCreate(&p.second);
  return p;
}

static void prof_drain(Ctx& c) {
  for (int k = 0; k < 3; ++k) {
    for (auto& p : c.pending[k]) {
      float ms = 0.f;
      if (hipEventSynchronize(p.second) == hipSuccess &&
          hipEventElapsedTime(&ms, p.first, p.second) == hipSuccess) {
        c.prof_ms[k] += ms;
        c.prof_n[k] += 1;
      }
      c.pool.push_back(p);
    }
    c.pending[k].clear();
  }
}

static int init_constants() {
  static bool done = false;
  if (done) return SLIO_OK;
  uint8_t pa[SLIO_NPROD], pb[SLIO_NPROD];
  product_table(pa, pb);
  SLIO_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_pa), pa, sizeof(pa)));
  SLIO_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_pb), pb, sizeof(pb)));
  done = true;
  return SLIO_OK;
}

static PoseDev make_pose(const slio_pose* x) {
  PoseDev P;
  for (int j = 0; j < 4; ++j) {
    P.rq[j] = x->rot[j];
    P.lq[j] = x->rli[j];
  }
  for (int j = 0; j < 3; ++j) {
    P.pos[j] = x->pos[j];
    P.tli[j] = x->tli[j];
  }
  // Eigen QuaternionBase::toRotationMatrix
  auto tomat = [](const double* q, double* R) {
    const double w = q[0], x = q[1], y = q[2], z = q[3];
    const double tx = 2.0 * x, ty = 2.0 * y, tz = 2.0 * z;
    const double twx = tx * w, twy = ty * w, twz = tz * w;
    const double txx = tx * x, txy = ty * x, txz = tz * x;
    const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
    R[0] = 1.0 - (tyy + tzz);
    R[1] = txy - twz;
    R[2] = txz + twy;
    R[3] = txy + twz;
    R[4] = 1.0 - (txx + tzz);
    R[5] = tyz - twx;
    R[6] = txz - twy;
    R[7] = tyz + twx;
    R[8] = 1.0 - (txx + tyy);
  };
  tomat(x->rot, P.R);
  tomat(x->rli, P.RL);
  return P;
}

static void free_scan(Ctx* c) {
  (void)hipFree(c->bx);
  (void)hipFree(c->by);
  (void)hipFree(c->bz);
  (void)hipFree(c->nbr_idx);
  (void)hipFree(c->nbr_sqd);
  (void)hipFree(c->plane);
  (void)hipFree(c->sel);
  (void)hipFree(c->resid);
  (void)hipFree(c->chunk_part);
  c->bx = c->by = c->bz = nullptr;
  c->nbr_idx = nullptr;
  c->nbr_sqd = nullptr;
  c->plane = nullptr;
  c->sel = nullptr;
  c->resid = nullptr;
  c->chunk_part = nullptr;
}

}  // namespace slio

using namespace slio;

struct slio_ctx {
  Ctx c;
};

namespace slio {
void* internal_stream(slio_handle h) { return h ? (void*)h->c.stream : nullptr; }
}  // namespace slio

#define SLIO_CHECK_H(h)                                  \
  do {                                                   \
    if (!(h)) {                                          \
      set_error("null handle");                          \
      return SLIO_EINVAL;                                \
    }                                                    \
    SLIO_HIP(hipSetDevice((h)->c.prm.device));           \
  } while (0)

extern "C" {

const char* slio_last_error(void) { return g_err.c_str(); }

int slio_params_default(slio_params* p) {
  if (!p) return SLIO_EINVAL;
  std::memset(p, 0, sizeof(*p));
  p->device = 0;
  p->max_points = 100000;
  p->rank = 0;
  p->nranks = 1;
  p->grid_cell = 1.0f;
  p->plane_threshold = 0.1f;
  p->max_match_sqd = 5.0f;
  p->max_grid_cells = (int64_t)1 << 29;
  return SLIO_OK;
}

int slio_create(slio_handle* out, const slio_params* p) {
  if (!out || !p) {
    set_error("slio_create: null argument");
    return SLIO_EINVAL;
  }
  *out = nullptr;
  if (p->max_points <= 0 || p->nranks <= 0 || (SLIO_NSUPER % p->nranks) != 0 || p->rank < 0 ||
      p->rank >= p->nranks) {
    set_error("slio_create: bad max_points / rank / nranks");
    return SLIO_EINVAL;
  }
  int ndev = 0;
  SLIO_HIP(hipGetDeviceCount(&ndev));
  if (p->device < 0 || p->device >= ndev) {
    set_error("slio_create: no such HIP device");
    return SLIO_EDEVICE;
  }
  SLIO_HIP(hipSetDevice(p->device));
  int rc = init_constants();
  if (rc) return rc;
  auto* h = new slio_ctx();
  h->c.prm = *p;
  if (h->c.prm.grid_cell <= 0.0f) h->c.prm.grid_cell = 1.0f;
  if (h->c.prm.max_grid_cells <= 0) h->c.prm.max_grid_cells = (int64_t)1 << 29;
  if (hipStreamCreateWithFlags(&h->c.own_stream, hipStreamNonBlocking) != hipSuccess) {
    delete h;
    set_error("slio_create: hipStreamCreate failed");
    return SLIO_EDEVICE;
  }
  h->c.stream = h->c.own_stream;
  if (hipMalloc(&h->c.d_super_own, sizeof(double) * SLIO_NSUPER * SLIO_NPROD) != hipSuccess ||
      hipHostMalloc(&h->c.h_super, sizeof(double) * SLIO_NSUPER * SLIO_NPROD) != hipSuccess) {
    set_error("slio_create: allocation failed");
    slio_destroy(h);
    return SLIO_ENOMEM;
  }
  h->c.d_super = h->c.d_super_own;
  *out = h;
  return SLIO_OK;
}

int slio_destroy(slio_handle h) {
  if (!h) return SLIO_OK;
  (void)hipSetDevice(h->c.prm.device);
  if (h->c.stream) (void)hipStreamSynchronize(h->c.stream);
  free_scan(&h->c);
  prof_drain(h->c);
  for (auto& p : h->c.pool) {
    (void)hipEventDestroy(p.first);
    (void)hipEventDestroy(p.second);
  }
  (void)hipFree(h->c.d_super_own);
  (void)hipHostFree(h->c.h_super);
  h->c.map.reset();
  if (h->c.own_stream) (void)hipStreamDestroy(h->c.own_stream);
  delete h;
  return SLIO_OK;
}

int slio_set_stream(slio_handle h, void* s) {
  SLIO_CHECK_H(h);
  h->c.stream = s ? (hipStream_t)s : h->c.own_stream;
  return SLIO_OK;
}

int slio_map_upload(slio_handle h, const float* x, const float* y, const float* z, int64_t n) {
  SLIO_CHECK_H(h);
  if (n < 0 || (n > 0 && (!x || !y || !z)) || n >= (int64_t)0xFFFFFFFFll) {
    set_error("slio_map_upload: bad arguments");
    return SLIO_EINVAL;
  }
  auto m = std::make_shared<MapDev>();
  m->device = h->c.prm.device;
  m->n = n;
  hipStream_t st = h->c.stream;
  // bounding box on the host (the snapshot is host-resident anyway)
  float mn[3] = {0, 0, 0}, mx[3] = {0, 0, 0};
  const float* xyz[3] = {x, y, z};
  for (int a = 0; a < 3; ++a) {
    if (n == 0) break;
    float lo = xyz[a][0], hi = xyz[a][0];
    for (int64_t i = 0; i < n; ++i) {
      const float v = xyz[a][i];
      if (!std::isfinite(v)) {
        set_error("slio_map_upload: non-finite map coordinate");
        return SLIO_EINVAL;
      }
      lo = v < lo ? v : lo;
      hi = v > hi ? v : hi;
    }
    mn[a] = lo;
    mx[a] = hi;
  }
  GridGeom g;
  float hcell = h->c.prm.grid_cell;
  for (;;) {
    g.ox = mn[0];
    g.oy = mn[1];
    g.oz = mn[2];
    g.h = hcell;
    g.inv_h = 1.0f / hcell;
    g.dx = cell_coord(mx[0], g.ox, g.inv_h) + 1;
    g.dy = cell_coord(mx[1], g.oy, g.inv_h) + 1;
    g.dz = cell_coord(mx[2], g.oz, g.inv_h) + 1;
    const int64_t nc = (int64_t)g.dx * g.dy * g.dz;
    if (nc <= h->c.prm.max_grid_cells && nc < (int64_t)0xFFFFFFF0ll) break;
    hcell *= 1.25f;  // grow cells until the dense table fits the budget
  }
  float mag = 0.0f;
  for (int a = 0; a < 3; ++a) mag = std::max(mag, std::max(std::fabs(mn[a]), std::fabs(mx[a])));
  mag = std::max(mag, (float)std::max(g.dx, std::max(g.dy, g.dz)) * g.h);
  g.tol = mag * 3.814697265625e-06f + 1.0e-5f;  // 2^-18 relative: >= 64 ulps
  m->g = g;
  m->ncells = (int64_t)g.dx * g.dy * g.dz;

  SLIO_HIP(hipMalloc(&m->start, sizeof(uint32_t) * (m->ncells + 1)));
  if (n > 0) SLIO_HIP(hipMalloc(&m->pts, sizeof(float4) * n));
  if (n == 0) {
    SLIO_HIP(hipMemsetAsync(m->start, 0, sizeof(uint32_t) * (m->ncells + 1), st));
    SLIO_HIP(hipStreamSynchronize(st));
    h->c.map = m;
    return SLIO_OK;
  }
  float *dx_ = nullptr, *dy_ = nullptr, *dz_ = nullptr;
  uint32_t *k0 = nullptr, *k1 = nullptr, *v0 = nullptr, *v1 = nullptr, *cnt = nullptr;
  void* tmp = nullptr;
  int rc = SLIO_OK;
  auto fail = [&](const char* what, hipError_t e) {
    set_error(std::string("slio_map_upload: ") + what + ": " + hipGetErrorString(e));
    rc = SLIO_EDEVICE;
  };
  do {
    hipError_t e;
    if ((e = hipMalloc(&dx_, 4 * n)) || (e = hipMalloc(&dy_, 4 * n)) || (e = hipMalloc(&dz_, 4 * n)) ||
        (e = hipMalloc(&k0, 4 * n)) || (e = hipMalloc(&k1, 4 * n)) || (e = hipMalloc(&v0, 4 * n)) ||
        (e = hipMalloc(&v1, 4 * n)) || (e = hipMalloc(&cnt, 4 * (m->ncells + 1)))) {
      fail("hipMalloc", e);
      rc = SLIO_ENOMEM;
      break;
    }
    if ((e = hipMemcpyAsync(dx_, x, 4 * n, hipMemcpyHostToDevice, st)) ||
        (e = hipMemcpyAsync(dy_, y, 4 * n, hipMemcpyHostToDevice, st)) ||
        (e = hipMemcpyAsync(dz_, z, 4 * n, hipMemcpyHostToDevice, st))) {
      fail("H2D", e);
      break;
    }
    const int nb = (int)((n + 255) / 256);
    k_cell_keys<<<nb, 256, 0, st>>>(dx_, dy_, dz_, n, g, k0, v0);
    int end_bit = 1;
    while (end_bit < 32 && ((int64_t)1 << end_bit) < m->ncells) ++end_bit;
    size_t tb = 0;
    if ((e = hipcub::DeviceRadixSort::SortPairs(nullptr, tb, k0, k1, v0, v1, (int)n, 0, end_bit, st))) {
      fail("sort size", e);
      break;
    }
    size_t tb2 = 0;
    if ((e = hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, cnt, m->start, (int)(m->ncells + 1), st))) {
      fail("scan size", e);
      break;
    }
    tb = std::max(tb, tb2);
    if ((e = hipMalloc(&tmp, tb))) {
      fail("hipMalloc tmp", e);
      rc = SLIO_ENOMEM;
      break;
    }
    if ((e = hipcub::DeviceRadixSort::SortPairs(tmp, tb, k0, k1, v0, v1, (int)n, 0, end_bit, st))) {
      fail("sort", e);
      break;
    }
    if ((e = hipMemsetAsync(cnt, 0, 4 * (m->ncells + 1), st))) {
      fail("memset", e);
      break;
    }
    k_cell_hist<<<nb, 256, 0, st>>>(k1, n, cnt);
    if ((e = hipcub::DeviceScan::ExclusiveSum(tmp, tb, cnt, m->start, (int)(m->ncells + 1), st))) {
      fail("scan", e);
      break;
    }
    k_gather_sorted<<<nb, 256, 0, st>>>(dx_, dy_, dz_, v1, n, m->pts);
    if ((e = hipGetLastError()) || (e = hipStreamSynchronize(st))) {
      fail("build kernels", e);
      break;
    }
  } while (0);
  (void)hipFree(dx_);
  (void)hipFree(dy_);
  (void)hipFree(dz_);
  (void)hipFree(k0);
  (void)hipFree(k1);
  (void)hipFree(v0);
  (void)hipFree(v1);
  (void)hipFree(cnt);
  (void)hipFree(tmp);
  if (rc) return rc;
  h->c.map = m;
  h->c.searched = false;
  return SLIO_OK;
}

int slio_map_share(slio_handle h, slio_handle src) {
  SLIO_CHECK_H(h);
  if (!src || !src->c.map || src->c.prm.device != h->c.prm.device) {
    set_error("slio_map_share: source has no map on this device");
    return SLIO_EINVAL;
  }
  h->c.map = src->c.map;
  h->c.searched = false;
  return SLIO_OK;
}

int slio_map_info(slio_handle h, int32_t dims[3], float* cell, int64_t* n) {
  SLIO_CHECK_H(h);
  if (!h->c.map) {
    set_error("slio_map_info: no map");
    return SLIO_ESTATE;
  }
  if (dims) {
    dims[0] = h->c.map->g.dx;
    dims[1] = h->c.map->g.dy;
    dims[2] = h->c.map->g.dz;
  }
  if (cell) *cell = h->c.map->g.h;
  if (n) *n = h->c.map->n;
  return SLIO_OK;
}

int slio_scan_upload(slio_handle h, const float* x, const float* y, const float* z, int64_t n) {
  SLIO_CHECK_H(h);
  Ctx& c = h->c;
  if (n < 0 || (n > 0 && (!x || !y || !z))) {
    set_error("slio_scan_upload: bad arguments");
    return SLIO_EINVAL;
  }
  if (n > c.prm.max_points) {
    set_error("slio_scan_upload: scan exceeds max_points");
    return SLIO_ECAPACITY;
  }
  if (!c.bx) {
    const int64_t cap = c.prm.max_points;
    const int64_t capc = num_chunks(cap) + 1;
    hipError_t e;
    if ((e = hipMalloc(&c.bx, 4 * cap)) || (e = hipMalloc(&c.by, 4 * cap)) ||
        (e = hipMalloc(&c.bz, 4 * cap)) || (e = hipMalloc(&c.nbr_idx, 4 * 5 * cap)) ||
        (e = hipMalloc(&c.nbr_sqd, 4 * 5 * cap)) || (e = hipMalloc(&c.plane, 16 * cap)) ||
        (e = hipMalloc(&c.sel, cap)) || (e = hipMalloc(&c.resid, 4 * cap)) ||
        (e = hipMalloc(&c.chunk_part, 8 * SLIO_NPROD * capc))) {
      free_scan(&c);
      set_error(std::string("slio_scan_upload: hipMalloc: ") + hipGetErrorString(e));
      return SLIO_ENOMEM;
    }
  }
  c.n = n;
  if (n > 0) {
    SLIO_HIP(hipMemcpyAsync(c.bx, x, 4 * n, hipMemcpyHostToDevice, c.stream));
    SLIO_HIP(hipMemcpyAsync(c.by, y, 4 * n, hipMemcpyHostToDevice, c.stream));
    SLIO_HIP(hipMemcpyAsync(c.bz, z, 4 * n, hipMemcpyHostToDevice, c.stream));
    SLIO_HIP(hipMemsetAsync(c.sel, 0, n, c.stream));
  }
  c.searched = false;
  return SLIO_OK;
}

int slio_shard_range(slio_handle h, int64_t* begin, int64_t* end) {
  SLIO_CHECK_H(h);
  int64_t c0, c1;
  rank_chunks(h->c.n, h->c.prm.rank, h->c.prm.nranks, &c0, &c1);
  if (begin) *begin = std::min(c0 * SLIO_CHUNK, h->c.n);
  if (end) *end = std::min(c1 * SLIO_CHUNK, h->c.n);
  return SLIO_OK;
}

int slio_iterate_async(slio_handle h, const slio_pose* x, int do_search, int extrinsic_est,
                       double** d_super) {
  SLIO_CHECK_H(h);
  Ctx& c = h->c;
  if (!x) {
    set_error("slio_iterate_async: null pose");
    return SLIO_EINVAL;
  }
  if (!c.map) {
    set_error("slio_iterate_async: no map uploaded");
    return SLIO_ESTATE;
  }
  if (!c.bx && c.n > 0) {
    set_error("slio_iterate_async: no scan uploaded");
    return SLIO_ESTATE;
  }
  if (!do_search && !c.searched) {
    set_error("slio_iterate_async: reuse pass before any search pass");
    return SLIO_ESTATE;
  }
  const int64_t C = num_chunks(c.n);
  int64_t c0, c1;
  rank_chunks(c.n, c.prm.rank, c.prm.nranks, &c0, &c1);
  PassCfg cfg;
  cfg.plane_thr = c.prm.plane_threshold;
  cfg.max_sqd = c.prm.max_match_sqd;
  cfg.extrinsic = extrinsic_est ? 1 : 0;
  cfg.c_begin = c0;
  cfg.c_end = c1;
  PassOut o{c.nbr_idx, c.nbr_sqd, c.plane, c.sel, c.resid, c.chunk_part};
  ScanDev s{c.bx, c.by, c.bz, c.n};
  const PoseDev P = make_pose(x);
  const int64_t nblk = c1 - c0;
  if (c.prof && (c.pending[0].size() + c.pending[1].size()) > 256) prof_drain(c);
  if (nblk > 0) {
    const int kind = do_search ? SLIO_KERNEL_SEARCH : SLIO_KERNEL_REUSE;
    std::pair<hipEvent_t, hipEvent_t> ev{nullptr, nullptr};
    if (c.prof) {
      ev = prof_pair(c);
      (void)hipEventRecord(ev.first, c.stream);
    }
    if (do_search) {
      const MapView mv{c.map->g, c.map->n, c.map->pts, c.map->start};
      k_search_pass<<<(unsigned)nblk, kBlock, 0, c.stream>>>(mv, s, P, cfg, o);
    } else {
      k_reuse_pass<<<(unsigned)nblk, SLIO_CHUNK, 0, c.stream>>>(s, P, cfg, o);
    }
    if (c.prof) {
      (void)hipEventRecord(ev.second, c.stream);
      c.pending[kind].push_back(ev);
    }
  }
  const int per = SLIO_NSUPER / c.prm.nranks;
  std::pair<hipEvent_t, hipEvent_t> ev2{nullptr, nullptr};
  if (c.prof) {
    ev2 = prof_pair(c);
    (void)hipEventRecord(ev2.first, c.stream);
  }
  k_super_sums<<<SLIO_NSUPER, 128, 0, c.stream>>>(c.chunk_part, C, c.prm.rank * per,
                                                   (c.prm.rank + 1) * per, c.d_super);
  if (c.prof) {
    (void)hipEventRecord(ev2.second, c.stream);
    c.pending[SLIO_KERNEL_SUPER].push_back(ev2);
  }
  SLIO_HIP(hipGetLastError());
  if (do_search) c.searched = true;
  if (d_super) *d_super = c.d_super;
  return SLIO_OK;
}

int slio_set_super_buffer(slio_handle h, double* dev_buf) {
  SLIO_CHECK_H(h);
  h->c.d_super = dev_buf ? dev_buf : h->c.d_super_own;
  return SLIO_OK;
}

int slio_profile(slio_handle h, int enable) {
  SLIO_CHECK_H(h);
  Ctx& c = h->c;
  prof_drain(c);
  c.prof = enable != 0;
  for (int k = 0; k < 3; ++k) {
    c.prof_ms[k] = 0.0;
    c.prof_n[k] = 0;
  }
  return SLIO_OK;
}

int slio_profile_read(slio_handle h, int kind, double* ms, int64_t* launches) {
  SLIO_CHECK_H(h);
  if (kind < 0 || kind > 2) {
    set_error("slio_profile_read: bad kind");
    return SLIO_EINVAL;
  }
  Ctx& c = h->c;
  SLIO_HIP(hipStreamSynchronize(c.stream));
  prof_drain(c);
  if (ms) *ms = c.prof_ms[kind];
  if (launches) *launches = c.prof_n[kind];
  return SLIO_OK;
}

int slio_super_download(slio_handle h, double* super_out) {
  SLIO_CHECK_H(h);
  Ctx& c = h->c;
  SLIO_HIP(hipMemcpyAsync(c.h_super, c.d_super, sizeof(double) * SLIO_NSUPER * SLIO_NPROD,
                          hipMemcpyDeviceToHost, c.stream));
  SLIO_HIP(hipStreamSynchronize(c.stream));
  if (super_out) std::memcpy(super_out, c.h_super, sizeof(double) * SLIO_NSUPER * SLIO_NPROD);
  return SLIO_OK;
}

int slio_reduce_super(const double* sup, double* HTH, double* HTh, int64_t* m) {
  if (!sup) return SLIO_EINVAL;
  double tot[SLIO_NPROD];
  for (int k = 0; k < SLIO_NPROD; ++k) {
    double a = sup[k];
    for (int s = 1; s < SLIO_NSUPER; ++s) a = a + sup[s * SLIO_NPROD + k];
    tot[k] = a;
  }
  if (HTH) std::memcpy(HTH, tot, sizeof(double) * SLIO_NHTH);
  if (HTh) std::memcpy(HTh, tot + SLIO_NHTH, sizeof(double) * 12);
  if (m) *m = (int64_t)llround(tot[90]);
  return SLIO_OK;
}

int slio_iterate(slio_handle h, const slio_pose* x, int do_search, int extrinsic_est,
                 double* HTH, double* HTh, int64_t* m) {
  int rc = slio_iterate_async(h, x, do_search, extrinsic_est, nullptr);
  if (rc) return rc;
  double sup[SLIO_NSUPER * SLIO_NPROD];
  rc = slio_super_download(h, sup);
  if (rc) return rc;
  return slio_reduce_super(sup, HTH, HTh, m);
}

int slio_get_neighbors(slio_handle h, int32_t* idx, float* sqd, uint8_t* sel) {
  SLIO_CHECK_H(h);
  Ctx& c = h->c;
  int64_t b, e;
  slio_shard_range(h, &b, &e);
  const int64_t n = e - b;
  SLIO_HIP(hipStreamSynchronize(c.stream));
  if (n <= 0) return SLIO_OK;
  if (idx) SLIO_HIP(hipMemcpy(idx, c.nbr_idx + b * 5, 4 * 5 * n, hipMemcpyDeviceToHost));
  if (sqd) SLIO_HIP(hipMemcpy(sqd, c.nbr_sqd + b * 5, 4 * 5 * n, hipMemcpyDeviceToHost));
  if (sel) SLIO_HIP(hipMemcpy(sel, c.sel + b, n, hipMemcpyDeviceToHost));
  return SLIO_OK;
}

int slio_get_planes(slio_handle h, float* abcd) {
  SLIO_CHECK_H(h);
  Ctx& c = h->c;
  int64_t b, e;
  slio_shard_range(h, &b, &e);
  const int64_t n = e - b;
  SLIO_HIP(hipStreamSynchronize(c.stream));
  if (n <= 0 || !abcd) return SLIO_OK;
  SLIO_HIP(hipMemcpy(abcd, c.plane + b, 16 * n, hipMemcpyDeviceToHost));
  return SLIO_OK;
}

int slio_get_residuals(slio_handle h, float* pd2) {
  SLIO_CHECK_H(h);
  Ctx& c = h->c;
  int64_t b, e;
  slio_shard_range(h, &b, &e);
  const int64_t n = e - b;
  SLIO_HIP(hipStreamSynchronize(c.stream));
  if (n <= 0 || !pd2) return SLIO_OK;
  SLIO_HIP(hipMemcpy(pd2, c.resid + b, 4 * n, hipMemcpyDeviceToHost));
  return SLIO_OK;
}

}  // extern "C"
