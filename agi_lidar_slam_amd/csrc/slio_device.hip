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
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rccl/rccl.h>

#include <algorithm>
#include <type_traits>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstddef>
#include <cstring>
#include <type_traits>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <vector>

#include "slio_common.hpp"
#include "slio_plane.hpp"
#include "slio_so3.hpp"

// -DSLIO_SOLVE_STAMP: wall-clock stamps of the filter-step phases (diagnostic
// builds only; read with slio_dbg_solve_stamps).
#ifdef SLIO_SOLVE_STAMP
__device__ unsigned long long g_sstamp[64];
#define SSTAMP(k)                                       \
  do {                                                  \
    __builtin_amdgcn_sched_barrier(0);                  \
    if (threadIdx.x == 0) g_sstamp[k] = wall_clock64(); \
    __builtin_amdgcn_sched_barrier(0);                  \
  } while (0)
#else
#define SSTAMP(k) \
  do {            \
  } while (0)
#endif

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

constexpr int kBlock = 256;                      // threads per search workgroup
constexpr int kDefaultLPQ = 2;                   // lanes per query (tuned on MI355X)
#ifndef SLIO_SEARCH_U
#define SLIO_SEARCH_U 3                          // candidate loads in flight per lane and step (A/B on MI355X, block rows: 3 < 4 < 2)
#endif
constexpr uint64_t kInfKey = ~0ull;

#ifdef SLIO_ABL_STAMP
// diagnostic build only: per-block phase timestamps (s_memrealtime, 100 MHz)
__device__ unsigned long long g_stamps[8192][8];
__device__ uint32_t g_hwid[8192][2];  // HW_ID (cu, simd, se) and XCC_ID of wave 0
__device__ unsigned long long g_wstamps[8192][4][4];  // per wave: refine start/end, fallback end, rounds
#define WSTAMP(k, v)                                                               \
  do {                                                                             \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 8192)                              \
      g_wstamps[blockIdx.x][threadIdx.x >> 6][k] = (v);                            \
  } while (0)
__device__ unsigned long long g_rstamps[8192][6];  // thread 0's last wide refinement
#define RSTAMP(k)                                                                  \
  do {                                                                             \
    if (threadIdx.x == 0 && blockIdx.x < 8192)                                     \
      g_rstamps[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime();                 \
  } while (0)
// ... and its candidates, runs, lanes and whether its bound was finite
#define RINFO(T, nr, RL, fin)                                                      \
  do {                                                                             \
    if (threadIdx.x == 0 && blockIdx.x < 8192) {                                   \
      g_rstamps[blockIdx.x][4] = (T);                                              \
      g_rstamps[blockIdx.x][5] = (nr) | ((RL) << 8) | ((fin) ? 0x10000 : 0);       \
    }                                                                              \
  } while (0)
// fit phase of thread 0 (wave 0): entry, loads landed, plane + gate, row formed, end
__device__ unsigned long long g_fstamps[8192][6];
#define FSTAMP(k, wait)                                                            \
  do {                                                                             \
    __builtin_amdgcn_sched_barrier(0);                                             \
    if (wait) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                     \
    if (threadIdx.x == 0 && blockIdx.x < 8192)                                     \
      g_fstamps[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime();                 \
    __builtin_amdgcn_sched_barrier(0);                                             \
  } while (0)
#define STAMP(slot)                                                                \
  do {                                                                             \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 8192) {                            \
      g_stamps[blockIdx.x][slot] = __builtin_amdgcn_s_memrealtime();               \
      if ((slot) == 0 && threadIdx.x == 0) {                                       \
        g_hwid[blockIdx.x][0] = __builtin_amdgcn_s_getreg((31 << 11) | 4);         \
        g_hwid[blockIdx.x][1] = __builtin_amdgcn_s_getreg((31 << 11) | 20);        \
      }                                                                            \
    }                                                                              \
  } while (0)
#else
#define STAMP(slot) \
  do {              \
  } while (0)
#define WSTAMP(k, v) \
  do {               \
  } while (0)
#define RSTAMP(k) \
  do {            \
  } while (0)
#define RINFO(T, nr, RL, fin) \
  do {                        \
  } while (0)
#define FSTAMP(k, wait) \
  do {                  \
  } while (0)
#endif

__constant__ uint8_t c_pa[SLIO_NPROD];
__constant__ uint8_t c_pb[SLIO_NPROD];

// ---------------------------------------------------------------- map index
struct GridGeom {
  float ox, oy, oz;   // origin = bbox min
  float h, inv_h;     // cell edge and its reciprocal
  float tol;          // conservative slack on cell-boundary coordinates
  int dx, dy, dz;     // dims
};

// Coarse level for the queries the fine grid cannot finish cheaply (5th
// neighbour beyond the 5x5x5 fine cube, query cells outside the grid): cells
// of edge 4h on the fine grid's origin -- coarse cell (cx, cy, cz) is the fine
// cells [4cx, 4cx + 4) x [4cy, 4cy + 4) x [4cz, 4cz + 4), so its points are 16
// runs of the fine cell-sorted pts (one per fine (y, z) row) -- and a bounding
// box of every coarse cell's points: exact pruning, since a float distance to
// a point is never below the float distance to a box that contains it, both
// rounded monotonically.  An upload or a sorting rebuild makes the boxes
// tight; a merge rebuild (the live map) only widens them by its additions
// (k_coarse_extend): a deleted point leaves a box merely conservative.  No
// coarse copy of the points, so a merge rebuild does not rewrite one.
struct CoarseView {
  GridGeom g;               // h = 4 x the fine cell edge
  const float4* lo;         // per coarse cell: min x, y, z, bits(points ever counted: 0 = empty)
  const float4* hi;         // per coarse cell: max x, y, z
};

struct Ctx;

struct MapDev {
  GridGeom g;
  int64_t n = 0;
  int64_t ncells = 0;
  float4* pts = nullptr;          // sorted by cell: x, y, z, bits(map index)
  uint32_t* start = nullptr;      // ncells + 1 prefix offsets
  // coarse level (CoarseView)
  GridGeom cg;
  int64_t nccells = 0;
  float4* clo = nullptr;
  float4* chi = nullptr;
  // block rows (optional, ~9x the points): entry (x, y, z) holds the points
  // of the 9 cells (x, y + j, z + k), j, k in {-1, 0, 1}, with .w = their
  // position in pts; entries are laid out in cell order, so the 3x3x3 block
  // around a cell is ONE contiguous range [bstart[c - 1], bstart[c + 2])
  float4* blk = nullptr;
  uint32_t* bstart = nullptr;     // ncells + 1 prefix offsets into blk
  int64_t nblk = 0;
  int device = 0;
  // map maintenance (slio_map_add_points / slio_map_delete_boxes /
  // slio_map_incremental): deletions are flags on pts positions, additions
  // wait in add4 (id order) until the next rebuild of the index (map_refresh,
  // before the next search pass or download).  Point ids: 0..n-1 for the
  // upload, then the next ids for every surviving added point.
  uint8_t* keep = nullptr;        // n: 0 = deleted since the last build
  float4* add4 = nullptr;         // x, y, z, bits(id)
  uint8_t* akeep = nullptr;
  int64_t nadd = 0, add_cap = 0;
  uint32_t next_id = 0;
  // stored points deleted since the coarse boxes were last made tight (merge
  // rebuilds only widen them): past n / kCoarseRetighten they are rebuilt
  int64_t del_loose = 0;
  std::atomic<uint64_t> version{1};  // bumped by every rebuild (positions change)
  std::atomic<bool> dirty{false};
  // block rows of a rebuilt map are built once it has been searched
  // kBlkAfterPasses times unchanged (a map changed every scan goes without:
  // they cost ~1 ms per rebuild and save ~5 us per search pass)
  std::atomic<bool> blk_deferred{false};
  int stable_passes = 0;
  // Sharing (slio_map_share).  Changes -- edits, rebuilds, block rows --
  // hold mu exclusively; passes and reads hold it shared from reading the
  // views through their launches.  Streams: a change first orders its stream
  // after everything the other users have enqueued (they may still be
  // reading what it overwrites: map_write_begin), then records `ready` and
  // bumps `epoch`; a reader whose stream has not yet waited for the current
  // epoch waits for `ready` (map_read_sync).
  std::shared_mutex mu;
  std::vector<Ctx*> users;  // handles holding this map
  hipEvent_t ready = nullptr;
  uint64_t epoch = 0;
  bool broken = false;  // an index rebuild failed part-way: unusable until a new upload
  int64_t sequential_calls = 0;  // Add_Points calls that took k_ds_sequential (diagnostic)
  float cell0 = 1.0f;             // requested grid cell and cell budget (slio_params)
  int64_t max_cells = 0;
  // device allocations kept across index rebuilds (capacity in bytes): a
  // rebuild per scan must not pay hipMalloc / hipFree of ~GB tables
  struct Buf {
    void* p = nullptr;
    size_t cap = 0;
  };
  Buf b_pts, b_keep, b_start, b_clo, b_chi, b_bstart, b_blk, b_tmp[8], b_ref[6], b_add[8], b_start2, b_keep2;
  static hipError_t take(Buf& b, size_t bytes) {
    bytes = std::max<size_t>(bytes, 16);
    if (bytes <= b.cap) return hipSuccess;
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.cap = 0;
    size_t want = bytes + bytes / 4;  // headroom: the map grows scan by scan
    hipError_t e = hipMalloc(&b.p, want);
    if (e) {
      (void)hipGetLastError();
      want = bytes;
      e = hipMalloc(&b.p, want);
    }
    if (!e) b.cap = want;
    return e;
  }
  void free_index() {  // the views only; allocations stay for the next build
    pts = nullptr;
    start = nullptr;
    blk = nullptr;
    bstart = nullptr;
    clo = nullptr;
    chi = nullptr;
    keep = nullptr;
    n = ncells = nccells = nblk = 0;
  }
  ~MapDev() {
    if (ready) (void)hipEventDestroy(ready);
    for (Buf* b : {&b_pts, &b_keep, &b_start, &b_clo, &b_chi, &b_bstart, &b_blk, &b_start2, &b_keep2})
      if (b->p) (void)hipFree(b->p);
    for (Buf& b : b_tmp)
      if (b.p) (void)hipFree(b.p);
    for (Buf& b : b_ref)
      if (b.p) (void)hipFree(b.p);
    for (Buf& b : b_add)
      if (b.p) (void)hipFree(b.p);
    if (add4) (void)hipFree(add4);
    if (akeep) (void)hipFree(akeep);
  }
};

// trivially-copyable kernel argument view of a MapDev
struct MapView {
  GridGeom g;
  int64_t n;
  const float4* pts;
  const uint32_t* start;
  const float4* blk;       // null: the 3x3x3 block is scanned as 9 runs of pts
  const uint32_t* bstart;
  int64_t nblk;
  int64_t ncells;
  CoarseView cl;
};

#ifdef SLIO_BOUNDS_CHECK
__constant__ int64_t c_dbg_npts, c_dbg_ncells;  // set by slio_map_upload
// diagnostic build only: report and neutralise an out-of-range index
#define SLIO_BCHK(idx, lim, what)                                                       \
  do {                                                                                  \
    if ((int64_t)(idx) < 0 || (int64_t)(idx) >= (int64_t)(lim)) {                       \
      printf("slio bounds: %s idx %lld lim %lld block %d thread %d\n", what,             \
             (long long)(idx), (long long)(lim), (int)blockIdx.x, (int)threadIdx.x);     \
      idx = 0;                                                                          \
    }                                                                                   \
  } while (0)
#else
#define SLIO_BCHK(idx, lim, what) \
  do {                            \
  } while (0)
#endif

__device__ __host__ __forceinline__ int cell_coord(float p, float o, float inv_h) {
  float t = floorf((p - o) * inv_h);
  t = fminf(fmaxf(t, -1.0e8f), 1.0e8f);
  return (int)t;
}

// per-cell counts of SORTED keys (cell = key >> shift): one atomic per run of
// equal cells inside a wavefront (sorted keys put up to 64 lanes on one
// counter; per-lane atomics serialised there: 0.64 ms for the coarse level
// of a 10M map)
template <typename K>
__global__ void k_cell_hist_sorted(const K* __restrict__ keys, int64_t n, int shift,
                                   uint32_t* __restrict__ counts) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = i < n;
  const uint32_t c = live ? (uint32_t)(keys[i] >> shift) : 0xFFFFFFFFu;
  const int lane = threadIdx.x & 63;
  const uint32_t prev = __shfl_up(c, 1, 64);
  const bool head = live && (lane == 0 || prev != c);
  const uint64_t heads = __ballot(head);
  const uint64_t livem = __ballot(live);
  if (head) {
    const uint64_t above = lane == 63 ? 0ull : heads & ~((2ull << lane) - 1ull);
    const int end = above ? __ffsll((long long)above) - 1 : 64 - __clzll((long long)livem);
    atomicAdd(&counts[c], (uint32_t)(end - lane));
  }
}

// block rows: entry sizes, then the fill, one thread per cell.  A source
// row (y + j, z + k) whose start[] is equal at both ends of a segment of
// kBlkSeg x cells is empty there: k_blk_live marks the live rows per segment
// (2 loads a row), and the cell threads read only those (95 % of a 10M
// street map's 33M cells are empty; every cell thread used to spend 18 loads).
// Sources in (z, y) order, each cell's points in pts order.
constexpr int kBlkSeg = 16;
constexpr int kBlkAfterPasses = 8;
__device__ __forceinline__ uint32_t blk_rows_live(const uint32_t* __restrict__ start, GridGeom g, int x0,
                                                  int x1, int y, int z) {
  uint32_t live = 0;
  for (int k = -1; k <= 1; ++k)
    for (int j = -1; j <= 1; ++j) {
      const int yy = y + j, zz = z + k;
      const int q = (k + 1) * 3 + (j + 1);
      if (yy < 0 || yy >= g.dy || zz < 0 || zz >= g.dz) continue;
      const int64_t rb = ((int64_t)zz * g.dy + yy) * g.dx;
      if (start[rb + x1] != start[rb + x0]) live |= 1u << q;
    }
  return live;
}

// live source rows of every segment (9 bits)
__global__ void k_blk_live(const uint32_t* __restrict__ start, GridGeom g, int64_t nseg,
                           uint16_t* __restrict__ live) {
  const int64_t sg = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (sg >= nseg) return;
  const int segs = (g.dx + kBlkSeg - 1) / kBlkSeg;
  const int x0 = (int)(sg % segs) * kBlkSeg, x1 = min(x0 + kBlkSeg, g.dx);
  const int y = (int)((sg / segs) % g.dy);
  const int z = (int)(sg / ((int64_t)segs * g.dy));
  live[sg] = (uint16_t)blk_rows_live(start, g, x0, x1, y, z);
}

// one thread per cell; only the segment's live source rows are read
__global__ void k_blk_count(const uint32_t* __restrict__ start, const uint16_t* __restrict__ live,
                            GridGeom g, int64_t ncells, uint32_t* __restrict__ cnt9) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ncells) return;
  const int x = (int)(c % g.dx);
  const int64_t row = c / g.dx;
  const int segs = (g.dx + kBlkSeg - 1) / kBlkSeg;
  uint32_t m = live[row * segs + x / kBlkSeg];
  uint32_t s = 0;
  const int y = (int)(row % g.dy), z = (int)(row / g.dy);
  for (; m; m &= m - 1) {
    const int q = __ffs(m) - 1;
    const int64_t sc = ((int64_t)(z + q / 3 - 1) * g.dy + (y + q % 3 - 1)) * g.dx + x;
    s += start[sc + 1] - start[sc];
  }
  cnt9[c] = s;
}

__global__ void k_blk_fill(const float4* __restrict__ pts, const uint32_t* __restrict__ start,
                           const uint16_t* __restrict__ live, const uint32_t* __restrict__ bstart,
                           GridGeom g, int64_t ncells, float4* __restrict__ blk) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ncells) return;
  const int x = (int)(c % g.dx);
  const int64_t row = c / g.dx;
  const int segs = (g.dx + kBlkSeg - 1) / kBlkSeg;
  uint32_t m = live[row * segs + x / kBlkSeg];
  if (!m) return;
  const int y = (int)(row % g.dy), z = (int)(row / g.dy);
  uint32_t o = bstart[c];
  for (; m; m &= m - 1) {
    const int q = __ffs(m) - 1;
    const int64_t sc = ((int64_t)(z + q / 3 - 1) * g.dy + (y + q % 3 - 1)) * g.dx + x;
    for (uint32_t p = start[sc]; p < start[sc + 1]; ++p) {
      const float4 v = pts[p];
      blk[o++] = make_float4(v.x, v.y, v.z, __uint_as_float(p));
    }
  }
}

// coarse level: cell keys of the fine-sorted points, then the gather (values
// are fine positions, ascending inside a coarse cell after the stable sort)
__global__ void k_coarse_keys(const float4* __restrict__ pts, int64_t n, GridGeom cg,
                              uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 p = pts[i];
  int cx = min(max(cell_coord(p.x, cg.ox, cg.inv_h), 0), cg.dx - 1);
  int cy = min(max(cell_coord(p.y, cg.oy, cg.inv_h), 0), cg.dy - 1);
  int cz = min(max(cell_coord(p.z, cg.oz, cg.inv_h), 0), cg.dz - 1);
  keys[i] = ((uint32_t)cz * (uint32_t)cg.dy + (uint32_t)cy) * (uint32_t)cg.dx + (uint32_t)cx;
  vals[i] = (uint32_t)i;
}

// Coarse level without a sort.  A coarse cell (edge 4h, same origin) is the
// 4x4x4 fine cells [4c, 4c + 4) per axis, clipped to the fine grid, so its
// points are the fine runs of its 16 (y, z) rows -- each a contiguous x-range
// of cells of the cell-sorted pts -- and taking the rows in order lists them in
// fine position order, the order a stable sort by coarse cell gave.  (A point
// lies within tol of its fine cell, hence of that cell's coarse cell; the far
// search's bounds carry the same tol.)
__device__ __forceinline__ void coarse_decode(const GridGeom& cg, int64_t c, int& x, int& y, int& z) {
  x = (int)(c % cg.dx);
  const int64_t t = c / cg.dx;
  y = (int)(t % cg.dy);
  z = (int)(t / cg.dy);
}
__global__ void k_coarse_count(const uint32_t* __restrict__ start, GridGeom g, GridGeom cg, int64_t nc,
                               uint32_t* __restrict__ cnt) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c == 0) cnt[nc] = 0;
  if (c >= nc) return;
  int cx, cy, cz;
  coarse_decode(cg, c, cx, cy, cz);
  const int x0 = 4 * cx, x1 = min(4 * cx + 4, g.dx);
  uint32_t sum = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int fy = 4 * cy + (k & 3), fz = 4 * cz + (k >> 2);
    if (fy < g.dy && fz < g.dz) {
      const int64_t rb = ((int64_t)fz * g.dy + fy) * g.dx;
      sum += start[rb + x1] - start[rb + x0];
    }
  }
  cnt[c] = sum;
}
// one wavefront per 64 coarse cells: each lane reads its cell's size
// (k_coarse_count; empty cells -- most of a surface map's -- are written by
// their lane at once), then 16-lane groups read the non-empty cells' rows,
// four cells at a time, and form their tight boxes (count in lo.w).
__global__ void k_coarse_boxes(const float4* __restrict__ pts, const uint32_t* __restrict__ start, GridGeom g,
                               GridGeom cg, const uint32_t* __restrict__ cnt, int64_t nc,
                               float4* __restrict__ lo, float4* __restrict__ hi) {
  const int64_t c_base = (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) << 6;
  const int lane = threadIdx.x & 63;
  const float INF = __int_as_float(0x7f800000);
  const int64_t mc = c_base + lane;
  uint32_t mt = 0;
  if (mc < nc) {
    mt = cnt[mc];
    if (mt == 0) {
      lo[mc] = make_float4(INF, INF, INF, __uint_as_float(0u));
      hi[mc] = make_float4(-INF, -INF, -INF, 0.0f);
    }
  }
  // the non-empty cells, four at a time: 16 lanes per cell (lane r of a
  // group fetches row r's bounds), most cells hold a few dozen points
  const uint64_t busy = __ballot(mc < nc && mt != 0);
  const int nbusy = __popcll(busy);
  const int gi = lane >> 4, sl = lane & 15;
  for (int k0 = 0; k0 < nbusy; k0 += 4) {
    const int kk = k0 + gi;
    const bool act = kk < nbusy;
    uint64_t bm = busy;
    for (int q = 0; q < kk && bm; ++q) bm &= bm - 1;  // the kk-th set bit
    const int l = (act && bm) ? __ffsll((unsigned long long)bm) - 1 : 0;
    const int64_t c = c_base + l;
    // (every lane shuffles: a cross-lane read inside a condition would read
    // lanes the condition turned off)
    const uint32_t tsrc = __shfl(mt, l, 64);
    const uint32_t total = act ? tsrc : 0u;
    int cx, cy, cz;
    coarse_decode(cg, c, cx, cy, cz);
    const int x0 = 4 * cx, x1 = min(4 * cx + 4, g.dx);
    uint32_t rs = 0, len = 0;
    {
      const int fy = 4 * cy + (sl & 3), fz = 4 * cz + (sl >> 2);
      if (act && fy < g.dy && fz < g.dz) {
        const int64_t rb = ((int64_t)fz * g.dy + fy) * g.dx;
        rs = start[rb + x0];
        len = start[rb + x1] - rs;
      }
    }
    uint32_t inc = len;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const uint32_t v = __shfl_up(inc, o, 16);
      if (sl >= o) inc += v;
    }
    const uint32_t excl = inc - len;
    float l3[3] = {INF, INF, INF}, u3[3] = {-INF, -INF, -INF};
    // the cell's points as one flat list over its rows: lane j of the group
    // takes list entries j, j + 16, ... (row r = the last row starting at or
    // before the entry)
    uint32_t E[16], S[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      E[r] = __shfl(excl, r, 16);
      S[r] = __shfl(rs, r, 16) - E[r];  // list entry j of row r is pts[S[r] + j]
    }
    for (uint32_t j = sl; j < total; j += 16) {
      uint32_t src = S[0] + j;
#pragma unroll
      for (int r = 1; r < 16; ++r) src = (j >= E[r]) ? S[r] + j : src;
      const float4 v = pts[src];
      l3[0] = fminf(l3[0], v.x);
      l3[1] = fminf(l3[1], v.y);
      l3[2] = fminf(l3[2], v.z);
      u3[0] = fmaxf(u3[0], v.x);
      u3[1] = fmaxf(u3[1], v.y);
      u3[2] = fmaxf(u3[2], v.z);
    }
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int o = 8; o >= 1; o >>= 1) {
        l3[a] = fminf(l3[a], __shfl_xor(l3[a], o, 16));
        u3[a] = fmaxf(u3[a], __shfl_xor(u3[a], o, 16));
      }
    if (sl == 0 && act) {
      lo[c] = make_float4(l3[0], l3[1], l3[2], __uint_as_float(total));
      hi[c] = make_float4(u3[0], u3[1], u3[2], 0.0f);
    }
  }
}

// float min / max by compare-and-swap (vector atomics): the coarse boxes of
// a merge rebuild's additions
__device__ __forceinline__ void atomic_fmin(float* a, float v) {
  int* ai = reinterpret_cast<int*>(a);
  int old = __hip_atomic_load(ai, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  while (v < __int_as_float(old)) {
    const int prev = atomicCAS(ai, old, __float_as_int(v));
    if (prev == old) break;
    old = prev;
  }
}
__device__ __forceinline__ void atomic_fmax(float* a, float v) {
  int* ai = reinterpret_cast<int*>(a);
  int old = __hip_atomic_load(ai, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  while (v > __int_as_float(old)) {
    const int prev = atomicCAS(ai, old, __float_as_int(v));
    if (prev == old) break;
    old = prev;
  }
}
// widen the boxes (and counts) of the coarse cells the na additions fall in;
// a point's coarse cell is its (clamped) fine cell / 4 on every axis
__global__ void k_coarse_extend(const float4* __restrict__ adds, const uint8_t* __restrict__ keep, int64_t na,
                                GridGeom g, float4* __restrict__ lo, float4* __restrict__ hi, GridGeom cg) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= na || (keep && !keep[i])) return;
  const float4 v = adds[i];
  const int fx = min(max(cell_coord(v.x, g.ox, g.inv_h), 0), g.dx - 1);
  const int fy = min(max(cell_coord(v.y, g.oy, g.inv_h), 0), g.dy - 1);
  const int fz = min(max(cell_coord(v.z, g.oz, g.inv_h), 0), g.dz - 1);
  const int64_t c = ((int64_t)(fz >> 2) * cg.dy + (fy >> 2)) * cg.dx + (fx >> 2);
  float* l = reinterpret_cast<float*>(lo + c);
  float* h = reinterpret_cast<float*>(hi + c);
  atomic_fmin(l + 0, v.x);
  atomic_fmin(l + 1, v.y);
  atomic_fmin(l + 2, v.z);
  atomic_fmax(h + 0, v.x);
  atomic_fmax(h + 1, v.y);
  atomic_fmax(h + 2, v.z);
  atomicAdd(reinterpret_cast<unsigned int*>(l + 3), 1u);
}

// ---------------------------------------------------------------- math helpers
struct PoseDev {
  double rq[4], pos[3], lq[4], tli[3];  // quaternions (w, x, y, z)
  double R[9];                          // rot.matrix(), row-major
  double RL[9];                         // offset_R_L_I.matrix(), row-major
};

static_assert(sizeof(PoseDev) == 32 * sizeof(double), "PoseDev: 32 doubles (IkfCtl::pose)");
static_assert(sizeof(IkfCtl::pose[0]) == sizeof(PoseDev), "IkfCtl::pose slots hold a PoseDev");

// double e of pose_from_state(x) (the PoseDev layout), for the filter step
// to store the next pass's pose: the pass kernels then read it with scalar
// loads (pose_of_ctl) instead of forming the two matrices in vector
// registers that stay live through the kernel (in the search pass that
// pushed 3 float4 to scratch)
__device__ __forceinline__ double pose_elem(const slio_state& x, int e) {
  if (e < 4) return x.rot[e];
  if (e < 7) return x.pos[e - 4];
  if (e < 11) return x.rli[e - 7];
  if (e < 14) return x.tli[e - 11];
  const double* q = e < 23 ? x.rot : x.rli;
  const int k = e < 23 ? e - 14 : e - 23;
  double R[9];
  qmatrix(Quat{q[0], q[1], q[2], q[3]}, R);
  double v = R[0];
#pragma unroll
  for (int j = 1; j < 9; ++j) v = k == j ? R[j] : v;
  return v;
}
typedef __attribute__((address_space(4))) const double cdouble;  // constant: scalar loads
constexpr int kPoseSlots = 16;  // IkfCtl::pose
static_assert(offsetof(IkfCtl, pose) % 128 == 0 && sizeof(IkfCtl::pose) == kPoseSlots * 256, "IkfCtl: pose slots");
__device__ __forceinline__ PoseDev pose_of_ctl(const IkfCtl* ctl, int slot) {
  PoseDev P;
  cdouble* src = (cdouble*)(const void*)ctl->pose[slot & (kPoseSlots - 1)];
  double* dst = reinterpret_cast<double*>(&P);
#pragma unroll
  for (int e = 0; e < 32; ++e) dst[e] = src[e];
  return P;
}

__device__ __forceinline__ PoseDev pose_from_state(const slio_state& x) {
  PoseDev P;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    P.rq[j] = x.rot[j];
    P.lq[j] = x.rli[j];
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    P.pos[j] = x.pos[j];
    P.tli[j] = x.tli[j];
  }
  qmatrix(Quat{x.rot[0], x.rot[1], x.rot[2], x.rot[3]}, P.R);
  qmatrix(Quat{x.rli[0], x.rli[1], x.rli[2], x.rli[3]}, P.RL);
  return P;
}

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
  // without extrinsic estimation the reference's row ends in six zeros
  // (esekfom.hpp:218-220): B and C
  row[6] = B0;
  row[7] = B1;
  row[8] = B2;
  row[9] = extrinsic ? C0 : 0.0;
  row[10] = extrinsic ? C1 : 0.0;
  row[11] = extrinsic ? C2 : 0.0;
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
// Sorted top-5 list of 64-bit keys (float bits(squared distance) << 32) |
// position in the cell-sorted map: one u64 compare orders by distance, then
// by map position (squared distances are >= +0, whose bit patterns sort like
// the values).  The map index is read back from the point (float4.w) only for
// the five winners.
struct Top5 {
  uint64_t k[5];
};

__device__ __forceinline__ void top5_clear(Top5& t) {
#pragma unroll
  for (int j = 0; j < 5; ++j) t.k[j] = kInfKey;
}

// Branch-free insertion: slot j takes k[j-1] if key < k[j-1], key if
// k[j-1] <= key < k[j], else keeps k[j]; a key >= k[4] changes nothing.  All
// five slots update in parallel (no serial compare-swap chain, no divergent
// branch: across a wavefront some lane nearly always inserts).
__device__ __forceinline__ void top5_insert(Top5& t, uint64_t key) {
  bool c[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) c[j] = key < t.k[j];
#pragma unroll
  for (int j = 4; j > 0; --j) t.k[j] = c[j - 1] ? t.k[j - 1] : (c[j] ? key : t.k[j]);
  t.k[0] = c[0] ? key : t.k[0];
}

// A sorted top-5 list with the smallest squared distance it has DROPPED (an
// evicted entry or a rejected key): after a scan, every scanned candidate
// outside the list lies at >= m (the 6th distance of the scanned set).  The
// 5 and m certify later passes' searches (kNN certificate, k_search_pass).
struct Top5M {
  Top5 t;
  float m;
};

__device__ __forceinline__ void top5m_insert(Top5M& a, uint64_t key) {
  // the element that leaves (or never enters) the list; an empty slot's key
  // (all ones) reads as NaN, which fminf ignores
  const uint64_t drop = key < a.t.k[4] ? a.t.k[4] : key;
  a.m = fminf(a.m, __uint_as_float((uint32_t)(drop >> 32)));
  top5_insert(a.t, key);
}

// the same with the 6th entry kept (kNN certificates: the writer's list)
struct Top6M {
  uint64_t k[6];
  float m;
};

__device__ __forceinline__ void top6m_insert(Top6M& a, uint64_t key) {
  const uint64_t drop = key < a.k[5] ? a.k[5] : key;
  a.m = fminf(a.m, __uint_as_float((uint32_t)(drop >> 32)));
  bool c[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) c[j] = key < a.k[j];
#pragma unroll
  for (int j = 5; j > 0; --j) a.k[j] = c[j - 1] ? a.k[j - 1] : (c[j] ? key : a.k[j]);
  a.k[0] = c[0] ? key : a.k[0];
}

__device__ __forceinline__ void list_insert(Top5& t, uint64_t key) { top5_insert(t, key); }
__device__ __forceinline__ void list_insert(Top6M& t, uint64_t key) { top6m_insert(t, key); }
__device__ __forceinline__ void list_insert(Top5M& t, uint64_t key) { top5m_insert(t, key); }

__device__ __forceinline__ void consider(Top5& t, const float4 c, uint32_t pos, float qx, float qy,
                                         float qz) {
  const float ddx = qx - c.x, ddy = qy - c.y, ddz = qz - c.z;
  const float d = (ddx * ddx + ddy * ddy) + ddz * ddz;  // calc_dist, ikd_Tree.cpp:1539-1544
  top5_insert(t, ((uint64_t)__float_as_uint(d) << 32) | (uint64_t)pos);
}

// 64-bit lane exchange by DPP (a VALU operand modifier, no LDS round trip)
template <int CTRL>
__device__ __forceinline__ uint64_t dpp64(uint64_t v) {
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), CTRL, 0xF, 0xF, false);
  return ((uint64_t)(uint32_t)hi << 32) | (uint64_t)(uint32_t)lo;
}

template <int CTRL>
__device__ __forceinline__ void merge_round_dpp(Top5& t) {
  uint64_t ok[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) ok[j] = dpp64<CTRL>(t.k[j]);
#pragma unroll
  for (int j = 0; j < 5; ++j) top5_insert(t, ok[j]);
}
template <int CTRL>
__device__ __forceinline__ void merge_round_dpp(Top5M& a) {
  uint64_t ok[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) ok[j] = dpp64<CTRL>(a.t.k[j]);
  const float om = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(a.m), CTRL, 0xF, 0xF, false));
#pragma unroll
  for (int j = 0; j < 5; ++j) top5m_insert(a, ok[j]);
  a.m = fminf(a.m, om);
}

template <int CTRL>
__device__ __forceinline__ void merge_round_dpp(Top6M& a) {
  uint64_t ok[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) ok[j] = dpp64<CTRL>(a.k[j]);
  const float om = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(a.m), CTRL, 0xF, 0xF, false));
#pragma unroll
  for (int j = 0; j < 6; ++j) top6m_insert(a, ok[j]);
  a.m = fminf(a.m, om);
}

// the 2-lane merge of a query pair's lists (both lanes end with the merged
// list and the union's dropped minimum)
__device__ __forceinline__ void group_merge2(Top5M& a) { merge_round_dpp<0xB1>(a); }
__device__ __forceinline__ void group_merge2(Top6M& a) { merge_round_dpp<0xB1>(a); }

// butterfly merge of the LPQ per-lane lists of a query group (lanes of a
// group are consecutive and aligned, and all active or all inactive).  Up to
// 16 lanes by DPP: quad_perm [1,0,3,2] and [2,3,0,1] merge each quad, then
// row_half_mirror (lane i <-> 7 - i) pairs the two quads of 8 lanes and
// row_mirror (i <-> 15 - i) the two halves of 16; wider groups by ds_bpermute.
template <int LPQ>
__device__ __forceinline__ void group_merge(Top5& t) {
  if (LPQ >= 2) merge_round_dpp<0xB1>(t);
  if (LPQ >= 4) merge_round_dpp<0x4E>(t);
  if (LPQ >= 8) merge_round_dpp<0x141>(t);
  if (LPQ >= 16) merge_round_dpp<0x140>(t);
#pragma unroll
  for (int m = 16; m < LPQ; m <<= 1) {
    uint64_t ok[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) ok[j] = __shfl_xor(t.k[j], m);
#pragma unroll
    for (int j = 0; j < 5; ++j) top5_insert(t, ok[j]);
  }
}

// The same merge as a rolled loop over ds_bpermute rounds: for cold code
// (the refinement path runs in few workgroups, so its instructions are
// rarely in the instruction cache, and the unrolled DPP merge is ~5 KB).
__device__ __forceinline__ void group_merge_rolled(Top5& t, int width) {
#pragma unroll 1
  for (int m = 1; m < width; m <<= 1) {
    uint64_t ok[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) ok[j] = __shfl_xor(t.k[j], m);
#pragma unroll
    for (int j = 0; j < 5; ++j) top5_insert(t, ok[j]);
  }
}

// Conservative lower bound of the distance from coordinate q to the points
// assigned to grid cell i along one axis (cell edges are known to +-tol).
__device__ __forceinline__ float axis_gap(float q, int i, float o, float h, float tol) {
  const float lo = o + (float)i * h - tol;
  const float hi = o + (float)(i + 1) * h + tol;
  return fmaxf(fmaxf(lo - q, q - hi), 0.0f);
}

// A "run" is a contiguous x-range of cells in one (y, z) row: contiguous
// points in the cell-sorted map.  Runs are named by bits of a 64-bit mask:
// bit rr (0..24) = row (dy, dz) = (rr % 5 - 2, rr / 5 - 2) of the 5x5 rows
// around the query cell, bit 32 + rr = a second (right) segment of that row.
// Search regions (all exact, see k_search_pass):
//   mode 1: the 3x3x3 block (x in [cx-1, cx+1]);
//   mode 2: cells of the 5x5x5 cube with box gap^2 <= lim, minus the 3x3x3 block;
//   mode 3: cells of the 5x5x5 cube with box gap^2 <= lim (a sphere);
//   mode 4: cells with lim0 < box gap^2 <= lim (the shell a grown sphere adds).
struct RunCtx {
  int cx, cy, cz;
  float qx, qy, qz;
  int mode;
  float lim0, lim;
};

__device__ __forceinline__ float sq_gap(float q, int i, float o, const GridGeom& g) {
  const float a = axis_gap(q, i, o, g.h, g.tol);
  return a * a;
}

// rows of the 5x5 whose (y, z) gap is within lim and which lie in the grid
__device__ __forceinline__ uint64_t sphere_rows(const GridGeom& g, const RunCtx& rc, float lim) {
  float gy[5], gz[5];
#pragma unroll
  for (int d = 0; d < 5; ++d) {
    gy[d] = sq_gap(rc.qy, rc.cy - 2 + d, g.oy, g);
    gz[d] = sq_gap(rc.qz, rc.cz - 2 + d, g.oz, g);
  }
  uint64_t m = 0;
#pragma unroll
  for (int rr = 0; rr < 25; ++rr) {
    const int dy = rr % 5, dz = rr / 5;
    const int yy = rc.cy - 2 + dy, zz = rc.cz - 2 + dz;
    const bool in = yy >= 0 && yy < g.dy && zz >= 0 && zz < g.dz;
    if (in && gy[dy] + gz[dz] <= lim) m |= 1ull << rr;
  }
  return m;
}

// contiguous x-range [lo, hi] around cx of the cells with gap^2 <= rem
__device__ __forceinline__ void sphere_span(const GridGeom& g, const RunCtx& rc, float rem, int& lo,
                                            int& hi) {
  const float gm2 = sq_gap(rc.qx, rc.cx - 2, g.ox, g), gm1 = sq_gap(rc.qx, rc.cx - 1, g.ox, g);
  const float gp1 = sq_gap(rc.qx, rc.cx + 1, g.ox, g), gp2 = sq_gap(rc.qx, rc.cx + 2, g.ox, g);
  lo = (gm2 <= rem) ? rc.cx - 2 : (gm1 <= rem) ? rc.cx - 1 : rc.cx;
  hi = (gp2 <= rem) ? rc.cx + 2 : (gp1 <= rem) ? rc.cx + 1 : rc.cx;
  if (rem < 0.0f) {
    lo = 1;
    hi = 0;
  }
}

__device__ __forceinline__ void run_range(const GridGeom& g, const RunCtx& rc, int bit, int& yy,
                                          int& zz, int& xa, int& xb) {
  const int rr = bit & 31;
  const int dy = rr % 5, dz = rr / 5;
  yy = rc.cy - 2 + dy;
  zz = rc.cz - 2 + dz;
  const bool right = bit >= 32;
  if (rc.mode == 1) {
    xa = rc.cx - 1;
    xb = rc.cx + 1;
  } else {
    // recomputed rather than looked up: a runtime-indexed gy[]/gz[] would be
    // lowered to scratch memory
    const float gyz = sq_gap(rc.qy, yy, g.oy, g) + sq_gap(rc.qz, zz, g.oz, g);
    int lo, hi;
    sphere_span(g, rc, rc.lim - gyz, lo, hi);
    if (rc.mode == 3) {
      xa = lo;
      xb = hi;
    } else {
      // exclude the cells an earlier pass already scanned: [cx-1, cx+1] of
      // the inner rows (mode 2) or the smaller sphere's span (mode 4)
      int lo0, hi0;
      if (rc.mode == 2) {
        const bool inner = dy >= 1 && dy <= 3 && dz >= 1 && dz <= 3;
        lo0 = inner ? rc.cx - 1 : 1;
        hi0 = inner ? rc.cx + 1 : 0;
      } else {
        sphere_span(g, rc, rc.lim0 - gyz, lo0, hi0);
      }
      if (lo0 > hi0) {  // nothing scanned before in this row
        xa = right ? 1 : lo;
        xb = right ? 0 : hi;
      } else if (!right) {
        xa = lo;
        xb = min(hi, lo0 - 1);
      } else {
        xa = max(lo, hi0 + 1);
        xb = hi;
      }
    }
  }
  xa = max(xa, 0);
  xb = min(xb, g.dx - 1);
  if (yy < 0 || yy >= g.dy || zz < 0 || zz >= g.dz) {
    xa = 1;
    xb = 0;
  }
}

// Strided, software-pipelined sweep of a flattened candidate list made of up
// to 9 contiguous runs (rs = run starts, pre = prefix lengths, T = total): the
// U loads of step k+1 are issued before step k's candidates are consumed.
// Flat position tt lies in the last run q with pre[q] <= tt, at map position
// tt + (rs[q] - pre[q]): one compare and one select per run.  The run bounds
// p1..p8 and deltas d0..d8 are plain local scalars of scan_flat (a macro, not
// an array or struct: from a memory object the compiler turns the select
// chain into a select of an index plus a load from scratch memory).
#define SLIO_FLAT_POS(tt, out)   \
  do {                            \
    int32_t d_ = d0;              \
    d_ = (tt) >= p1 ? d1 : d_;    \
    d_ = (tt) >= p2 ? d2 : d_;    \
    d_ = (tt) >= p3 ? d3 : d_;    \
    d_ = (tt) >= p4 ? d4 : d_;    \
    d_ = (tt) >= p5 ? d5 : d_;    \
    d_ = (tt) >= p6 ? d6 : d_;    \
    d_ = (tt) >= p7 ? d7 : d_;    \
    d_ = (tt) >= p8 ? d8 : d_;    \
    (out) = (tt) + (uint32_t)d_;  \
  } while (0)

// U addresses of step t0; slots past the end re-read the list's last
// candidate (valid: T >= 1), so loads need no branch
#define SLIO_FLAT_ADDR(t0, a)                                          \
  do {                                                                 \
    _Pragma("unroll") for (int u = 0; u < U; ++u) {                    \
      const uint32_t tt_ = min((t0) + u * LPQ, T - 1);                 \
      SLIO_FLAT_POS(tt_, a[u]);                                        \
    }                                                                  \
  } while (0)

// distances of U loaded candidates into the lane's list (past the end: a
// no-op key instead of a branch)
template <int LPQ, int U>
__device__ __forceinline__ void consume(Top5& t, const float4 (&c)[U], const uint32_t (&a)[U],
                                        uint32_t t0, uint32_t T, float qx, float qy, float qz) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const float ddx = qx - c[u].x, ddy = qy - c[u].y, ddz = qz - c[u].z;
    const float d = (ddx * ddx + ddy * ddy) + ddz * ddz;  // calc_dist, ikd_Tree.cpp:1539-1544
    const uint64_t key = ((uint64_t)__float_as_uint(d) << 32) | (uint64_t)a[u];
    top5_insert(t, (t0 + u * LPQ < T) ? key : kInfKey);
  }
}

// Two register sets (A, B) alternate, so the loads of step k+1 stay in flight
// while step k is consumed: no loop-carried copy of loaded registers (a copy
// makes the compiler wait for the loads at the end of the iteration).  The run
// deltas are plain scalars (SLIO_FLAT_POS).
template <int LPQ, int U>
__device__ __forceinline__ void scan_flat(const float4* __restrict__ pts, const uint32_t (&rs)[9],
                                          const uint32_t (&pre)[10], uint32_t T, int sub,
                                          float qx, float qy, float qz, Top5& t) {
  uint32_t t0 = sub;
  if (t0 >= T) return;
  const uint32_t p1 = pre[1], p2 = pre[2], p3 = pre[3], p4 = pre[4], p5 = pre[5], p6 = pre[6],
                 p7 = pre[7], p8 = pre[8];
  const int32_t d0 = (int32_t)(rs[0] - pre[0]), d1 = (int32_t)(rs[1] - pre[1]),
                d2 = (int32_t)(rs[2] - pre[2]), d3 = (int32_t)(rs[3] - pre[3]),
                d4 = (int32_t)(rs[4] - pre[4]), d5 = (int32_t)(rs[5] - pre[5]),
                d6 = (int32_t)(rs[6] - pre[6]), d7 = (int32_t)(rs[7] - pre[7]),
                d8 = (int32_t)(rs[8] - pre[8]);
  constexpr uint32_t kStep = U * LPQ;
  uint32_t aA[U], aB[U];
  float4 cA[U], cB[U];
  SLIO_FLAT_ADDR(t0, aA);
#ifdef SLIO_BOUNDS_CHECK
  for (int u = 0; u < U; ++u) SLIO_BCHK(aA[u], c_dbg_npts, "flat0");
#endif
#pragma unroll
  for (int u = 0; u < U; ++u) cA[u] = pts[aA[u]];
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  for (;;) {
    // set B is consumed even when it lies wholly past the end (its keys are
    // then no-ops): a loop exit between its loads and their use would let the
    // compiler sink the loads down to the use
    const uint32_t t1 = t0 + kStep, t2 = t1 + kStep;
    SLIO_FLAT_ADDR(t1, aB);
#ifdef SLIO_BOUNDS_CHECK
    for (int u = 0; u < U; ++u) SLIO_BCHK(aB[u], c_dbg_npts, "flatB");
#endif
#pragma unroll
    for (int u = 0; u < U; ++u) cB[u] = pts[aB[u]];
    // keep the loads here: not merged with the other set's, not sunk to their use
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    consume<LPQ, U>(t, cA, aA, t0, T, qx, qy, qz);
    SLIO_FLAT_ADDR(t2, aA);
#ifdef SLIO_BOUNDS_CHECK
    for (int u = 0; u < U; ++u) SLIO_BCHK(aA[u], c_dbg_npts, "flatA");
#endif
#pragma unroll
    for (int u = 0; u < U; ++u) cA[u] = pts[aA[u]];
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    consume<LPQ, U>(t, cB, aB, t1, T, qx, qy, qz);
    if (t2 >= T) break;
    t0 = t2;
  }
}

// The 3x3x3 block from the block rows: one contiguous range, so a flat
// position is an address (no run lookup); keys carry the pts position (.w),
// identical to the keys of the 9-run scan.  Same pipeline as scan_flat.
template <int LPQ, int U, class TL>
__device__ __forceinline__ void scan_block_rows(const float4* __restrict__ blk, uint32_t s,
                                                uint32_t T, int sub, float qx, float qy, float qz,
                                                TL& t) {
  uint32_t t0 = sub;
  if (t0 >= T) return;
  constexpr uint32_t kStep = U * LPQ;
  float4 cA[U], cB[U];
#pragma unroll
  for (int u = 0; u < U; ++u) cA[u] = blk[s + min(t0 + u * LPQ, T - 1)];
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  auto eat = [&](const float4 (&c)[U], uint32_t tb) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float ddx = qx - c[u].x, ddy = qy - c[u].y, ddz = qz - c[u].z;
      const float d = (ddx * ddx + ddy * ddy) + ddz * ddz;  // calc_dist, ikd_Tree.cpp:1539-1544
      const uint64_t key = ((uint64_t)__float_as_uint(d) << 32) | (uint64_t)__float_as_uint(c[u].w);
      list_insert(t, (tb + u * LPQ < T) ? key : kInfKey);
    }
  };
  for (;;) {
    const uint32_t t1 = t0 + kStep, t2 = t1 + kStep;
#pragma unroll
    for (int u = 0; u < U; ++u) cB[u] = blk[s + min(t1 + u * LPQ, T - 1)];
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    eat(cA, t0);
#pragma unroll
    for (int u = 0; u < U; ++u) cA[u] = blk[s + min(t2 + u * LPQ, T - 1)];
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    eat(cB, t1);
    if (t2 >= T) break;
    t0 = t2;
  }
}

// Scan the runs of `mask` into the lane's list: run bounds are fetched 9 runs
// at a time (their loads overlap), then the lanes of the group stride over
// the flattened candidate list with U float4 loads in flight per lane.
template <int LPQ, int U>
__device__ __forceinline__ void scan_runs(const float4* __restrict__ pts, const uint32_t* __restrict__ start,
                          const GridGeom& g, const RunCtx& rc, uint64_t mask, int sub, Top5& t) {
  while (mask) {
    uint32_t rs[9], pre[10];
    pre[0] = 0;
#pragma unroll
    for (int q = 0; q < 9; ++q) {
      uint32_t s = 0, e = 0;
      if (mask) {
        const int bit = __ffsll((unsigned long long)mask) - 1;
        mask &= mask - 1;
        int yy, zz, xa, xb;
        run_range(g, rc, bit, yy, zz, xa, xb);
        if (xa <= xb) {
          const uint32_t rb = ((uint32_t)zz * (uint32_t)g.dy + (uint32_t)yy) * (uint32_t)g.dx;
#ifdef SLIO_BOUNDS_CHECK
          uint32_t j0 = rb + xa, j1 = rb + xb + 1;
          SLIO_BCHK(j0, c_dbg_ncells + 1, "runs0");
          SLIO_BCHK(j1, c_dbg_ncells + 1, "runs1");
#endif
          s = start[rb + xa];
          e = start[rb + xb + 1];
        }
      }
      rs[q] = s;
      pre[q + 1] = pre[q] + (e - s);
    }
    const uint32_t T = pre[9];
    scan_flat<LPQ, U>(pts, rs, pre, T, sub, rc.qx, rc.qy, rc.qz, t);
  }
}

// Full grid-clamped cube [c-r, c+r]^3 (general fallback: queries outside the
// grid, or a 5th neighbour beyond the 5x5x5 cube).
template <int LPQ, int U>
__device__ __forceinline__ void scan_cube(const float4* __restrict__ pts, const uint32_t* __restrict__ start,
                          const GridGeom& g, int cx, int cy, int cz, int r, int sub, float qx,
                          float qy, float qz, Top5& t) {
  const int z0 = max(cz - r, 0), z1 = min(cz + r, g.dz - 1);
  const int y0 = max(cy - r, 0), y1 = min(cy + r, g.dy - 1);
  const int xlo = max(cx - r, 0), xhi = min(cx + r, g.dx - 1);
  if (xlo > xhi || y0 > y1 || z0 > z1) return;
  const int ny = y1 - y0 + 1;
  const int nrun = ny * (z1 - z0 + 1);
  for (int j0 = 0; j0 < nrun; j0 += 9) {
    uint32_t rs[9], pre[10];
    pre[0] = 0;
#pragma unroll
    for (int q = 0; q < 9; ++q) {
      const int j = j0 + q;
      const bool ok = j < nrun;
      const int jj = ok ? j : 0;
      const int yy = y0 + jj % ny, zz = z0 + jj / ny;
      const uint32_t rb = ((uint32_t)zz * (uint32_t)g.dy + (uint32_t)yy) * (uint32_t)g.dx;
      const uint32_t s = start[rb + xlo];
      const uint32_t e = start[rb + xhi + 1];
      rs[q] = s;
      pre[q + 1] = pre[q] + (ok ? e - s : 0u);
    }
    const uint32_t T = pre[9];
    for (uint32_t t0 = sub; t0 < T; t0 += U * LPQ) {
      uint32_t a[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t tt = t0 + u * LPQ;
        uint32_t ad = 0;
#pragma unroll
        for (int q = 0; q < 9; ++q)
          if (tt >= pre[q]) ad = rs[q] + (tt - pre[q]);
        a[u] = ad;
      }
#pragma unroll
      for (int u = 1; u < U; ++u) a[u] = (t0 + u * LPQ < T) ? a[u] : a[0];
      float4 c[U];
#ifdef SLIO_BOUNDS_CHECK
      for (int u = 0; u < U; ++u) SLIO_BCHK(a[u], c_dbg_npts, "cube");
#endif
#pragma unroll
      for (int u = 0; u < U; ++u) c[u] = pts[a[u]];
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (t0 + u * LPQ < T) consider(t, c[u], a[u], qx, qy, qz);
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
  int32_t* nbr_idx;  // n * 5  (map point ids)
  uint32_t* nbr_pos; // n * 5  (positions in the cell-sorted pts, for map_incremental)
  float* nbr_sqd;    // n * 5
  float4* plane;     // n
  uint8_t* sel;      // n
  float* resid;      // n
  double* chunk_part;  // C * NPROD (global chunk index)
  uint32_t* far_ctr;   // [1]: deferred (far) queries of this pass, all chunks
  PoseDev* pose;       // the pass's pose (block 0), for nbr_settle
  uint32_t* chunk_cost;  // per chunk of the rank (relative index): candidates + refinement / far weights
  // kNN certificates (device-resident passes after the first, see
  // k_search_pass): per point the query of its last full search and the
  // squared-distance bound G of every map point outside its 5 nearest (which
  // nbr_pos holds); per chunk the update epoch the entries belong to
  float4* kq;
  uint32_t* k6;         // the 6th of the certified set (nbr_pos holds the other 5)
  uint32_t* kepoch;     // per chunk (global index)
  uint32_t* kc_count;   // [0] certified queries, [1] queries searched with a certificate written
};

// far_query_margin: squared distance from the query to the grid's bounding box
__device__ __forceinline__ bool far_outside(const GridGeom& g, float far_sq, float qx, float qy,
                                            float qz) {
  if (far_sq <= 0.0f) return false;
  const float gx = fmaxf(fmaxf(g.ox - qx, qx - (g.ox + g.h * (float)g.dx)), 0.0f);
  const float gy = fmaxf(fmaxf(g.oy - qy, qy - (g.oy + g.h * (float)g.dy)), 0.0f);
  const float gz = fmaxf(fmaxf(g.oz - qz, qz - (g.oz + g.h * (float)g.dz)), 0.0f);
  return gx * gx + gy * gy + gz * gz > far_sq;
}

struct PassCfg {
  IkfCtl* ctl;        // device-resident update: pose + pass selection from HBM (else null)
  int want_search;    // with ctl: run only if ctl->search_now == want_search
  float plane_thr;
  float max_sqd;
  float radius_sq;  // sphere-first search radius^2 (0: 3x3x3 block first)
  float far_sq;     // far_query_margin^2 (0: no cut)
  int extrinsic;
  int64_t c_begin, c_end;  // global chunk range of this rank
  int pass_idx;            // with ctl: run only if ctl->passes == pass_idx
  int knn_only;            // 1: neighbours only (nbr_*), no fit / rows / products
  int mfma;                // chunk sums on the matrix cores (chunk_products_mfma), else VALU
  const uint32_t* perm;    // block -> chunk order within each XCD's range (chunk_order), or null
  uint32_t kc_epoch;       // kNN certificates of this update (0: off); see k_search_pass
  int32_t seq;             // fused group pass: run only if ctl->seq == seq (0: no check)
};

// The plane output's .x bits when esti_plane rejected the point's 5 neighbours
// (a quiet NaN: the output reads as NaN, as the oracle's, and a certified pass
// whose 5 keep their order reuses the rejection without the QR)
constexpr uint32_t kPlaneRejected = 0x7fc00e57u;

// ---------------------------------------------------------------- far queries
// A query the fine grid cannot finish (its 5th neighbour lies beyond the
// 5x5x5 fine cube, or its cell lies outside the grid) is DEFERRED to the end
// of the kNN phase of its workgroup, where the workgroup's wavefronts answer
// the chunk's deferred queries one per wavefront (far_search, all 64 lanes
// on one query).  Such queries are rare (returns with no map support within
// a few metres, e.g. a scan taken from inside a building or far outside the
// map); handled inline on their own 2 lanes they serialised the wavefront
// that held them.  (An earlier global work queue spread them over the chip
// but made workgroups wait on each other; this keeps every workgroup
// independent.)
typedef __attribute__((address_space(1))) uint32_t gu32;

__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void wave_fence() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ void st_sc1_u32(uint32_t* p, uint32_t v) {
  __hip_atomic_store((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_sc1_u32(const uint32_t* p) {
  return __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// exclusive prefix sum over the wavefront's 64 lanes; total to every lane
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t& total) {
  const int lane = threadIdx.x & 63;
  uint32_t s = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(s, d, 64);
    if (lane >= d) s += o;
  }
  total = __shfl(s, 63, 64);
  return s - v;
}

// The exact 5-NN of one query by a whole wavefront on the coarse level:
// Chebyshev rings R = 0, 1, ... of coarse cells around the query's (clamped)
// cell; a cell is scanned unless its tight box lies farther than the bound
// (the 5th distance found so far, or bound0: the 5th distance of 5 real map
// points, or +inf).  The candidate cells of a batch of 64 ring positions are
// expanded, four at a time, into their 16 runs of the fine pts (one per fine
// (y, z) row), flattened into one list (lane prefix sums in LDS, a 6-step
// binary search per candidate) and swept with U loads in flight per lane.  The search ends
// when every unscanned cell lies beyond the 5th distance: the bound over the
// six slabs outside the ring's cube is per-axis exact (face distance on the
// slab's axis, distance to the grid's range on the other two).  Keys carry
// the fine pts position, so results equal the fine grid's.  Returns the list
// in every lane.
template <int U>
__device__ __forceinline__ void far_search(const MapView& map, float qx, float qy, float qz,
                                        float bound, uint32_t* __restrict__ pre,
                                        uint32_t* __restrict__ beg, Top5& t) {
  const int lane = threadIdx.x & 63;
  const CoarseView& cv = map.cl;
  const GridGeom g = cv.g, fg = map.g;
  const float INF = __int_as_float(0x7f800000);
  top5_clear(t);
  bool full = false;
  float d5 = INF;
  const int CX = min(max(cell_coord(qx, g.ox, g.inv_h), 0), g.dx - 1);
  const int CY = min(max(cell_coord(qy, g.oy, g.inv_h), 0), g.dy - 1);
  const int CZ = min(max(cell_coord(qz, g.oz, g.inv_h), 0), g.dz - 1);
  // distance of q to the grid's range on each axis (every map point lies in it)
  auto range_gap = [&](float q, float o, int d) {
    const float lo = o - g.tol, hi = o + (float)d * g.h + g.tol;
    return fmaxf(fmaxf(lo - q, q - hi), 0.0f);
  };
  const float ax = range_gap(qx, g.ox, g.dx), ay = range_gap(qy, g.oy, g.dy),
              az = range_gap(qz, g.oz, g.dz);
  // conservative squared gap from q to the cells [a0, a1] of one axis
  auto span_gap = [&](float q, float o, int a0, int a1) {
    const float lo = o + (float)a0 * g.h - g.tol, hi = o + (float)(a1 + 1) * g.h + g.tol;
    const float d = fmaxf(fmaxf(lo - q, q - hi), 0.0f);
    return d * d;
  };
  for (int R = 0;; ++R) {
    const int x0 = max(CX - R, 0), x1 = min(CX + R, g.dx - 1);
    const int y0 = max(CY - R, 0), y1 = min(CY + R, g.dy - 1);
    const int z0 = max(CZ - R, 0), z1 = min(CZ + R, g.dz - 1);
    // the ring's shell (cube R minus cube R-1, clipped to the grid) as up to
    // six face rectangles: x faces over the full (y, z) span, y faces over
    // the inner x span, z faces over the inner x and y spans.  A face whose
    // box lies beyond the bound is skipped whole (its cells would all fail
    // the per-cell test below).
    const int xi0 = max(CX - R + 1, 0), xi1 = min(CX + R - 1, g.dx - 1);
    const int yi0 = max(CY - R + 1, 0), yi1 = min(CY + R - 1, g.dy - 1);
    const float lim_f = fminf(bound, d5);
    int fa[6], fna[6], fb[6], fv[6], cum[7];
    cum[0] = 0;
#pragma unroll
    for (int f = 0; f < 6; ++f) {
      const int fax = f >> 1;                              // fixed axis
      const int C = fax == 0 ? CX : fax == 1 ? CY : CZ;
      const int D = fax == 0 ? g.dx : fax == 1 ? g.dy : g.dz;
      const int v = (f & 1) ? C + R : C - R;
      const bool ok = (f == 0 || R > 0) && v >= 0 && v < D;
      int a0, a1, b0, b1;
      float gsum;
      if (fax == 0) {
        a0 = y0; a1 = y1; b0 = z0; b1 = z1;
        gsum = (span_gap(qx, g.ox, v, v) + span_gap(qy, g.oy, a0, a1)) + span_gap(qz, g.oz, b0, b1);
      } else if (fax == 1) {
        a0 = xi0; a1 = xi1; b0 = z0; b1 = z1;
        gsum = (span_gap(qx, g.ox, a0, a1) + span_gap(qy, g.oy, v, v)) + span_gap(qz, g.oz, b0, b1);
      } else {
        a0 = xi0; a1 = xi1; b0 = yi0; b1 = yi1;
        gsum = (span_gap(qx, g.ox, a0, a1) + span_gap(qy, g.oy, b0, b1)) + span_gap(qz, g.oz, v, v);
      }
      const bool live_f = ok && a0 <= a1 && b0 <= b1 && !(gsum * 0.99999f > lim_f);
      fa[f] = a0;
      fb[f] = b0;
      fv[f] = v;
      fna[f] = live_f ? a1 - a0 + 1 : 0;
      cum[f + 1] = cum[f] + (live_f ? (a1 - a0 + 1) * (b1 - b0 + 1) : 0);
    }
    const int total = cum[6];
    for (int base = 0; base < total; base += 64) {
      const int p = base + lane;
      bool pass = false;
      int ccx = 0, ccy = 0, ccz = 0;
      if (p < total) {
        int f = 0;
#pragma unroll
        for (int j = 1; j < 6; ++j) f = p >= cum[j] ? j : f;
        int A = 0, B = 0, V = 0, NA = 1;
#pragma unroll
        for (int j = 0; j < 6; ++j)
          if (f == j) {
            A = fa[j];
            B = fb[j];
            V = fv[j];
            NA = fna[j];
          }
        const int l = p - (f == 0 ? 0 : f == 1 ? cum[1] : f == 2 ? cum[2] : f == 3 ? cum[3] : f == 4 ? cum[4] : cum[5]);
        const int ua = A + l % NA, ub = B + l / NA;
        const int fax = f >> 1;
        ccx = fax == 0 ? V : ua;
        ccy = fax == 0 ? ua : fax == 1 ? V : ub;
        ccz = fax == 2 ? V : ub;
        const uint32_t c = ((uint32_t)ccz * (uint32_t)g.dy + (uint32_t)ccy) * (uint32_t)g.dx + (uint32_t)ccx;
        const float4 lo = cv.lo[c];
        if (__float_as_uint(lo.w)) {
          const float4 hi = cv.hi[c];
          const float gx = fmaxf(fmaxf(lo.x - qx, qx - hi.x), 0.0f);
          const float gy = fmaxf(fmaxf(lo.y - qy, qy - hi.y), 0.0f);
          const float gz = fmaxf(fmaxf(lo.z - qz, qz - hi.z), 0.0f);
          const float gd = (gx * gx + gy * gy) + gz * gz;
          pass = !(gd > fminf(bound, d5));  // a point at exactly d5 may still win on position
        }
      }
      // the passing coarse cells, four at a time: lane l reads the bounds of
      // fine row (l & 15) of passing cell (l >> 4), one run of the fine pts
      uint64_t pm = __ballot(pass);
      const int gi = lane >> 4, sl = lane & 15;
      while (pm) {
        uint64_t bm = pm;
        for (int q = 0; q < gi && bm; ++q) bm &= bm - 1;  // the gi-th passing cell
        const bool act = bm != 0;
        const int src = act ? __ffsll((unsigned long long)bm) - 1 : 0;
        // (every lane shuffles: a cross-lane read inside a condition would
        // read lanes the condition turned off)
        const int x = __shfl(ccx, src, 64), y = __shfl(ccy, src, 64), z = __shfl(ccz, src, 64);
        for (int q = 0; q < 4 && pm; ++q) pm &= pm - 1;
        uint32_t s = 0, k = 0;
        const int fy = 4 * y + (sl & 3), fz = 4 * z + (sl >> 2);
        if (act && fy < fg.dy && fz < fg.dz) {
          const int64_t rb = ((int64_t)fz * fg.dy + fy) * fg.dx;
          s = map.start[rb + 4 * x];
          k = map.start[rb + min(4 * x + 4, fg.dx)] - s;
        }
        if (!__any(k != 0)) continue;
        uint32_t tot;
        const uint32_t ex = wave_excl_scan(k, tot);
        pre[lane] = ex;
        beg[lane] = s;
        wave_fence();
        for (uint32_t f0 = 0; f0 < tot; f0 += 64 * U) {
          uint32_t a[U];
          float4 c[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const uint32_t f = min(f0 + (uint32_t)(u * 64 + lane), tot - 1);
            int j = 0;
#pragma unroll
            for (int st = 32; st > 0; st >>= 1)
              if (pre[j + st] <= f) j += st;
            a[u] = beg[j] + (f - pre[j]);
          }
#pragma unroll
          for (int u = 0; u < U; ++u) c[u] = map.pts[a[u]];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const float ddx = qx - c[u].x, ddy = qy - c[u].y, ddz = qz - c[u].z;
            const float d = (ddx * ddx + ddy * ddy) + ddz * ddz;  // calc_dist, ikd_Tree.cpp:1539-1544
            const uint64_t key = ((uint64_t)__float_as_uint(d) << 32) | (uint64_t)a[u];
            top5_insert(t, (f0 + (uint32_t)(u * 64 + lane) < tot) ? key : kInfKey);
          }
        }
        group_merge<64>(t);  // every lane: the merged list
        full = t.k[4] != kInfKey;
        if (full) d5 = __uint_as_float((uint32_t)(t.k[4] >> 32));
        if (lane != 0) top5_clear(t);  // lane 0 keeps it
        wave_fence();                  // pre / beg are rewritten by the next batch
      }
    }
    // lower bound of the squared distance to every cell outside this cube
    float lb = INF;
    bool covers = true;
    auto slab = [&](bool open, float face_gap, float o1, float o2) {
      if (!open) return;
      covers = false;
      const float f = fmaxf(face_gap, 0.0f);
      lb = fminf(lb, (f * f + o1 * o1) + o2 * o2);
    };
    slab(x0 > 0, qx - (g.ox + (float)x0 * g.h + g.tol), ay, az);
    slab(x1 < g.dx - 1, (g.ox + (float)(x1 + 1) * g.h - g.tol) - qx, ay, az);
    slab(y0 > 0, qy - (g.oy + (float)y0 * g.h + g.tol), ax, az);
    slab(y1 < g.dy - 1, (g.oy + (float)(y1 + 1) * g.h - g.tol) - qy, ax, az);
    slab(z0 > 0, qz - (g.oz + (float)z0 * g.h + g.tol), ax, ay);
    slab(z1 < g.dz - 1, (g.oz + (float)(z1 + 1) * g.h - g.tol) - qz, ax, ay);
    if (covers || (full && d5 < lb * 0.99999f)) break;
    if (R > g.dx + g.dy + g.dz) break;  // unreachable: the cube covers the grid long before
  }
#pragma unroll
  for (int j = 0; j < 5; ++j) t.k[j] = __shfl(t.k[j], 0, 64);
}

__device__ __forceinline__ int64_t xcd_chunk(int64_t c_begin, int64_t nblk) {
  // blocks b and b+8 share an XCD: give each XCD group a contiguous chunk range
  const int64_t b = blockIdx.x;
  const int64_t xcd = b & 7, q = nblk >> 3, rr = nblk & 7;
  const int64_t base = xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q;
  return c_begin + base + (b >> 3);
}

// ---------------------------------------------------------------- filter step
constexpr int kSolveThreads = 256;
constexpr int kSuperSeg = 8;                     // segments per super-chunk
constexpr int kNSeg = SLIO_NSUPER * kSuperSeg;   // segment rows per pass: one workgroup each

// global-address-space views for the in-launch hand-off (sc1 accesses)
typedef __attribute__((address_space(1))) double gdouble;
typedef __attribute__((address_space(1))) uint32_t guint;
typedef __attribute__((address_space(1))) uint64_t guint64;

__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store((gdouble*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double* p) {
  return __hip_atomic_load((gdouble*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The caller's mapped host block is read with system-scope loads: the previous update's final
// workgroup wrote the same lines from the GPU (x, P, the flags), and a plain
// load on that workgroup's XCD could be served from its L2 copy instead of
// the host's new contents.
__device__ __forceinline__ double ld_sys(const double* p) {
  return __hip_atomic_load((const gdouble*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint32_t ld_sys_u32(const uint32_t* p) {
  return __hip_atomic_load((const guint*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// Per-point outputs of a pass (plane, selection, residual, neighbour
// positions, certificates), stored write-through (sc1): they leave no dirty
// lines in the XCDs' L2s for the end-of-kernel write-back that every pass
// boundary waits for.  SLIO_OUT_MODE (A/B): 0 plain stores, 1 agent-scope
// atomic stores (16-B values as two 8-B halves), 2 non-temporal stores, 3
// (default) 16-B values as one global_store_dwordx4 sc1 -- whole lines per
// wavefront instead of two half-line writes each
#ifndef SLIO_OUT_MODE
#define SLIO_OUT_MODE 3
#endif
typedef __attribute__((address_space(1))) uint8_t gu8;
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_out16(void* p, uint32_t x, uint32_t y, uint32_t z, uint32_t w) {
#if SLIO_OUT_MODE == 0
  *reinterpret_cast<uint4*>(p) = make_uint4(x, y, z, w);
#elif SLIO_OUT_MODE == 1
  __hip_atomic_store((guint64*)(uint64_t*)p, ((uint64_t)y << 32) | x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store((guint64*)(uint64_t*)p + 1, ((uint64_t)w << 32) | z, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
#elif SLIO_OUT_MODE == 2
  v4u32 v = {x, y, z, w};
  __builtin_nontemporal_store(v, reinterpret_cast<v4u32*>(p));
#else
  v4u32 v = {x, y, z, w};
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
#endif
}
__device__ __forceinline__ void st_out(float4* p, float4 v) {
  st_out16(p, __float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w));
}
__device__ __forceinline__ void st_out(uint4* p, uint4 v) { st_out16(p, v.x, v.y, v.z, v.w); }
__device__ __forceinline__ void st_out(uint32_t* p, uint32_t v) {
#if SLIO_OUT_MODE == 0
  *p = v;
#elif SLIO_OUT_MODE == 2
  __builtin_nontemporal_store(v, p);
#else
  __hip_atomic_store((guint*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
}
__device__ __forceinline__ void st_out(float* p, float v) { st_out(reinterpret_cast<uint32_t*>(p), __float_as_uint(v)); }
__device__ __forceinline__ void st_out(uint8_t* p, uint8_t v) {
#if SLIO_OUT_MODE == 0
  *p = v;
#elif SLIO_OUT_MODE == 2
  __builtin_nontemporal_store(v, p);
#else
  __hip_atomic_store((gu8*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
}

__device__ __forceinline__ uint32_t arrive(uint32_t* p) {
  return __hip_atomic_fetch_add((guint*)p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void reset_counter(uint32_t* p) {
  __hip_atomic_store((guint*)p, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// LDS of the filter step.  D = 6 without extrinsic estimation (H's columns
// 6..11 are zero, esekfom.hpp:218-220), 12 with it.
struct StepLds {
  struct {
    double Z[144];  // D x D: S^-1 M             (P update)
    double K[288];  // 24 x D: G S^-1 M = K H[:, :D]
  } zk;
  double sup[SLIO_NSUPER][SLIO_NPROD];  // super-chunk sums
  double tot[SLIO_NPROD];               // H^T H (78, upper triangle), H^T h (12), m
  double Mt[SLIO_NHTH];                 // H^T H / R (upper triangle)
  double hR[12];                        // H^T h / R
  double P[576];
  double P11i[144];                     // D x D: (P[:D, :D])^-1
  double G[288];                        // 24 x D: P[:, :D] P11^-1
  double dxn[24];
  slio_state x, xprop;                  // staged control-block fields
  int32_t fl[8];
  int ok, s_final;
};
static_assert(offsetof(IkfCtl, xprop) == sizeof(slio_state), "IkfCtl: x, xprop adjacent");
static_assert(offsetof(StepLds, xprop) - offsetof(StepLds, x) == sizeof(slio_state),
              "StepLds: x, xprop adjacent");
static_assert(offsetof(IkfCtl, mode) - offsetof(IkfCtl, converge) == 7 * sizeof(int32_t),
              "IkfCtl: 8 contiguous flags");
constexpr int kStateD = sizeof(slio_state) / sizeof(double);
// flag slots of IkfCtl::converge..mode
enum { F_CONV, F_T, F_DONE, F_SEARCH, F_PASSES, F_SEARCHES, F_VALID, F_MODE };

// upper-triangle product index of (i, j), i <= j (product_table order)
__device__ __forceinline__ int tri_index(int i, int j) { return i * 12 - (i * (i - 1)) / 2 + (j - i); }

// double offset inside slio_state of error-state component k in [0, 24) for
// the vector blocks (pos 0-2, T_LI 9-11, vel, bg, ba, grav); rotations 3-8
// go through so3 exp / log.
__device__ __forceinline__ int state_off(int k) { return k < 3 ? k : k + 2; }

// The control-block doubles a filter step reads, as one compact list:
// x, x_prop | P | P11^-1 (D x D) | G (24 x D) | dx_new.  ctl_src gives the
// double offset inside IkfCtl, ctl_dst the LDS home.
template <int D>
struct CtlList {
  static constexpr int nX = 2 * kStateD, nP = 576, nI = D * D, nG = 24 * D, nD = 24;
  static constexpr int total = nX + nP + nI + nG + nD;
};
template <int D>
__device__ __forceinline__ int ctl_src(int e) {
  using CL = CtlList<D>;
  constexpr int oP = (int)(offsetof(IkfCtl, P) / sizeof(double));
  constexpr int oI = (int)(offsetof(IkfCtl, P11i) / sizeof(double));
  constexpr int oG = (int)(offsetof(IkfCtl, G) / sizeof(double));
  constexpr int oD = (int)(offsetof(IkfCtl, dxn) / sizeof(double));
  if (e < CL::nX) return e;
  e -= CL::nX;
  if (e < CL::nP) return oP + e;
  e -= CL::nP;
  if (e < CL::nI) return oI + e;
  e -= CL::nI;
  if (e < CL::nG) return oG + e;
  return oD + (e - CL::nG);
}
template <int D>
__device__ __forceinline__ double& ctl_dst(StepLds& L, int e) {
  using CL = CtlList<D>;
  if (e < CL::nX) return reinterpret_cast<double*>(&L.x)[e];
  e -= CL::nX;
  if (e < CL::nP) return L.P[e];
  e -= CL::nP;
  if (e < CL::nI) return L.P11i[e];
  e -= CL::nI;
  if (e < CL::nG) return L.G[e];
  return L.dxn[e - CL::nG];
}

// One round trip: nrows doubles of pass sums (sc1 loads: written by other
// workgroups of this launch, or plain ones written before it) into rows_lds,
// and the control block from src into LDS (kept in HBM at ctl on the first
// pass of an update, whose src is the caller's mapped host block).  Every
// load is issued before the first LDS store.  All threads call it.
template <int NT, int D, int NROWS>
__device__ __forceinline__ void step_load(StepLds& L, double* rows_lds, const double* rows, bool rows_sc1,
                                          const IkfCtl* src, IkfCtl* ctl) {
  constexpr int kR = (NROWS + NT - 1) / NT;
  constexpr int nC = CtlList<D>::total, kC = (nC + NT - 1) / NT;
  const int t = threadIdx.x;
  const bool first = src != ctl;
  const gdouble* gc = (const gdouble*)(const double*)src;
  double rv[kR], cv[kC];
#pragma unroll
  for (int u = 0; u < kR; ++u) {
    const int e = t + u * NT;
    rv[u] = e < NROWS ? (rows_sc1 ? ld_sc1(rows + e) : ((const gdouble*)rows)[e]) : 0.0;
  }
#pragma unroll
  for (int u = 0; u < kC; ++u) {
    const int e = t + u * NT;
    cv[u] = e < nC ? (first ? ld_sys(reinterpret_cast<const double*>(src) + ctl_src<D>(e)) : gc[ctl_src<D>(e)])
                   : 0.0;
  }
  typedef __attribute__((address_space(1))) int32_t gint;
  const int32_t fl = t < 8 ? (first ? (int32_t)ld_sys_u32(reinterpret_cast<const uint32_t*>(&src->converge) + t)
                                    : ((const gint*)(const int32_t*)&src->converge)[t])
                           : 0;
#pragma unroll
  for (int u = 0; u < kR; ++u) {
    const int e = t + u * NT;
    if (e < NROWS) rows_lds[e] = rv[u];
  }
#pragma unroll
  for (int u = 0; u < kC; ++u) {
    const int e = t + u * NT;
    if (e < nC) {
      ctl_dst<D>(L, e) = cv[u];
      if (first) reinterpret_cast<double*>(ctl)[ctl_src<D>(e)] = cv[u];  // keep it in HBM
    }
  }
  if (t < 8) L.fl[t] = fl;
  if (first && t == 0) ctl->singular = 0;
}

// The pass's total (fixed order: super rows 0..7) and M = H^T H / R, H^T h / R
// from L.sup; threads < 91.  Followed by a barrier in the caller.
__device__ __forceinline__ void step_totals(StepLds& L, double R) {
  const int t = threadIdx.x;
  if (t < SLIO_NPROD) {
    double v = L.sup[0][t];
#pragma unroll
    for (int q = 1; q < SLIO_NSUPER; ++q) v = v + L.sup[q][t];
    L.tot[t] = v;
    if (t < SLIO_NHTH)
      L.Mt[t] = v / R;
    else if (t < SLIO_NHTH + 12)
      L.hR[t - SLIO_NHTH] = v / R;
  }
}

// 1 / sqrt(d): hardware estimate + two Newton steps (< 1 ulp), far shorter
// than IEEE sqrt followed by IEEE division
__device__ __forceinline__ double rsqrt_nr(double d) {
  double inv = __builtin_amdgcn_rsq(d);
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const double r = fma(-(d * inv), inv, 1.0);
    inv = fma(0.5 * inv, r, inv);
  }
  return inv;
}

// x [+] dx of a rotation on the device: Sophus SO3::exp (the small-angle
// Taylor branch of so3_exp for the IKF's increments) and the quaternion
// product, normalised by one reciprocal square root (rsqrt_nr) instead of
// sqrt and four divisions -- the same values to rounding, a much shorter
// dependent chain.  Falls back to so3_exp beyond the Taylor range.
__device__ __forceinline__ Quat qnormalized_fast(const Quat& q) {
  const double inv = rsqrt_nr(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
  return Quat{q.w * inv, q.x * inv, q.y * inv, q.z * inv};
}
__device__ __forceinline__ Quat so3_boxplus_dev(const Quat& q, const double om[3]) {
  const double theta2 = om[0] * om[0] + om[1] * om[1] + om[2] * om[2];
  Quat e;
  if (theta2 < kSmallEps * kSmallEps) {
    // Sophus' small-angle branch: cos(theta / 2) is 1.0 in double below
    // 1e-10 (a rotation the update leaves alone, e.g. R_LI without
    // extrinsic estimation)
    const double t4 = theta2 * theta2;
    const double imag = 0.5 - 0.0208333 * theta2 + 0.000260417 * t4;
    e = qnormalized_fast(Quat{1.0, imag * om[0], imag * om[1], imag * om[2]});
  } else if (theta2 < 0.0625) {  // half-angle < 0.125
    const double u = 0.25 * theta2;
    const double sh = 1.0 + u * (-1.0 / 6 + u * (1.0 / 120 + u * (-1.0 / 5040 + u * (1.0 / 362880 +
                      u * (-1.0 / 39916800 + u * (1.0 / 6227020800.0))))));
    const double real = 1.0 + u * (-0.5 + u * (1.0 / 24 + u * (-1.0 / 720 + u * (1.0 / 40320 +
                        u * (-1.0 / 3628800 + u * (1.0 / 479001600.0))))));
    const double imag = 0.5 * sh;
    e = qnormalized_fast(Quat{real, imag * om[0], imag * om[1], imag * om[2]});
  } else {
    e = so3_exp(om);
  }
  return qnormalized_fast(qmul(q, e));
}

// One filter step of update_iterated_dyn_share_modified (esekfom.hpp:303-344)
// by one workgroup of NT threads, in information form restricted to the D
// columns H can have non-zero (6 without extrinsic estimation, 12 with):
//   K_front[:, :D] = (P^-1 + E^T M E)^-1 E^T = G S^-1,  G = P[:, :D] P_DD^-1,
//   S = P_DD^-1 + M,  M = H^T H / R   (push-through identity, P_DD = P[:D, :D])
//   dx = K h + (K H - I) dx_new = G S^-1 w - dx_new,  w = H^T h / R + M dx_new[:D]
// so a pass is one D x D Cholesky solve; the final pass forms
// K H [:, :D] = G S^-1 M and P = (I - K H) P (esekfom.hpp:341-343).  P_DD^-1
// and G are fixed during an update (P changes only at its end) and come from
// the host.  Algebraically the host filter_step (slio_ikf.cpp); rounding
// differs.  On entry L holds tot / Mt / hR (step_totals) and the control
// block; ctl (HBM) receives the new iterate and flags, hblk (the caller's
// mapped host block) x, P and the flags when the update ends.  All threads
// of the workgroup call this.
template <int NT, int D, bool WT = false>
__device__ __forceinline__ void ikf_step(IkfCtl* ctl, IkfCtl* hblk, double R, int i, int maxit,
                                         StepLds& L) {
  // WT (persistent update): the control block is written through -- the
  // launch's next pass reads it from any XCD -- and LM read back the same way
  auto stD = [](double* p, double v) {
    if (WT)
      st_sc1(p, v);
    else
      *p = v;
  };
  auto stU = [](void* p, uint32_t v) {
    if (WT)
      st_sc1_u32(reinterpret_cast<uint32_t*>(p), v);
    else
      *reinterpret_cast<uint32_t*>(p) = v;
  };
  static_assert(NT >= 256, "filter step: at least four wavefronts");
  static_assert(D == 6 || D == 12, "filter step: D is 6 or 12");
  const int t = threadIdx.x;
  SSTAMP(5);
  const int64_t m = (int64_t)llround(L.tot[SLIO_NPROD - 1]);
  const bool valid = m >= 1;
  // wave 0: the whole pass-to-pass chain, no workgroup barrier.  The D x D
  // Cholesky solve runs on every lane with uniform operands (LDS broadcast
  // reads): no cross-lane traffic on the critical path.
  double a[D][D];  // lower triangle: S, then its factor L (rows)
  double invd[D];
#pragma unroll
  for (int r = 0; r < D; ++r) {
    invd[r] = 0.0;
#pragma unroll
    for (int c = 0; c < D; ++c) a[r][c] = 0.0;
  }
  if (t < 64) {
    bool ok = true, big = false;
    if (valid) {
#pragma unroll
      for (int r = 0; r < D; ++r)
#pragma unroll
        for (int c = 0; c <= r; ++c) a[r][c] = L.P11i[r * D + c] + L.Mt[tri_index(c, r)];
      double y[D];
#pragma unroll
      for (int r = 0; r < D; ++r) {
        double s2 = 0.0;
#pragma unroll
        for (int k = 0; k < D; ++k) s2 = fma(L.Mt[r <= k ? tri_index(r, k) : tri_index(k, r)], L.dxn[k], s2);
        y[r] = L.hR[r] + s2;  // w
      }
      SSTAMP(9);
      // S = L L^T, right-looking (column j scaled by 1 / L[j][j]), then
      // L z = w, L^T y = z -- the host filter_step's order of operations
#pragma unroll
      for (int j = 0; j < D; ++j) {
        const double d = a[j][j];
        ok = ok && (d > 0.0);
        const double inv = rsqrt_nr(d);
        invd[j] = inv;
        a[j][j] = d * inv;
#pragma unroll
        for (int r = j + 1; r < D; ++r) a[r][j] = a[r][j] * inv;
#pragma unroll
        for (int k = j + 1; k < D; ++k)
#pragma unroll
          for (int r = k; r < D; ++r) a[r][k] = fma(-a[r][j], a[k][j], a[r][k]);
      }
#pragma unroll
      for (int j = 0; j < D; ++j) {
        const double zj = y[j] * invd[j];
        y[j] = zj;
#pragma unroll
        for (int r = j + 1; r < D; ++r) y[r] = fma(-a[r][j], zj, y[r]);
      }
#pragma unroll
      for (int j = D - 1; j >= 0; --j) {
        const double yj = y[j] * invd[j];
        y[j] = yj;
#pragma unroll
        for (int r = 0; r < j; ++r) y[r] = fma(-a[j][r], yj, y[r]);
      }
      SSTAMP(10);
      if (ok) {
        // dx = G y - dx_new, |dx| > epsi (esekfom.hpp:17, 325-331): lane q < 24
        // forms component q (one dot product, its D LDS reads in flight); the
        // rotation lanes 32 / 33 take their 3 components from lanes 3..5 / 6..8
        const int lane = t;
        const int nq = lane < 24 ? 1 : ((lane == 32 || lane == 33) ? 3 : 0);
        double dq[3] = {0.0, 0.0, 0.0};
        {
          const int q = lane < 24 ? lane : 0;
          double s2 = 0.0;
#pragma unroll
          for (int k = 0; k < D; ++k) s2 = fma(L.G[q * D + k], y[k], s2);
          dq[0] = s2 - L.dxn[q];
        }
        {
          const int base = lane == 33 ? 6 : 3;  // (every lane shuffles; 32 / 33 keep theirs)
          const double r0 = __shfl(dq[0], base, 64), r1 = __shfl(dq[0], base + 1, 64),
                       r2 = __shfl(dq[0], base + 2, 64);
          if (lane == 32 || lane == 33) {
            dq[0] = r0;
            dq[1] = r1;
            dq[2] = r2;
          }
        }
        big = __ballot(lane < 24 && fabs(dq[0]) > 0.001) != 0;
        SSTAMP(11);
        // x [+] dx (esekfom.hpp:59-73): vector blocks on lanes 0..23, the
        // two rotations on lanes 32 / 33
        if (lane < 24) {
          if (lane < 3 || lane >= 9) {
            double* xs = reinterpret_cast<double*>(&L.x);
            xs[state_off(lane)] = xs[state_off(lane)] + dq[0];
          }
        } else if (nq == 3) {
          double* q = lane == 33 ? L.x.rli : L.x.rot;
          const Quat rq = so3_boxplus_dev(Quat{q[0], q[1], q[2], q[3]}, dq);
          q[0] = rq.w;
          q[1] = rq.x;
          q[2] = rq.y;
          q[3] = rq.z;
        }
        SSTAMP(12);
      }
    }
    if (t == 0) {
      L.ok = ok ? 1 : 0;
      int32_t* f = L.fl;
      int fin = 0;
      if (ok) {
        f[F_PASSES] += 1;
        f[F_SEARCHES] += f[F_SEARCH];
        if (valid) {
          f[F_VALID] += 1;
          if (f[F_MODE] == SLIO_MODE_FIXED) {
            fin = i == maxit - 1;
            f[F_SEARCH] = 1;
          } else {
            const int conv = big ? 0 : 1;
            f[F_CONV] = conv;
            if (conv) f[F_T] += 1;
            if (!f[F_T] && i == maxit - 2) f[F_CONV] = 1;
            fin = (f[F_T] > 1 || i == maxit - 1);
            f[F_SEARCH] = f[F_CONV];
          }
        } else if (i == maxit - 1) {
          // reference: the loop ends without the P update; fixed mode applies
          // the last valid pass's K H if there was one
          fin = (f[F_MODE] == SLIO_MODE_FIXED && f[F_VALID] > 0);
        }
        if (fin || i == maxit - 1) f[F_DONE] = 1;
      } else {
        f[F_DONE] = 1;  // non-positive pivot: the update stops (singular)
      }
      L.s_final = fin;
    }
    SSTAMP(13);
    SSTAMP(14);
  } else if (valid) {
    // waves 1..3, beside wave 0's chain: keep this pass's M for a final pass
    // without effective points (its factor is formed again from P_DD^-1 + M)
    for (int e = t - 64; e < SLIO_NHTH; e += NT - 64) stD(&ctl->LM[144 + e], L.Mt[e]);
  }
  __syncthreads();
  SSTAMP(6);
  if (!L.ok) {
    if (t == 0) {
      stU(&ctl->singular, 1u);
      stU(&ctl->done, 1u);
      hblk->singular = 1;
      hblk->done = 1;
      __threadfence_system();
      __hip_atomic_store(&hblk->published, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    return;
  }
  const bool fin = L.s_final != 0;
  constexpr int kPer = (576 + NT - 1) / NT;
  double pn[kPer];
  if (fin) {
    // P = (I - K H) P with K H [:, :D] = G S^-1 M (esekfom.hpp:341-343)
    if (t < 64) {
      if (!valid) {
        // the last valid pass's M (fixed mode: one exists, or the update
        // would not end here with a P update); its factor, formed again
        for (int e = t; e < SLIO_NHTH; e += 64) L.Mt[e] = WT ? ld_sc1(&ctl->LM[144 + e]) : ctl->LM[144 + e];
        wave_fence();
#pragma unroll
        for (int r = 0; r < D; ++r)
#pragma unroll
          for (int c = 0; c <= r; ++c) a[r][c] = L.P11i[r * D + c] + L.Mt[tri_index(c, r)];
#pragma unroll
        for (int j = 0; j < D; ++j) {
          const double d = a[j][j];
          const double inv = rsqrt_nr(d);
          invd[j] = inv;
          a[j][j] = d * inv;
#pragma unroll
          for (int r = j + 1; r < D; ++r) a[r][j] = a[r][j] * inv;
#pragma unroll
          for (int k = j + 1; k < D; ++k)
#pragma unroll
            for (int r = k; r < D; ++r) a[r][k] = fma(-a[r][j], a[k][j], a[r][k]);
        }
      }
      if (t < D) {
        // column t of Z = S^-1 M = L^-T L^-1 M
        const int cc = t;
        double zc[D];
#pragma unroll
        for (int j = 0; j < D; ++j) {
          double s2 = L.Mt[j <= cc ? tri_index(j, cc) : tri_index(cc, j)];
#pragma unroll
          for (int k = 0; k < j; ++k) s2 = fma(-a[j][k], zc[k], s2);
          zc[j] = s2 * invd[j];
        }
#pragma unroll
        for (int j = D - 1; j >= 0; --j) {
          double s2 = zc[j];
#pragma unroll
          for (int k = j + 1; k < D; ++k) s2 = fma(-a[k][j], zc[k], s2);
          zc[j] = s2 * invd[j];
        }
#pragma unroll
        for (int j = 0; j < D; ++j) L.zk.Z[j * D + cc] = zc[j];
      }
    }
    __syncthreads();
    for (int e = t; e < 24 * D; e += NT) {
      const int r = e / D, cc = e - r * D;
      double s2 = 0.0;
#pragma unroll
      for (int k = 0; k < D; ++k) s2 = fma(L.G[r * D + k], L.zk.Z[k * D + cc], s2);
      L.zk.K[e] = s2;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int e = t + u * NT;
      if (e < 576) {
        const int r = e / 24, cc = e - r * 24;
        double s2 = 0.0;
#pragma unroll
        for (int k = 0; k < D; ++k) s2 = fma(L.zk.K[r * D + k], L.P[k * 24 + cc], s2);
        pn[u] = L.P[e] - s2;
        stD(&ctl->P[e], pn[u]);
      }
    }
  }
  SSTAMP(7);
  {
    const double* xs = reinterpret_cast<const double*>(&L.x);
    double* xd = reinterpret_cast<double*>(&ctl->x);
    for (int e = t; e < kStateD; e += NT) stD(xd + e, xs[e]);
    // the next pass's pose, in the slot of the passes completed (L.fl: after
    // this step)
    if (t >= 64 && t < 96) stD(&ctl->pose[L.fl[F_PASSES] & (kPoseSlots - 1)][t - 64], pose_elem(L.x, t - 64));
  }
  if (t < 8) stU(reinterpret_cast<uint32_t*>(&ctl->converge) + t, (uint32_t)L.fl[t]);
  if (t == 0) {
    if (WT)
      __hip_atomic_store((guint64*)(uint64_t*)&ctl->last_m, (uint64_t)m, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    else
      ctl->last_m = m;
  }
  if (L.fl[F_DONE]) {
    // the update ends: x, P and the flags to the caller's mapped host block
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int e = t + u * NT;
      if (e < 576) hblk->P[e] = fin ? pn[u] : L.P[e];
    }
    const double* xs = reinterpret_cast<const double*>(&L.x);
    double* xd = reinterpret_cast<double*>(&hblk->x);
    for (int e = t; e < kStateD; e += NT) xd[e] = xs[e];
    if (t < 8) (&hblk->converge)[t] = L.fl[t];
    if (t == 0) {
      hblk->last_m = m;
      hblk->singular = 0;
    }
    // every thread's stores complete, then ONE system-scope release (the L2
    // write-back of the fence covers the whole workgroup's stores) and the
    // word the host polls for (a fence in each of the 256 threads cost ~2 us)
    drain_stores();
    __syncthreads();
    if (t == 0) {
      __threadfence_system();
      __hip_atomic_store(&hblk->published, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  SSTAMP(8);
}

// fixed-order product phase: rows[SLIO_CHUNK][kRow] in LDS -> chunk partial.
// Thread (half, k) sums row[a_k] * row[b_k] over its rows with 4 interleaved
// accumulators (rows r = 0,1,2,3 mod 4) to break the dependent fp64 add chain;
// the accumulators and halves are then combined in a fixed order.
template <int NT>
__device__ __forceinline__ double chunk_products_v(const double (*rows)[kRow], double (*part)[SLIO_NPROD]) {
  constexpr int kSplit = NT / 128;                 // row halves handled in parallel
  constexpr int kRowsPer = SLIO_CHUNK / kSplit;
  const int t = threadIdx.x;
  const int half = t >> 7, kk = t & 127;
  if (kk < SLIO_NPROD && half < kSplit) {
    const int a = c_pa[kk], b = c_pb[kk];
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    const int r0 = half * kRowsPer;
#pragma unroll 2
    for (int r = r0; r < r0 + kRowsPer; r += 4) {
      s0 = s0 + rows[r][a] * rows[r][b];
      s1 = s1 + rows[r + 1][a] * rows[r + 1][b];
      s2 = s2 + rows[r + 2][a] * rows[r + 2][b];
      s3 = s3 + rows[r + 3][a] * rows[r + 3][b];
    }
    part[half][kk] = (s0 + s1) + (s2 + s3);
  }
  __syncthreads();
  double s = 0.0;
  if (t < SLIO_NPROD) {
    s = part[0][t];
#pragma unroll
    for (int h = 1; h < kSplit; ++h) s = s + part[h][t];
  }
  return s;
}
template <int NT>
__device__ __forceinline__ void chunk_products(const double (*rows)[kRow], double (*part)[SLIO_NPROD],
                                               double* __restrict__ out, bool sc1 = false) {
  const double s = chunk_products_v<NT>(rows, part);
  const int t = threadIdx.x;
  if (t < SLIO_NPROD) {
    if (sc1)
      st_sc1(out + t, s);  // read by another workgroup of this launch
    else
      out[t] = s;
  }
}


// The same 91 chunk sums on the matrix cores: they are entries of the Gram
// matrix R^T R of the chunk's 128 x 14 row block R (H^T H, H^T h and m =
// rows[:, 13] . rows[:, 13]), one 16 x 16 f64 tile with the columns
// zero-padded.  Wave w forms R_w^T R_w of rows 32w..32w+31 in 8 k-steps of
// v_mfma_f64_16x16x4_f64 (A = R^T and B = R take the same operand: lane l
// holds R[k0 + (l >> 4)][l & 15]; D: col = l & 15, row = (l >> 4) + 4 reg),
// writes its tile over its own rows in LDS, and thread k < 91 adds the four
// tiles in a fixed order ((w0 + w1) + (w2 + w3)).  Deterministic, so chunk
// partials stay the same for any rank count; different rounding from
// chunk_products (rtol ~1e-16 of the sums).
typedef double f64x4 __attribute__((ext_vector_type(4)));
template <int NT>
__device__ __forceinline__ double chunk_products_mfma_v(double (*rows)[kRow]) {
  static_assert(NT == 256 && SLIO_CHUNK == 128 && kRow <= 16, "4 waves x 32 rows, 16 columns");
  const int t = threadIdx.x, w = t >> 6, l = t & 63;
  const int col = l & 15, kq = l >> 4;
  f64x4 acc = {0.0, 0.0, 0.0, 0.0};
  double v[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) v[s] = col < kRow ? rows[32 * w + 4 * s + kq][col] : 0.0;
#pragma unroll
  for (int s = 0; s < 8; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(v[s], v[s], acc, 0, 0, 0);
  // (the wave's LDS reads precede these writes in its own LDS queue)
  double* tile = &rows[32 * w][0];
#pragma unroll
  for (int r = 0; r < 4; ++r) tile[(kq + 4 * r) * 16 + col] = acc[r];
  __syncthreads();
  double s2 = 0.0;
  if (t < SLIO_NPROD) {
    const int e = (int)c_pa[t] * 16 + (int)c_pb[t];
    const double* r0 = &rows[0][0];
    constexpr int kW = 32 * kRow;  // doubles between the waves' tiles
    s2 = (r0[e] + r0[kW + e]) + (r0[2 * kW + e] + r0[3 * kW + e]);
  }
  return s2;
}
template <int NT>
__device__ __forceinline__ void chunk_products_mfma(double (*rows)[kRow], double* __restrict__ out,
                                                    bool sc1 = false) {
  const double s2 = chunk_products_mfma_v<NT>(rows);
  const int t = threadIdx.x;
  if (t < SLIO_NPROD) {
    if (sc1)
      st_sc1(out + t, s2);
    else
      out[t] = s2;
  }
}

// Refinement scan of ALL the runs of `mask` (<= 34: 25 rows + 9 right
// segments) by the RL lanes of a group as ONE flattened candidate list: lane
// j fetches the bounds of runs j, j + RL, ... (one round trip for all), the
// group's prefix table goes to LDS (pre / dl, kTab entries), and the lanes
// stride over the whole list with U loads in flight (scan_flat's pipeline),
// a flat position's run found by a 6-step binary search in the table.  The
// lanes share every run's points, so one dense run no longer sets the
// group's time (a per-lane subset of the runs did: ~10 us for one query).
// Every lane of the wavefront calls it (mask = 0: nothing to scan).
constexpr int kTab = 36;
template <int RL, int U>
__device__ __forceinline__ void scan_runs_wide(const float4* __restrict__ pts,
                                               const uint32_t* __restrict__ start, const GridGeom& g,
                                               const RunCtx& rc, uint64_t mask, int rsub,
                                               uint32_t* pre, int32_t* dl, Top5& t) {
  constexpr int W = (34 + RL - 1) / RL;  // runs per lane
  const int nr = __popcll(mask);
  RSTAMP(0);
  int bits[W];
#pragma unroll
  for (int w = 0; w < W; ++w) bits[w] = -1;
  {
    uint64_t m = mask;
    for (int q = 0; m; ++q) {
      const int bit = __ffsll((unsigned long long)m) - 1;
      m &= m - 1;
#pragma unroll
      for (int w = 0; w < W; ++w)
        if (q == rsub + w * RL) bits[w] = bit;
    }
  }
  uint32_t rs[W], len[W];
#pragma unroll
  for (int w = 0; w < W; ++w) {
    uint32_t s0 = 0, e0 = 0;
    if (bits[w] >= 0) {
      int yy, zz, xa, xb;
      run_range(g, rc, bits[w], yy, zz, xa, xb);
      if (xa <= xb) {
        const uint32_t rb = ((uint32_t)zz * (uint32_t)g.dy + (uint32_t)yy) * (uint32_t)g.dx;
        s0 = start[rb + xa];
        e0 = start[rb + xb + 1];
      }
    }
    rs[w] = s0;
    len[w] = e0 - s0;
  }
  // exclusive prefix over the runs in their order j = rsub + w * RL: the
  // runs of the earlier columns w, then those of the earlier lanes of this
  // column (a group scan per column)
  uint32_t own[W], T = 0;
#pragma unroll
  for (int w = 0; w < W; ++w) {
    uint32_t inc = len[w];
#pragma unroll
    for (int d = 1; d < RL; d <<= 1) {
      const uint32_t v = __shfl_up(inc, d, RL);
      if (rsub >= d) inc += v;
    }
    own[w] = T + inc - len[w];
    T += __shfl(inc, RL - 1, RL);
  }
  RSTAMP(1);
  RINFO(T, nr, RL, rc.lim < __int_as_float(0x7f800000));
  static_assert(RL * W >= kTab, "every table entry has an owner lane");
#pragma unroll
  for (int w = 0; w < W; ++w) {
    const int j = rsub + w * RL;
    if (j < kTab) {
      pre[j] = j < nr ? own[w] : 0xFFFFFFFFu;
      dl[j] = (int32_t)(rs[w] - own[w]);
    }
  }
  wave_fence();
  RSTAMP(2);
  if (rsub >= T) RSTAMP(3);
  uint32_t t0 = rsub;
  if (t0 >= T) return;
  auto addr = [&](uint32_t tt) {
    int lo = 0;
#pragma unroll
    for (int st = 32; st; st >>= 1) {
      const int c = lo + st;
      const uint32_t pv = c < kTab ? pre[min(c, kTab - 1)] : 0xFFFFFFFFu;
      lo = pv <= tt ? c : lo;
    }
    return tt + (uint32_t)dl[lo];
  };
  constexpr uint32_t kStep = U * RL;
  uint32_t aA[U], aB[U];
  float4 cA[U], cB[U];
#pragma unroll
  for (int u = 0; u < U; ++u) aA[u] = addr(min(t0 + u * RL, T - 1));
#pragma unroll
  for (int u = 0; u < U; ++u) cA[u] = pts[aA[u]];
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  for (;;) {
    const uint32_t t1 = t0 + kStep, t2 = t1 + kStep;
#pragma unroll
    for (int u = 0; u < U; ++u) aB[u] = addr(min(t1 + u * RL, T - 1));
#pragma unroll
    for (int u = 0; u < U; ++u) cB[u] = pts[aB[u]];
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    consume<RL, U>(t, cA, aA, t0, T, rc.qx, rc.qy, rc.qz);
#pragma unroll
    for (int u = 0; u < U; ++u) aA[u] = addr(min(t2 + u * RL, T - 1));
#pragma unroll
    for (int u = 0; u < U; ++u) cA[u] = pts[aA[u]];
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    consume<RL, U>(t, cB, aB, t1, T, rc.qx, rc.qy, rc.qz);
    if (t2 >= T) break;
    t0 = t2;
  }
  RSTAMP(3);
}

// The pass total and the filter step, by the workgroup that summed the last
// segment row: thread k < 91 loads the 64 segment values of product k (sc1:
// written by other workgroups of this launch) and adds them in registers (8
// super rows, then their ordered total -- the tree step_totals uses); the
// other 165 threads load the control block meanwhile (one round trip, no LDS
// staging of the rows).  CTL_SC1: parts of the block were written in this
// launch (dx_new by block 0 of a fused pass; the whole block by the first
// fused pass's prefetch), so every control load goes past the L2 (sc1).
template <int NT, int D, bool CTL_SC1, bool GROUP = false, bool WT = false>
__device__ __forceinline__ void final_step(StepLds& L, const double* seg_out, double* super_out, IkfCtl* ctl,
                                           const IkfCtl* src, IkfCtl* hblk, double R, int iter, int maxit) {
  const int t = threadIdx.x;
  if (t < SLIO_NPROD) {
    // the 8 super rows: from the 64 segment rows, or (GROUP) the ranks' super
    // rows themselves, formed by the same loop
    double sp[SLIO_NSUPER];
    if constexpr (GROUP) {
#pragma unroll
      for (int ss = 0; ss < SLIO_NSUPER; ++ss) sp[ss] = ld_sc1(seg_out + ss * SLIO_NPROD + t);
    } else {
      double v[kNSeg];
#pragma unroll
      for (int e = 0; e < kNSeg; ++e) v[e] = ld_sc1(seg_out + e * SLIO_NPROD + t);
#pragma unroll
      for (int ss = 0; ss < SLIO_NSUPER; ++ss) {
        double a = v[ss * kSuperSeg];
#pragma unroll
        for (int q = 1; q < kSuperSeg; ++q) a = a + v[ss * kSuperSeg + q];
        sp[ss] = a;
      }
    }
    double a = sp[0];
#pragma unroll
    for (int ss = 1; ss < SLIO_NSUPER; ++ss) a = a + sp[ss];
    L.tot[t] = a;
    if (t < SLIO_NHTH)
      L.Mt[t] = a / R;
    else if (t < SLIO_NHTH + 12)
      L.hR[t - SLIO_NHTH] = a / R;
    // (WT: write-through -- a persistent update's passes write them from
    // different XCDs, whose L2s would write their dirty copies back in any
    // order)
    if (!GROUP)
#pragma unroll
      for (int ss = 0; ss < SLIO_NSUPER; ++ss) {
        if (WT)
          st_sc1(super_out + ss * SLIO_NPROD + t, sp[ss]);
        else
          super_out[ss * SLIO_NPROD + t] = sp[ss];
      }
  } else {
    constexpr int NC = NT - SLIO_NPROD, nC = CtlList<D>::total, kC = (nC + NC - 1) / NC;
    const int tt = t - SLIO_NPROD;
    const bool first = src != ctl;
    const gdouble* gc = (const gdouble*)(const double*)src;
    double cv[kC];
#pragma unroll
    for (int u = 0; u < kC; ++u) {
      const int e = tt + u * NC;
      if (CTL_SC1)
        cv[u] = e < nC ? ld_sc1(reinterpret_cast<const double*>(src) + ctl_src<D>(e)) : 0.0;
      else if (first)
        cv[u] = e < nC ? ld_sys(reinterpret_cast<const double*>(src) + ctl_src<D>(e)) : 0.0;
      else
        cv[u] = e < nC ? gc[ctl_src<D>(e)] : 0.0;
    }
    typedef __attribute__((address_space(1))) int32_t gint;
    int32_t fl = 0;
    if (tt < 8)
      fl = CTL_SC1 ? (int32_t)ld_sc1_u32(reinterpret_cast<const uint32_t*>(&src->converge) + tt)
           : first ? (int32_t)ld_sys_u32(reinterpret_cast<const uint32_t*>(&src->converge) + tt)
                   : ((const gint*)(const int32_t*)&src->converge)[tt];
#pragma unroll
    for (int u = 0; u < kC; ++u) {
      const int e = tt + u * NC;
      if (e < nC) {
        ctl_dst<D>(L, e) = cv[u];
        if (first) reinterpret_cast<double*>(ctl)[ctl_src<D>(e)] = cv[u];  // keep it in HBM
      }
    }
    if (tt < 8) L.fl[tt] = fl;
    if (first && tt == 0) ctl->singular = 0;
  }
  __syncthreads();
  SSTAMP(4);
  if (src == ctl && L.fl[F_DONE]) return;  // the first pass of an update always runs
  ikf_step<NT, D, WT>(ctl, hblk, R, iter, maxit, L);
}

template <int LPQ>
constexpr int search_block() { return LPQ == 1 ? SLIO_CHUNK : kBlock; }

// One point of a non-search pass (esekfom.hpp:138-150 with converge ==
// false): the cached plane and selection of the last search pass, the
// residual gate re-evaluated at this pass's pose (:157-173), the Jacobian row
// (:197-226) into row[kRow] (zeros when not selected).  Shared by k_reuse_pass
// and the reuse branch of a fused pass, so both give the same rows.
__device__ __forceinline__ void reuse_row(const ScanDev& scan, const PoseDev& pose, const PassCfg& cfg,
                                          const PassOut& out, int64_t i, double (&row)[kRow]) {
#pragma unroll
  for (int j = 0; j < kRow; ++j) row[j] = 0.0;
  if (i >= scan.n) return;
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
    st_out(out.sel + i, (uint8_t)(sel ? 1 : 0));
  }
  st_out(out.resid + i, sel ? pd2 : __int_as_float(0x7fc00000));
}

// The chunk's 91 products of the rows in LDS (256 threads): on the matrix
// cores, or the VALU form under SLIO_NO_MFMA; product t in thread t < 91.
__device__ __forceinline__ double chunk_sums_256(double (*rows)[kRow], double (*part)[SLIO_NPROD],
                                                 bool mfma) {
  return mfma ? chunk_products_mfma_v<256>(rows) : chunk_products_v<256>(rows, part);
}

// dx_new = x [-] x_propagated (esekfom.hpp:236-258) of the iterate a
// device-resident pass runs at, for that pass's filter step: formed by block
// 0 of the pass kernel (lanes 0..23 the vector blocks, lanes 32 / 64 the
// two rotations, on different wavefronts) while the pass itself runs, off
// the filter step's critical path.  Needs >= 128 threads.  Stored
// write-through (sc1): a fused pass's filter step reads it in the same launch,
// possibly from another XCD.  SC1: the iterate is read write-through too (a
// persistent update's earlier pass wrote it in the same launch).
template <bool SC1>
__device__ __forceinline__ void ikf_dx_new(IkfCtl* ctl) {
  if (blockIdx.x != 0) return;
  const int t = threadIdx.x;
  auto ld = [](const double* p) { return SC1 ? ld_sc1(p) : *p; };
  if (t < 24) {
    const int k = t;
    if (k < 3 || k >= 9) {
      const double* xs = reinterpret_cast<const double*>(&ctl->x);
      const double* ps = reinterpret_cast<const double*>(&ctl->xprop);
      st_sc1(&ctl->dxn[k], ld(xs + state_off(k)) - ld(ps + state_off(k)));
    }
  } else if (t == 32 || t == 64) {
    const int u = t == 32;
    const double* q1 = u ? ctl->x.rli : ctl->x.rot;
    const double* q2 = u ? ctl->xprop.rli : ctl->xprop.rot;
    double d[3];
    so3_boxminus(Quat{ld(q1), ld(q1 + 1), ld(q1 + 2), ld(q1 + 3)}, Quat{ld(q2), ld(q2 + 1), ld(q2 + 2), ld(q2 + 3)},
                 d);
    st_sc1(&ctl->dxn[3 + 3 * u], d[0]);
    st_sc1(&ctl->dxn[4 + 3 * u], d[1]);
    st_sc1(&ctl->dxn[5 + 3 * u], d[2]);
  }
}

// Fused pass (single rank, device-resident update, the filter step in the
// pass's own launch): what the search workgroups need to finish the pass's
// sums and run its filter step.  Segment row b = 8 s + g of super-chunk s
// sums chunks c0 + g, c0 + g + 8, ... (k_super_sums' order); the workgroup
// that completes a segment's last chunk sums the row, and the one that
// completes the 64th row runs final_step.
struct FuseArgs {
  IkfCtl* ctl;        // the update's control block in HBM
  const IkfCtl* pre;  // first pass: the mapped host block, copied into ctl by block 0 at
                      // the launch's start (its PCIe round trip hidden behind the search),
                      // so the filter step reads HBM (src == ctl); else null
  double* seg_out;    // 64 segment rows
  double* super_out;  // 8 super rows (slio_super_download)
  const IkfCtl* src;  // control block source (ctl: passes after the first)
  IkfCtl* hblk;       // mapped host block
  uint32_t* cnt;      // [0] row arrivals, [4..6] far queue, [kSegCnt + b] chunk arrivals of row b
  double R;
  int iter, maxit;
  int64_t C;          // chunks of the scan
  // fused group pass (slio_group_ikf_update, ranks sharing a device): this
  // rank's segment rows (64 / ranks) and first super-chunk; the group's super
  // rows and arrival counter (rank 0's); null gsup: a single rank
  int nrows, s0, granks;
  double* gsup;
  uint32_t* garrive;     // [0] the ranks' arrivals; [2..3] gflag (u64): (seq << 32) | done << 31 | passes
  int32_t gseq;          // the update's sequence number
  // persistent update (k_update_persist): 8 replicas (one per XCD, 128 B
  // apart) of the flag (gseq << 32) | done << 31 | passes its filter step
  // publishes after each pass; null otherwise
  uint64_t* goflag;
  // device-side waits (k_update_persist): give up after this many 100 MHz
  // ticks (0: 1 s), raising the mapped host block's timeout word
  uint64_t wait_ticks;
};
constexpr int kGoFlagStride = 16;  // uint64 words between the replicas
constexpr int kSegCnt = 16;
constexpr int kCountWords = kSegCnt + kNSeg;
constexpr int kKcCount = 8;  // count[8..9]: certified / searched queries (slio_debug_knn_cert)

// the segment row of chunk c (single rank) and its number of chunks
__device__ __forceinline__ int seg_of_chunk(int64_t C, int64_t c, int64_t& lim) {
  int s = 0;
#pragma unroll
  for (int q = 1; q < SLIO_NSUPER; ++q) s = super_lo(C, q) <= c ? q : s;
  const int64_t c0 = super_lo(C, s), c1 = super_lo(C, s + 1);
  const int g = (int)((c - c0) % kSuperSeg);
  lim = (c1 - c0 - g + kSuperSeg - 1) / kSuperSeg;
  return s * kSuperSeg + g;
}

// The first fused pass: block 0 copies the control list (x, x_prop, P,
// P_DD^-1, G, dx_new) and the flags from the caller's mapped host block into
// the HBM block, write-through, at the start of the launch; its stores drain
// before its chunk's arrival, so the filter step (after every arrival) reads
// them from HBM (sc1) instead of over PCIe (measured: the staging step of the
// first pass took 5.7 us against 2.4 us for the later passes).
template <int D>
__device__ __forceinline__ void prefetch_ctl(const IkfCtl* __restrict__ hsrc, IkfCtl* __restrict__ ctl) {
  constexpr int nC = CtlList<D>::total;
  const double* hs = reinterpret_cast<const double*>(hsrc);
  double* cd = reinterpret_cast<double*>(ctl);
  for (int e = threadIdx.x; e < nC; e += blockDim.x) {
    const int o = ctl_src<D>(e);
    st_sc1(cd + o, ld_sys(hs + o));
  }
  if (threadIdx.x < 8)
    st_sc1_u32(reinterpret_cast<uint32_t*>(&ctl->converge) + threadIdx.x,
               ld_sys_u32(reinterpret_cast<const uint32_t*>(&hsrc->converge) + threadIdx.x));
  if (threadIdx.x == 8) st_sc1_u32(reinterpret_cast<uint32_t*>(&ctl->singular), 0u);
  if (threadIdx.x == 9)
    st_sc1_u32(reinterpret_cast<uint32_t*>(&ctl->seq), ld_sys_u32(reinterpret_cast<const uint32_t*>(&hsrc->seq)));
}

// After the chunk partial is stored (sc1): arrival on the chunk's segment row;
// the last arrival sums the row, and the last row runs the filter step.
// Every thread of the workgroup calls it.
template <int NT, int D, bool WT = false>
__device__ __forceinline__ void fused_tail(StepLds& L, int& bcast, const FuseArgs& fa, IkfCtl* ctl,
                                           const double* chunk_part, int64_t chunk, int iter) {
  const int t = threadIdx.x;
  int64_t lim;
  const int b = seg_of_chunk(fa.C, chunk, lim);
#ifdef SLIO_SOLVE_STAMP
  // the final workgroup's tail: partial issued, segment arrival, row stored,
  // row arrival (g_sstamp[16..19]); the launch's first block start is [20]
  unsigned long long ts[4] = {0, 0, 0, 0};
  if (t == 0) ts[0] = wall_clock64();
#endif
  drain_stores();
  __syncthreads();
  if (t == 0) bcast = (int)arrive(fa.cnt + kSegCnt + b);
  __syncthreads();
#ifdef SLIO_SOLVE_STAMP
  if (t == 0) ts[1] = wall_clock64();
#endif
  if (bcast != (int)lim - 1) return;
  if (t < SLIO_NPROD) {
    const int s = b / kSuperSeg, g = b - s * kSuperSeg;
    const double* p = chunk_part + (super_lo(fa.C, s) + g) * SLIO_NPROD + t;
    constexpr int kJ = 16;  // C2's 100k-point scan has <= 13 chunks per segment: one round trip
    double acc = 0.0;
    for (int64_t j0 = 0; j0 < lim; j0 += kJ) {
      double v[kJ];
#pragma unroll
      for (int j = 0; j < kJ; ++j) v[j] = (j0 + j < lim) ? ld_sc1(p + (j0 + j) * (kSuperSeg * SLIO_NPROD)) : 0.0;
#pragma unroll
      for (int j = 0; j < kJ; ++j) acc = acc + v[j];
    }
    st_sc1(fa.seg_out + b * SLIO_NPROD + t, acc);
  }
  if (t == 0) reset_counter(fa.cnt + kSegCnt + b);
  drain_stores();
  __syncthreads();
#ifdef SLIO_SOLVE_STAMP
  if (t == 0) ts[2] = wall_clock64();
#endif
  if (t == 0) bcast = (int)arrive(fa.cnt);
  __syncthreads();
  if (bcast != fa.nrows - 1) return;
#ifdef SLIO_SOLVE_STAMP
  if (t == 0) {
    ts[3] = wall_clock64();
    for (int k = 0; k < 4; ++k) g_sstamp[16 + k] = ts[k];
    // per pass: the final workgroup's partial issued / last row arrival
    g_sstamp[36 + ((iter + 1) & 3)] = ts[0];
    g_sstamp[32 + ((iter + 1) & 3)] = ts[3];
  }
#endif
  if (t == 0) {
    reset_counter(fa.cnt);
    // the pass's number of far queries (slio_far_queries); queue reset
    st_sc1_u32(fa.cnt + 6, ld_sc1_u32(fa.cnt + 5));
    st_sc1_u32(fa.cnt + 4, 0u);
    st_sc1_u32(fa.cnt + 5, 0u);
  }
  if (!fa.gsup) {
    final_step<NT, D, true, false, WT>(L, fa.seg_out, fa.super_out, ctl, fa.src, fa.hblk, fa.R, iter, fa.maxit);
    if (WT && fa.goflag) {
      // persistent update: the step's control block went out write-through
      // (ikf_step); every wave's stores drained, then the flag the waiting
      // workgroups poll, one replica per XCD
      drain_stores();
      __syncthreads();
      if (t < 8) {
        const uint64_t fl = ((uint64_t)(uint32_t)fa.gseq << 32) | (L.fl[F_DONE] ? 0x80000000ull : 0ull) |
                            (uint64_t)(uint32_t)L.fl[F_PASSES];
        __hip_atomic_store((guint64*)(fa.goflag + t * kGoFlagStride), fl, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  } else {
    // fused group pass: this rank's super rows (its 8 / ranks super-chunks,
    // each the sum of its 8 segment rows in order: k_super_sums' tree) into
    // the group's buffer, write-through and drained, then one arrival on the
    // group's counter; the rank that arrives last runs the filter step on
    // the 8 super rows (the same sums, the same bits as one rank) for the
    // whole group: the ranks' next passes read the group's control block.
    // No arrival word (garrive null): a rank of an all-reduce group
    // (slio_comm_init, a reduce hook, RCCL or the in-device reduce of
    // slio_create_group) -- its super rows and zeros in the other ranks'
    // rows, as k_super_sums leaves them, for the all-reduce and k_ikf_solve
    // that follow the launch.
    const int nsup = SLIO_NSUPER / fa.granks;
    if (t < SLIO_NPROD) {
      for (int k = 0; k < nsup; ++k) {
        const int ss = fa.s0 + k;
        double a = ld_sc1(fa.seg_out + (ss * kSuperSeg) * SLIO_NPROD + t);
#pragma unroll
        for (int q = 1; q < kSuperSeg; ++q) a = a + ld_sc1(fa.seg_out + (ss * kSuperSeg + q) * SLIO_NPROD + t);
        st_sc1(fa.gsup + ss * SLIO_NPROD + t, a);
      }
      if (!fa.garrive)
        for (int ss = 0; ss < SLIO_NSUPER; ++ss)
          if (ss < fa.s0 || ss >= fa.s0 + nsup) st_sc1(fa.gsup + ss * SLIO_NPROD + t, 0.0);
    }
    if (!fa.garrive) return;
    drain_stores();
    __syncthreads();
    if (t == 0) bcast = (int)arrive(fa.garrive);
    __syncthreads();
    if (bcast != fa.granks - 1) return;
    if (t == 0) reset_counter(fa.garrive);
    final_step<NT, D, true, true>(L, fa.gsup, nullptr, ctl, fa.src, fa.hblk, fa.R, iter, fa.maxit);
    // the step's control block (plain stores, possibly on another XCD than
    // the next passes' readers) out to memory, then the flag the ranks'
    // gates poll: (seq, done, passes)
    drain_stores();
    __syncthreads();
    if (t == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint64_t fl = ((uint64_t)(uint32_t)fa.gseq << 32) | (L.fl[F_DONE] ? 0x80000000ull : 0ull) |
                          (uint64_t)(uint32_t)L.fl[F_PASSES];
      __hip_atomic_store((guint64*)(uint64_t*)(fa.garrive + 2), fl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
#ifdef SLIO_SOLVE_STAMP
  if (t == 0) g_sstamp[25 + ((iter + 1) & 3)] = wall_clock64();  // per pass: the filter step's end
#endif
}

// One h_share_model search pass over one 128-point chunk.
// Phase 1 (kNN): LPQ lanes per scan point find the exact 5-NN; results go to
// LDS.  Phase 2 (fit): one lane per point reloads the 5 neighbours (L2-hot),
// runs esti_plane, the residual gate and the Jacobian row, and writes the
// row to LDS.  Phase 3: fixed-order fp64 products -> chunk partial.
// refinement lanes per query by the chunk's number of refining queries: 8
// lanes (one round of 32 queries) up to NT / SLIO_RL8_MAX of them, then 4, then 2
#ifndef SLIO_RL8_MAX
#define SLIO_RL8_MAX 8
#endif
// refinement records of a chunk (alias the Jacobian rows, which the fit phase
// writes only after the refinement)
struct RefLds {
  uint64_t top[SLIO_CHUNK][5];
  float4 q[SLIO_CHUNK];
  uint8_t slot[SLIO_CHUNK];
};
template <int NT>
struct SearchLds {
  union {
    double rows[SLIO_CHUNK][kRow];
    RefLds ref;
  } rr;
  double part[NT / 128][SLIO_NPROD];
  alignas(16) uint32_t nb_pos[SLIO_CHUNK][5];
  alignas(16) float nb_sqd[SLIO_CHUNK][5];  // pointSearchSqDis, stored by the fit phase
  alignas(16) int32_t nb_idx[SLIO_CHUNK][5];  // Nearest_Points ids, for one coalesced store
  float nb_d5[SLIO_CHUNK];
  float4 qw[SLIO_CHUNK];            // the query; .w: its certificate bound G (KC, -2: none written)
  float4 qb[SLIO_CHUNK];            // the body point (the fit phase's copy, loaded by the kNN lanes)
  float4 qpl[SLIO_CHUNK];           // KC: the last pass's plane of the point (loaded with its certificate)
  uint32_t kc_n[2];                 // KC: certified queries, searched queries
  uint32_t kx6[SLIO_CHUNK];         // KC: the 6th of the point's certified set
  uint8_t ksame[SLIO_CHUNK];        // KC: certified in the last pass's order (plane reusable)
  // deferred (far) queries of this chunk and the far workers' scratch
  int far_cnt, ref_cnt;
  uint32_t cost;  // block-row candidates of the chunk's queries (chunk_order)
  uint32_t tab_pre[NT / 16][kTab];  // scan_runs_wide's run tables, one per group
  int32_t tab_dl[NT / 16][kTab];
  float4 far_q[SLIO_CHUNK];
  uint8_t far_slot[SLIO_CHUNK];
  uint32_t far_pre[NT / 64][64], far_beg[NT / 64][64];
};
// a pass's LDS: the search, then (fused pass) the filter step
template <int NT>
union PassLds {
  SearchLds<NT> s;
  StepLds L;
};

// The pass body: the search (or, reuse, the reuse pass's rows), the chunk's
// products and (FUSE) the fused tail.  pose: the pass's pose; DEVPOSE: a
// pass after the first of a device-resident update (certificates, dx_new);
// PERS: a pass of the persistent update, whose control-block reads are
// write-through (the launch's earlier passes wrote it).
template <int LPQ, int U, bool SPHERE, bool DEVPOSE, bool FUSE, int FD, bool PERS>
__device__ __forceinline__ void search_pass_body(PassLds<search_block<LPQ>()>& lds, int& fuse_bcast,
                                                 const MapView& map, const ScanDev& scan, const PoseDev& pose,
                                                 const PassCfg& cfg, const PassOut& out, const FuseArgs& fa,
                                                 bool reuse, int iter) {
  constexpr int NT = search_block<LPQ>();
  // kNN certificates (passes after the first of a device-resident update,
  // 2 lanes per query, 3x3x3 block first): see the certificate below
  constexpr bool KC = DEVPOSE && LPQ == 2 && !SPHERE;
  if (DEVPOSE) ikf_dx_new<PERS>(cfg.ctl);
  constexpr int QPP = NT / LPQ;               // queries per kNN pass
  constexpr int PASSES = SLIO_CHUNK / QPP;    // kNN passes per chunk
  static_assert(SLIO_CHUNK % QPP == 0, "chunk must be a multiple of queries/pass");
  static_assert(NT >= SLIO_CHUNK, "fit phase needs one lane per point");
  auto& rows = lds.s.rr.rows;
  auto& ref = lds.s.rr.ref;
  auto& part = lds.s.part;
  auto& nb_pos = lds.s.nb_pos;
  auto& nb_sqd = lds.s.nb_sqd;
  auto& nb_idx = lds.s.nb_idx;
  auto& nb_d5 = lds.s.nb_d5;
  auto& qw = lds.s.qw;
  auto& far_cnt = lds.s.far_cnt;
  auto& ref_cnt = lds.s.ref_cnt;
  auto& tab_pre = lds.s.tab_pre;
  auto& tab_dl = lds.s.tab_dl;
  auto& far_q = lds.s.far_q;
  auto& far_slot = lds.s.far_slot;
  auto& far_pre = lds.s.far_pre;
  auto& far_beg = lds.s.far_beg;
  int64_t chunk = xcd_chunk(cfg.c_begin, cfg.c_end - cfg.c_begin);
  const int tid = threadIdx.x;
  // a fused pass of the device-resident update runs whichever pass the
  // update wants: a reuse pass (esekfom.hpp:138-150, converge == false) forms
  // its rows here and shares the products and the tail below with the search
  // pass (one copy of the tail in the kernel: a second one, in a branch of
  // its own, cost ~2.5 % of the search pass's time)
  if (reuse) {
    if (tid < SLIO_CHUNK) {
      double row[kRow];
      reuse_row(scan, pose, cfg, out, chunk * SLIO_CHUNK + tid, row);
#pragma unroll
      for (int j = 0; j < kRow; ++j) lds.s.rr.rows[tid][j] = row[j];
    }
    __syncthreads();
  } else {
  if (cfg.perm) {
    // (a permutation of [0, nblk) by construction; the range check only
    // keeps a corrupt order from writing outside the chunk arrays)
    const uint32_t pc = cfg.perm[chunk - cfg.c_begin];
    if (pc < (uint32_t)(cfg.c_end - cfg.c_begin)) chunk = cfg.c_begin + pc;
  }
  const int sub = tid & (LPQ - 1);
  const int grp = tid / LPQ;
  const GridGeom g = map.g;
  const float4* __restrict__ pts = map.pts;
  const uint32_t* __restrict__ start = map.start;
  // this chunk's certificates belong to this update (written by one of its
  // earlier passes): a uniform load
  bool cache_ok = false;
  if constexpr (KC) {
    // (PERS: this workgroup wrote the entry in an earlier pass of the launch;
    // a vector load, not the scalar cache)
    const uint32_t ke = PERS ? __builtin_amdgcn_readfirstlane(ld_sc1_u32(&out.kepoch[chunk])) : out.kepoch[chunk];
    cache_ok = cfg.kc_epoch != 0 && ke == cfg.kc_epoch;
  }
  if (tid == 0) STAMP(0);
  if (tid == 0) {
    far_cnt = 0;
    ref_cnt = 0;
    lds.s.cost = 0;
    if (KC) lds.s.kc_n[0] = lds.s.kc_n[1] = 0;
    if (blockIdx.x == 0 && !cfg.knn_only) *out.pose = pose;
  }
  __syncthreads();

  // ---------------- phase 1: exact 5-NN
  // (no early exit per lane: the refinement below needs the whole wavefront)
  for (int pass = 0; pass < PASSES; ++pass) {
    const int slot = pass * QPP + grp;
    const int64_t i = chunk * SLIO_CHUNK + slot;
    const bool live = i < scan.n;
    float qx = 0.0f, qy = 0.0f, qz = 0.0f;
    // KC: the point's certificate (earlier query + bound) and its 6 positions
    // (the last pass's 5 in order, then the 6th), loaded with the scan point:
    // no dependent round trip
    float4 ka = make_float4(0.0f, 0.0f, 0.0f, -1.0f);
    float4 kpl = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    uint32_t kp[6] = {~0u, ~0u, ~0u, ~0u, ~0u, ~0u};
    if (KC && cache_ok && live) {
      ka = out.kq[i];
#pragma unroll
      for (int j = 0; j < 5; ++j) kp[j] = out.nbr_pos[5 * i + j];
      kp[5] = out.k6[i];
      kpl = out.plane[i];  // (the fit reuses it when the certified 5 keep their order)
    }
    float bx = 0.0f, by = 0.0f, bz = 0.0f;
    if (live) {
      bx = scan.bx[i];
      by = scan.by[i];
      bz = scan.bz[i];
      body_to_world(pose, bx, by, bz, qx, qy, qz);
    }
    Top5 t;
    top5_clear(t);
    const bool finite = live && isfinite(qx) && isfinite(qy) && isfinite(qz) && map.n > 0 &&
                        !far_outside(g, cfg.far_sq, qx, qy, qz);
    int cx = 0, cy = 0, cz = 0, r = 1;
    bool done = !finite;
    bool refine = false;   // exact 5x5x5 refinement wanted (lim = refine bound)
    float lim = 0.0f;
    // kNN certificate (KC).  A full search on the block rows keeps the 6
    // nearest and the smallest squared distance it dropped (Top6M), so every
    // map point outside the 6 lies at squared distance >= G = min(dropped,
    // b1^2) (b1: the block faces' bound) from that query, less a 2e-5
    // relative margin for float rounding -- a bound on the TRUE squared
    // distance.  A later pass of the same update, its query moved by
    // delta <= |q - q_old|, evaluates the 6 (nbr_pos + k6: a certified pass
    // rewrites the same set) at the new query; if (sqrt(G) - delta)^2
    // (1 - 1e-5) exceeds the new 5th squared distance, no point outside the 6
    // can enter the top 5 (its float distance is strictly larger), so the 5
    // smallest keys of the 6 ARE the exact search's result, tie order
    // included (same keys).  Otherwise the query searches.  When the 5 come
    // out in the last pass's order, esti_plane's input is the same and its
    // plane is reused (the fit phase).
    bool reused = false;
    bool same5 = false;    // certified, in the last pass's order
    float kG = -1.0f;      // this search's certificate bound (-1: none)
    uint32_t kx6 = ~0u;    // the 6th position this pass leaves
    if constexpr (KC) {
      // (branch-free up to the gathers, so the certificate loads stay whole)
      const double ex0 = (double)qx - (double)ka.x, ey0 = (double)qy - (double)ka.y,
                   ez0 = (double)qz - (double)ka.z;
      const double dl = sqrt(ex0 * ex0 + ey0 * ey0 + ez0 * ez0) * (1.0 + 1e-9) + 1e-9;
      const double A = sqrt((double)fmaxf(ka.w, 0.0f)) - dl;
      if (cache_ok && finite && ka.w > 0.0f) {
        {
          if (A > 0.0) {
            // the pair's lanes take 3 of the 6 each, then merge (as a search)
            uint32_t ps[3];
#pragma unroll
            for (int j = 0; j < 3; ++j) ps[j] = sub == 0 ? kp[j] : kp[3 + j];
            float4 cc[3];
#pragma unroll
            for (int j = 0; j < 3; ++j) cc[j] = pts[ps[j] != ~0u ? ps[j] : 0u];
            Top5 tr;
            top5_clear(tr);
#pragma unroll
            for (int j = 0; j < 3; ++j) {
              const float ddx = qx - cc[j].x, ddy = qy - cc[j].y, ddz = qz - cc[j].z;
              const float d = (ddx * ddx + ddy * ddy) + ddz * ddz;  // calc_dist, ikd_Tree.cpp:1539-1544
              top5_insert(tr, ps[j] != ~0u ? (((uint64_t)__float_as_uint(d) << 32) | (uint64_t)ps[j]) : kInfKey);
            }
            group_merge<2>(tr);
            if (tr.k[4] != kInfKey &&
                A * A * (1.0 - 1e-5) > (double)__uint_as_float((uint32_t)(tr.k[4] >> 32))) {
              t = tr;
              reused = true;
              done = true;
              same5 = true;
#pragma unroll
              for (int j = 0; j < 5; ++j) same5 = same5 && (uint32_t)tr.k[j] == kp[j];
              // the one of the 6 left out of the 5 (the set stays the same)
#pragma unroll
              for (int j = 0; j < 6; ++j) {
                bool in5 = false;
#pragma unroll
                for (int q = 0; q < 5; ++q) in5 = in5 || (uint32_t)tr.k[q] == kp[j];
                if (!in5) kx6 = kp[j];
              }
            }
          }
        }
      }
    }
    if (finite && !reused) {
      cx = cell_coord(qx, g.ox, g.inv_h);
      cy = cell_coord(qy, g.oy, g.inv_h);
      cz = cell_coord(qz, g.oz, g.inv_h);
      const int ex = max(max(-cx, cx - (g.dx - 1)), 0);
      const int ey = max(max(-cy, cy - (g.dy - 1)), 0);
      const int ez = max(max(-cz, cz - (g.dz - 1)), 0);
      r = max(1, max(ex, max(ey, ez)));
      if (r == 1 && !SPHERE) {
        // (1) the 3x3x3 block around the query cell: 9 runs, one batch
        // (r == 1 also covers query cells one step outside the grid: the
        // block rows exist only for cells inside it)
        if (map.blk && (ex | ey | ez) == 0) {
          const uint32_t rb = ((uint32_t)cz * (uint32_t)g.dy + (uint32_t)cy) * (uint32_t)g.dx;
          uint32_t i0 = rb + max(cx - 1, 0), i1 = rb + min(cx + 1, g.dx - 1) + 1;
          SLIO_BCHK(i0, map.ncells + 1, "bstart0");
          SLIO_BCHK(i1, map.ncells + 1, "bstart1");
          const uint32_t b0 = map.bstart[i0];
          const uint32_t b1 = map.bstart[i1];
#ifdef SLIO_BOUNDS_CHECK
          if (b1 < b0 || (int64_t)b1 > map.nblk)
            printf("slio bounds: block range %u %u nblk %lld\n", b0, b1, (long long)map.nblk);
#endif
          if (KC && cfg.kc_epoch) {
            Top6M tm;
#pragma unroll
            for (int j = 0; j < 6; ++j) tm.k[j] = kInfKey;
            tm.m = __int_as_float(0x7f800000);
            scan_block_rows<LPQ, U>(map.blk, b0, b1 - b0, sub, qx, qy, qz, tm);
            group_merge2(tm);
#pragma unroll
            for (int j = 0; j < 5; ++j) t.k[j] = tm.k[j];
            kx6 = (uint32_t)tm.k[5];
            kG = tm.m;
          } else {
            scan_block_rows<LPQ, U>(map.blk, b0, b1 - b0, sub, qx, qy, qz, t);
            group_merge<LPQ>(t);
          }
          if (sub == 0 && out.chunk_cost) atomicAdd(&lds.s.cost, b1 - b0);
        } else {
          RunCtx rc{cx, cy, cz, qx, qy, qz, 1, 0.0f, 0.0f};
          scan_runs<LPQ, U>(pts, start, g, rc, 0x739c0ull /* rows 6-8, 11-13, 16-18 */, sub, t);
          group_merge<LPQ>(t);
        }
        bool covers;
        const float b1 = outside_bound(g, cx, cy, cz, 1, qx, qy, qz, covers);
        const float d5 = __uint_as_float((uint32_t)(t.k[4] >> 32));
        done = covers || (t.k[4] != kInfKey && b1 > 0.0f && d5 < (b1 * b1) * 0.99999f);
        // the certificate bound: dropped block candidates and the block faces
        // (+inf when the block covers the grid); none off the block rows
        if (KC) kG = (done && kG >= 0.0f) ? fminf(kG, b1 * b1) * (1.0f - 2e-5f) : -1.0f;
        if (!done) {
          // (2) exact refinement (below): every cell of the 5x5x5 cube whose
          // conservative box gap is within the current 5th distance, minus
          // the block already scanned.  When the block held fewer than 5
          // points (e.g. a long-range ground return a metre below the ground
          // at a slightly wrong pose: its block lies under the ground
          // cells) or its 5th distance reaches past the cube, the whole cube
          // is scanned (no limit); the result is exact if its 5th distance
          // then lies within the cube's bound, else the query is deferred
          // to the far queue (3) with that bound.
          bool covers2;
          const float b2 = outside_bound(g, cx, cy, cz, 2, qx, qy, qz, covers2);
#ifdef SLIO_NO_STARVED_REFINE
          refine = t.k[4] != kInfKey && (covers2 || (b2 > 0.0f && d5 < (b2 * b2) * 0.99999f));
#else
          refine = true;
#endif
          lim = (t.k[4] != kInfKey && (covers2 || (b2 > 0.0f && d5 < (b2 * b2) * 0.99999f)))
                    ? d5 * 1.00001f
                    : __int_as_float(0x7f800000);
        }
        r = 2;
#ifndef SLIO_NO_R2_REFINE
      } else if (r == 2 && !SPHERE) {
        // query cell two cells outside the grid (e.g. a long-range ground
        // return below the padded grid at a slightly wrong pose): its 3x3x3
        // block is empty; the 5x5x5 cube is the refinement with no limit,
        // exact if the 5th distance then lies within the cube's bound
        refine = true;
        lim = __int_as_float(0x7f800000);
#endif
      } else if (r == 1) {
        // sphere-first search: (1) cells of the 5x5x5 cube whose box gap^2 <=
        // rho0^2, exact once 5 neighbours lie within rho0; (2) the shell out
        // to the current 5th distance, exact while it stays inside the cube
        RunCtx rc{cx, cy, cz, qx, qy, qz, 3, 0.0f, cfg.radius_sq * 1.00001f};
        bool covers2;
        const float b2 = outside_bound(g, cx, cy, cz, 2, qx, qy, qz, covers2);
        const float cube2 = covers2 ? __int_as_float(0x7f800000) : b2 * b2 * 0.99999f;
        uint64_t mask = sphere_rows(g, rc, rc.lim);
        for (int step = 0; step < 2; ++step) {
          scan_runs<LPQ, U>(pts, start, g, rc, mask, sub, t);
          group_merge<LPQ>(t);
          if (step == 1) {
            done = true;
            break;
          }
          const bool valid = t.k[4] != kInfKey;
          const float d5 = __uint_as_float((uint32_t)(t.k[4] >> 32));
          done = valid && d5 <= cfg.radius_sq && d5 < cube2;
          if (done || !valid || !(d5 < cube2)) break;
          rc.mode = 4;
          rc.lim0 = rc.lim;
          rc.lim = fmaxf(d5 * 1.00001f, rc.lim0);
          const uint64_t rows = sphere_rows(g, rc, rc.lim);
          mask = rows | (rows << 32);
          if (sub != 0) top5_clear(t);  // lane 0 keeps the merged list
        }
        r = 2;
      }
    }
    if (!SPHERE) {
      // (2) the refinement is deferred to the block-wide pass after the
      // fast path: the query's merged list and bound go to LDS
      const uint64_t nrf = __ballot(refine && sub == 0);
      (void)nrf;
      WSTAMP(3, __popcll(nrf));
      if (refine && sub == 0) {
        const int k = atomicAdd(&ref_cnt, 1);
        ref.slot[k] = (uint8_t)slot;
        ref.q[k] = make_float4(qx, qy, qz, lim);
#pragma unroll
        for (int j = 0; j < 5; ++j) ref.top[k][j] = t.k[j];
      }
    }
    // (3) not finished on the fine grid: deferred to the far queue (the
    // group's list is merged: its 5th distance, if any, bounds the search)
    if (!done && !refine && sub == 0) {
      const int k = atomicAdd(&far_cnt, 1);
      far_slot[k] = (uint8_t)slot;
      far_q[k] = make_float4(qx, qy, qz,
                             t.k[4] != kInfKey ? __uint_as_float((uint32_t)(t.k[4] >> 32))
                                               : __int_as_float(0x7f800000));
    }
    WSTAMP(2, __builtin_amdgcn_s_memrealtime());
    // Nearest_Points / pointSearchSqDis for this point, to LDS: the fit phase
    // writes them out (no global stores in the kNN phase, whose workgroup
    // barriers would wait for them)
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      if (j % LPQ == sub && live && done) {
        const uint64_t mk = t.k[j];
        nb_sqd[slot][j] = (mk == kInfKey) ? __int_as_float(0x7f800000)
                                                 : __uint_as_float((uint32_t)(mk >> 32));
        nb_pos[slot][j] = (mk == kInfKey) ? 0xFFFFFFFFu : (uint32_t)mk;
      }
    }
    if (sub == 0) {
      // kNN gate (esekfom.hpp:144-147): 5 neighbours and d5 <= 5
      const float d5 = __uint_as_float((uint32_t)(t.k[4] >> 32));
      nb_d5[slot] = (t.k[4] != kInfKey) ? d5 : __int_as_float(0x7f800000);
      // (KC: a certified query keeps the certificate it was certified by)
      qw[slot] = make_float4(qx, qy, qz, KC ? (reused ? -2.0f : kG) : 0.0f);
      lds.s.qb[slot] = make_float4(bx, by, bz, 0.0f);
      if (KC) lds.s.qpl[slot] = kpl;
      if (KC) {
        lds.s.kx6[slot] = kx6;
        lds.s.ksame[slot] = same5 ? 1 : 0;
      }
    }
    if constexpr (KC) {
      const uint64_t br = __ballot(sub == 0 && live && reused), bs = __ballot(sub == 0 && live && !reused);
      if ((tid & 63) == 0 && cfg.kc_epoch) {
        atomicAdd(&lds.s.kc_n[0], (uint32_t)__popcll(br));
        atomicAdd(&lds.s.kc_n[1], (uint32_t)__popcll(bs));
      }
    }
  }
  if ((tid >> 6) < 4) STAMP(4 + (tid >> 6));  // per-wave end of the fast path
  __syncthreads();
  if (!SPHERE) {
    // (2) the chunk's refinements, spread over the whole workgroup: RL lanes
    // per query (64 when at most 4 refine, else 16) scan the region as one
    // flattened candidate list (scan_runs_wide); with more than 16, 8 lanes
    // per query, each with a share of the runs (measured faster there: one
    // round instead of two).  A wavefront's
    // refinements used to run on that wavefront alone, 8 per round with a
    // per-lane share of the runs, ~10 us a round, so one wave with 30
    // refining queries set the kernel's end.
    const int nref = ref_cnt;
    WSTAMP(0, __builtin_amdgcn_s_memrealtime());
    auto refine_all = [&](auto rl) {
      constexpr int RL = decltype(rl)::value;
      const int lane = tid & 63;
      const int rsub = lane % RL;
      for (int base = (tid >> 6) * (64 / RL); base < nref; base += NT / RL) {
        const int k = base + lane / RL;
        const bool has = k < nref;
        const float4 q = has ? ref.q[k] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        int rx = 0, ry = 0, rz = 0;
        Top5 tr;
        top5_clear(tr);
        uint64_t runs = 0;
        if (has) {
          rx = cell_coord(q.x, g.ox, g.inv_h);
          ry = cell_coord(q.y, g.oy, g.inv_h);
          rz = cell_coord(q.z, g.oz, g.inv_h);
        }
        const RunCtx rq{rx, ry, rz, q.x, q.y, q.z, 2, 0.0f, q.w};
        if (has) {
          const uint64_t rows = sphere_rows(g, rq, rq.lim);
          runs = rows | ((rows & 0x739c0ull) << 32);
        }
        if constexpr (RL >= 16) {
          const int gi = (tid >> 6) * (64 / RL) + lane / RL;
          scan_runs_wide<RL, U>(pts, start, g, rq, runs, rsub, tab_pre[gi], tab_dl[gi], tr);
        } else if (has) {
          // many refining queries: each lane scans its own share of the runs
          // (runs rsub, rsub + RL, ...), one batch of run bounds per lane
          constexpr uint64_t kShare = RL == 8 ? 0x0101010101010101ull
                                              : (RL == 4 ? 0x1111111111111111ull : 0x5555555555555555ull);
          scan_runs<1, U>(pts, start, g, rq, runs & (kShare << rsub), 0, tr);
        }
#ifdef SLIO_REFINE_DPP_MERGE
        group_merge<RL>(tr);
#else
        group_merge_rolled(tr, RL);
#endif
        if (has && rsub == 0) {
#pragma unroll
          for (int j = 0; j < 5; ++j) top5_insert(tr, ref.top[k][j]);
          // exact once the 5th distance lies inside the 5x5x5 cube's bound
          // (always, when the block's own 5th distance did: lim = d5)
          bool cov2;
          const float b2 = outside_bound(g, rx, ry, rz, 2, q.x, q.y, q.z, cov2);
          const float d5n = __uint_as_float((uint32_t)(tr.k[4] >> 32));
          const bool fin = cov2 || (tr.k[4] != kInfKey && b2 > 0.0f && d5n < (b2 * b2) * 0.99999f);
          const int slot = ref.slot[k];
          if (fin) {
#pragma unroll
            for (int j = 0; j < 5; ++j) {
              const uint64_t mk = tr.k[j];
              nb_sqd[slot][j] = (mk == kInfKey) ? __int_as_float(0x7f800000)
                                                       : __uint_as_float((uint32_t)(mk >> 32));
              nb_pos[slot][j] = (mk == kInfKey) ? 0xFFFFFFFFu : (uint32_t)mk;
            }
            nb_d5[slot] = (tr.k[4] != kInfKey) ? d5n : __int_as_float(0x7f800000);
          } else {
            const int f = atomicAdd(&far_cnt, 1);
            far_slot[f] = (uint8_t)slot;
            far_q[f] = make_float4(q.x, q.y, q.z, tr.k[4] != kInfKey ? d5n : __int_as_float(0x7f800000));
          }
        }
      }
    };
    if (nref > 0) {
      if (nref <= NT / 64)
        refine_all(std::integral_constant<int, 64>{});
      else if (nref <= NT / 16)
        refine_all(std::integral_constant<int, 16>{});
      else if (nref <= NT / SLIO_RL8_MAX)
        refine_all(std::integral_constant<int, 8>{});
      else if (nref <= NT / 4)
        refine_all(std::integral_constant<int, 4>{});
      else
        refine_all(std::integral_constant<int, 2>{});
      __syncthreads();
    }
    WSTAMP(1, __builtin_amdgcn_s_memrealtime());
  }
  if (tid == 0) STAMP(1);
  const int nfar = far_cnt;
  if (nfar > 0) {
    // (3) this chunk's deferred queries, one per wavefront on the coarse
    // level (far_search); no other workgroup is involved or waited for
    if (tid == 0)
      __hip_atomic_fetch_add((gu32*)(out.far_ctr + 1), (uint32_t)nfar, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    const int lane = tid & 63;
    for (int k = tid >> 6; k < nfar; k += NT / 64) {
      const float4 q = far_q[k];
      Top5 tf;
      far_search<4>(map, q.x, q.y, q.z, q.w, far_pre[tid >> 6], far_beg[tid >> 6], tf);
      const int slot = far_slot[k];
      uint64_t mk = tf.k[0];
#pragma unroll
      for (int j = 1; j < 5; ++j) mk = (lane == j) ? tf.k[j] : mk;
      if (lane < 5) {
        nb_sqd[slot][lane] = (mk == kInfKey) ? __int_as_float(0x7f800000)
                                                    : __uint_as_float((uint32_t)(mk >> 32));
        nb_pos[slot][lane] = (mk == kInfKey) ? 0xFFFFFFFFu : (uint32_t)mk;
      }
      if (lane == 0)
        nb_d5[slot] = (tf.k[4] != kInfKey) ? __uint_as_float((uint32_t)(tf.k[4] >> 32))
                                           : __int_as_float(0x7f800000);
    }
    __syncthreads();
  }

  // ---------------- phase 2: plane fit, residual gate, Jacobian row
  // (lanes 0..127, two of the four wavefronts; spreading the fit over the
  // first lane of each query's pair, all four wavefronts, measured slower:
  // 25.0k vs 26.0k IKF it/s, the fit's instructions issue twice as often)
  if (tid < SLIO_CHUNK) {
    const int slot = tid;
    const int64_t i = chunk * SLIO_CHUNK + slot;
    double row[kRow];
#pragma unroll
    for (int j = 0; j < kRow; ++j) row[j] = 0.0;
    if (i < scan.n) {
      const float d5 = nb_d5[slot];
      bool sel = !(d5 > cfg.max_sqd);   // +inf when fewer than 5 map points
      float abcd[4] = {__int_as_float(0x7fc00000), __int_as_float(0x7fc00000),
                       __int_as_float(0x7fc00000), __int_as_float(0x7fc00000)};
      float pd2 = __int_as_float(0x7fc00000);
      const float4 q = qw[slot];
      FSTAMP(0, false);
      const float4 qb = lds.s.qb[slot];
      const float bx = qb.x, by = qb.y, bz = qb.z;
      // KC: certified with the last pass's 5 in the same order -- the same
      // esti_plane input, so its result is reused: the plane when it had one,
      // and its rejection (the kPlaneRejected NaN the fit stores when
      // esti_plane returns false: 9 % of C2's points, in 82 % of the fit's
      // wavefronts, which all used to rerun the QR in every certified pass)
      bool rp = false, rf = false;
      float4 cpl = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      if constexpr (KC) {
        if (lds.s.ksame[slot]) {
          cpl = lds.s.qpl[slot];
          rp = isfinite(cpl.x) && isfinite(cpl.y) && isfinite(cpl.z) && isfinite(cpl.w);
          rf = __float_as_uint(cpl.x) == kPlaneRejected;
        }
      }
      // the 5 neighbours: coordinates for the fit, map index for
      // Nearest_Points (-1 when the map has fewer than 5 points)
      float nb[5][3];
#pragma unroll
      for (int j = 0; j < 5 && !rp && !rf; ++j) {
        const uint32_t ps = nb_pos[slot][j];
        float4 c = make_float4(0.0f, 0.0f, 0.0f, __int_as_float(-1));
#ifdef SLIO_BOUNDS_CHECK
        if (ps != 0xFFFFFFFFu && ps >= map.n) {
          printf("slio bounds: nb_pos %u n %lld block %d slot %d j %d\n", ps, (long long)map.n,
                 (int)blockIdx.x, slot, j);
          continue;
        }
#endif
        if (ps != 0xFFFFFFFFu) c = pts[ps];
        nb[j][0] = c.x;
        nb[j][1] = c.y;
        nb[j][2] = c.z;
        nb_idx[slot][j] = (int32_t)__float_as_uint(c.w);
      }
      FSTAMP(1, true);
      if (cfg.knn_only) sel = false;
      if (sel && rp) {
        abcd[0] = cpl.x;
        abcd[1] = cpl.y;
        abcd[2] = cpl.z;
        abcd[3] = cpl.w;
        sel = residual_gate(abcd, q.x, q.y, q.z, bx, by, bz, pd2);
      } else if (sel && rf) {
        sel = false;
        abcd[0] = __uint_as_float(kPlaneRejected);
      } else if (sel) {
        float pl[4];
        sel = esti_plane_dev(nb, cfg.plane_thr, pl);
        if (sel) {
#pragma unroll
          for (int j = 0; j < 4; ++j) abcd[j] = pl[j];
          sel = residual_gate(abcd, q.x, q.y, q.z, bx, by, bz, pd2);
        } else {
          abcd[0] = __uint_as_float(kPlaneRejected);  // (a NaN: the plane output stays NaN)
        }
      }
      FSTAMP(2, false);
      st_out(out.plane + i, make_float4(abcd[0], abcd[1], abcd[2], abcd[3]));
      st_out(out.sel + i, (uint8_t)(sel ? 1 : 0));
      st_out(out.resid + i, sel ? pd2 : __int_as_float(0x7fc00000));
      if constexpr (KC) {
        // this search's certificate: the query and G (its 5 go to nbr_pos),
        // and the 6th (a certified pass's: the one of the 6 left out)
        if (cfg.kc_epoch) {
          if (q.w != -2.0f) st_out(out.kq + i, q);
          st_out(out.k6 + i, lds.s.kx6[slot]);
        }
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
    FSTAMP(3, false);
#pragma unroll
    for (int j = 0; j < kRow; ++j) rows[slot][j] = row[j];
    FSTAMP(4, true);
  }
  __syncthreads();
  if (tid == 0) STAMP(2);
  if (tid == 0 && out.chunk_cost)
    out.chunk_cost[chunk - cfg.c_begin] = lds.s.cost + 256u * (uint32_t)ref_cnt + 1024u * (uint32_t)nfar;
  if constexpr (KC) {
    if (tid == 0 && cfg.kc_epoch) {
      // every live query of the chunk searched (and wrote its entry) when the
      // chunk's entries were another update's
      if (!cache_ok) out.kepoch[chunk] = cfg.kc_epoch;
      if (out.kc_count) {
        atomicAdd(out.kc_count, lds.s.kc_n[0]);
        atomicAdd(out.kc_count + 1, lds.s.kc_n[1]);
      }
    }
  }
  // the chunk's cell-sorted neighbour positions ([slot][5] in LDS, [i][5]
  // in HBM: one contiguous run of 5 * live words, 16-B stores).  Nearest_Points
  // ids and pointSearchSqDis are derived from them only when read
  // (nbr_settle: pts[pos].w, and calc_dist from the pass's pose), except in
  // kNN-only passes, whose callers read the distances on the device.
  {
    const int64_t base = chunk * SLIO_CHUNK;
    const int nw = (int)(5 * min((int64_t)SLIO_CHUNK, scan.n - base));
    const int na = cfg.knn_only ? 3 : 1;
    auto dst = [&](int a) {
      return a == 0 ? out.nbr_pos + base * 5
                    : (uint32_t*)(a == 1 ? (void*)out.nbr_idx : (void*)out.nbr_sqd) + base * 5;
    };
    auto src = [&](int a) {
      return a == 0 ? &nb_pos[0][0]
                    : (const uint32_t*)(a == 1 ? (const void*)&nb_idx[0][0] : (const void*)&nb_sqd[0][0]);
    };
    if ((nw & 3) == 0) {
      const int nv = nw >> 2;
      for (int k = tid; k < na * nv; k += NT) {
        const int a = k >= nv ? (k >= 2 * nv ? 2 : 1) : 0;
        const int v = k - a * nv;
        st_out(reinterpret_cast<uint4*>(dst(a)) + v, reinterpret_cast<const uint4*>(src(a))[v]);
      }
    } else {
      for (int k = tid; k < na * nw; k += NT) {
        const int a = k >= nw ? (k >= 2 * nw ? 2 : 1) : 0;
        const int v = k - a * nw;
        st_out(dst(a) + v, src(a)[v]);
      }
    }
  }
  }  // search pass
  // ---------------- phase 3: fixed-order products
  if (cfg.knn_only) return;
  if constexpr (FUSE) {
    const double pv = chunk_sums_256(rows, part, cfg.mfma);
    if (tid < SLIO_NPROD) st_sc1(out.chunk_part + chunk * SLIO_NPROD + tid, pv);  // read by another workgroup
    if (tid == 0) STAMP(3);
    fused_tail<NT, FD, PERS>(lds.L, fuse_bcast, fa, fa.ctl, out.chunk_part, chunk, iter);
  } else {
    if constexpr (NT == 256) {
      const double pv = chunk_sums_256(rows, part, cfg.mfma);
      if (tid < SLIO_NPROD) out.chunk_part[chunk * SLIO_NPROD + tid] = pv;
    } else {
      chunk_products<NT>(rows, part, out.chunk_part + chunk * SLIO_NPROD);
    }
    if (tid == 0) STAMP(3);
  }
}

template <int LPQ, int U, bool SPHERE, bool DEVPOSE, bool FUSE = false, int FD = 6>
__global__ __launch_bounds__(search_block<LPQ>(), SPHERE ? 2 : 4) void k_search_pass(
    const MapView map, const ScanDev scan, const PoseDev pose_arg, const PassCfg cfg,
    const PassOut out, const FuseArgs fa) {
  static_assert(!FUSE || search_block<LPQ>() == kSolveThreads, "fused pass: 256 threads");
#ifdef SLIO_SOLVE_STAMP
  if (FUSE && blockIdx.x == 0 && threadIdx.x == 0) {
    g_sstamp[20] = wall_clock64();
    g_sstamp[21 + ((fa.iter + 1) & 3)] = g_sstamp[20];  // per pass: block 0's start
  }
#endif
  if constexpr (FUSE && !DEVPOSE)
    if (blockIdx.x == 0 && fa.pre) prefetch_ctl<FD>(fa.pre, fa.ctl);
  // DEVPOSE: pose and pass selection come from the device-resident update.
  // A fused pass runs whichever pass the update wants (search or reuse,
  // ctl->search_now = converge, esekfom.hpp:138): one launch per pass in the
  // reference control flow too.
  if (DEVPOSE && (cfg.ctl->done || cfg.ctl->passes != cfg.pass_idx ||
                  (!FUSE && cfg.ctl->search_now != cfg.want_search) || (cfg.seq && cfg.ctl->seq != cfg.seq)))
    return;
  __shared__ PassLds<search_block<LPQ>()> lds;
  __shared__ int fuse_bcast;
  const PoseDev pose = DEVPOSE ? pose_of_ctl(cfg.ctl, cfg.pass_idx) : pose_arg;
  bool reuse = false;
  if constexpr (FUSE && DEVPOSE) reuse = !cfg.ctl->search_now;
  search_pass_body<LPQ, U, SPHERE, DEVPOSE, FUSE, FD, false>(lds, fuse_bcast, map, scan, pose, cfg, out, fa,
                                                            reuse, fa.iter);
}

// The persistent update (single rank, fused passes): ONE launch runs every
// pass of slio_ikf_update_device.  Each workgroup owns one chunk for the whole
// update; after a pass it waits (one lane, write-through polls with s_sleep)
// for the flag the pass's filter step publishes (fused_tail: the control
// block written through, drained, then (seq, done, passes)), reads the next
// pose and whether the pass searches (converge, esekfom.hpp:138) write-through,
// and runs the pass; done ends every workgroup.  No kernel boundary between
// passes (their end-of-kernel write-back and the next launch's start).  The
// host launches it only when every workgroup is resident at once (occupancy
// check) -- a pass's filter step needs all its chunks; a wait past ~1 s gives
// up (the update then reports that it did not complete) instead of hanging.
template <int U, int FD>
__global__ __launch_bounds__(kSolveThreads, 4) void k_update_persist(const MapView map, const ScanDev scan,
                                                                     const PoseDev pose0, const PassCfg cfg,
                                                                     const PassOut out, const FuseArgs fa,
                                                                     const int npasses) {
  __shared__ PassLds<kSolveThreads> lds;
  __shared__ int fuse_bcast;
  __shared__ int s_go;
#ifdef SLIO_SOLVE_STAMP
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    g_sstamp[20] = wall_clock64();
    g_sstamp[21 + ((fa.iter + 1) & 3)] = g_sstamp[20];  // per pass: block 0's start
  }
#endif
  if (blockIdx.x == 0 && fa.pre) prefetch_ctl<FD>(fa.pre, fa.ctl);
  search_pass_body<2, U, false, false, true, FD, true>(lds, fuse_bcast, map, scan, pose0, cfg, out, fa, false,
                                                       fa.iter);
  const uint64_t* flag = fa.goflag + (blockIdx.x & 7) * kGoFlagStride;
  // The pass cycle is entered at two points (the second never taken: npasses
  // >= 1): an irreducible cycle is no natural loop to the optimizer, which
  // would otherwise hoist the body's loop-invariant address arithmetic out of
  // it and keep those values live in scratch across every pass.
  int p = 1;
  if (npasses < 0) goto run;
wait:
  if (p >= npasses) return;
  if (threadIdx.x == 0) {
    int go = 0;
    const unsigned long long t0 = wall_clock64();
    const unsigned long long lim = fa.wait_ticks ? fa.wait_ticks : 100000000ull;
#ifdef SLIO_SOLVE_STAMP
    if (blockIdx.x == 0) g_sstamp[40 + ((fa.iter + p + 1) & 3)] = t0;  // per pass: block 0 waits
#endif
    while (true) {
      if (lim == 1) {  // give up at once (the test hook of slio_debug_wait_limit)
        __hip_atomic_store(&fa.hblk->timeout, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      const uint64_t fl = __hip_atomic_load((const guint64*)flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((int32_t)(fl >> 32) == fa.gseq) {
        if (fl & 0x80000000ull) break;  // the update ended
        if ((int32_t)(fl & 0x7fffffffull) >= p) {
          go = (int)(fl & 0x7fffffffull);
          break;
        }
      }
      if (wall_clock64() - t0 > lim) {  // 100 MHz: 1 s
        __hip_atomic_store(&fa.hblk->timeout, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(4);  // (1 / 16 / 64: the same pass times, profiles/r05_persist_stamps.log)
    }
    s_go = go;
#ifdef SLIO_SOLVE_STAMP
    if (blockIdx.x == 0) g_sstamp[21 + ((fa.iter + p + 1) & 3)] = wall_clock64();
#endif
  }
  __syncthreads();
  if (!s_go) return;
run:
  {
    // the pose slot of the passes counted (== p), taken from the flag, so the
    // scalar loads cannot move above the wait
    const PoseDev pose = pose_of_ctl(fa.ctl, __builtin_amdgcn_readfirstlane(s_go));
    const bool reuse =
        __builtin_amdgcn_readfirstlane(ld_sc1_u32(reinterpret_cast<const uint32_t*>(&fa.ctl->search_now))) == 0;
    search_pass_body<2, U, false, true, true, FD, true>(lds, fuse_bcast, map, scan, pose, cfg, out, fa, reuse,
                                                        fa.iter + p);
  }
  ++p;
  goto wait;
}

// Nearest_Points ids and pointSearchSqDis of the last search pass, derived
// from its neighbour positions: the id is the map point's .w and the
// distance is calc_dist (ikd_Tree.cpp:1539-1544) from the same float query
// (the pass's pose, the same body point), so both equal what the pass found.
__global__ __launch_bounds__(256) void k_nbr_derive(const ScanDev scan, const float4* __restrict__ pts,
                                                    const uint32_t* __restrict__ pos,
                                                    const PoseDev* __restrict__ pose, int64_t b,
                                                    int64_t e, int32_t* __restrict__ idx,
                                                    float* __restrict__ sqd) {
  const int64_t i = b + (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= e) return;
  float qx, qy, qz;
  body_to_world(*pose, scan.bx[i], scan.by[i], scan.bz[i], qx, qy, qz);
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const uint32_t ps = pos[i * 5 + j];
    int32_t id = -1;
    float d = __int_as_float(0x7f800000);
    if (ps != 0xFFFFFFFFu) {
      const float4 c = pts[ps];
      const float ddx = qx - c.x, ddy = qy - c.y, ddz = qz - c.z;
      d = (ddx * ddx + ddy * ddy) + ddz * ddz;
      id = (int32_t)__float_as_uint(c.w);
    }
    idx[i * 5 + j] = id;
    sqd[i * 5 + j] = d;
  }
}

// Non-search pass: reuse neighbours/plane/selection (esekfom.hpp:138-150 with
// converge == false), one lane per point (threads < 128 of 256), the chunk's
// products as in the search pass (chunk_sums_256) -- the same rows and sums
// as the reuse branch of a fused pass.
template <bool DEVPOSE>
__global__ __launch_bounds__(256) void k_reuse_pass(const ScanDev scan,
                                                    const PoseDev pose_arg,
                                                    const PassCfg cfg, const PassOut out) {
  if (DEVPOSE && (cfg.ctl->done || cfg.ctl->passes != cfg.pass_idx ||
                  cfg.ctl->search_now != cfg.want_search))
    return;
  const PoseDev pose = DEVPOSE ? pose_of_ctl(cfg.ctl, cfg.pass_idx) : pose_arg;
  if (DEVPOSE) ikf_dx_new<false>(cfg.ctl);
  __shared__ double rows[SLIO_CHUNK][kRow];
  __shared__ double part[2][SLIO_NPROD];
  const int64_t chunk = xcd_chunk(cfg.c_begin, cfg.c_end - cfg.c_begin);
  const int t = threadIdx.x;
  if (t < SLIO_CHUNK) {
    double row[kRow];
    reuse_row(scan, pose, cfg, out, chunk * SLIO_CHUNK + t, row);
#pragma unroll
    for (int j = 0; j < kRow; ++j) rows[t][j] = row[j];
  }
  __syncthreads();
  const double pv = chunk_sums_256(rows, part, cfg.mfma);
  if (t < SLIO_NPROD) out.chunk_part[chunk * SLIO_NPROD + t] = pv;
}

// chunk_order: the order in which the next search pass's workgroups take
// the chunks of XCD x's range (xcd_chunk gives each XCD a contiguous range,
// so the map region an XCD's L2 serves does not change).  Workgroups are
// placed round-robin (block b on CU b mod #CUs; measured: r3a stamps), so
// local block j of the XCD runs on its CU j mod W in round j / W, and the
// rounds share the CU.  The chunks are ranked by this pass's cost (heaviest
// first) and dealt in snake order -- round 0 ranks 0..W-1, round 1 ranks
// 2W-1..W, ... -- so every CU gets a similar sum of work and the 4th-round
// blocks of a 782-chunk scan the lightest.  Speed only: every order gives
// the same chunk partials.
__device__ __forceinline__ void chunk_order(const uint32_t* __restrict__ cost, uint32_t* __restrict__ perm,
                                            int64_t nblk, int x, int W, uint32_t* cs) {
  const int64_t q = nblk >> 3, rr = nblk & 7;
  const int64_t base = x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q;
  const int n = (int)(q + (x < rr ? 1 : 0));
  const int t = threadIdx.x;
  if (n > (int)blockDim.x || W <= 0) {
    for (int i = t; i < n; i += blockDim.x) perm[base + i] = (uint32_t)(base + i);
    return;
  }
  if (t < n) cs[t] = cost[base + t];
  __syncthreads();
  if (t < n) {
    const uint32_t c = cs[t];
    int rank = 0;
    int j = 0;
    for (; j + 8 <= n; j += 8) {  // 8 independent LDS reads in flight
      uint32_t d[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) d[u] = cs[j + u];
#pragma unroll
      for (int u = 0; u < 8; ++u) rank += (d[u] > c || (d[u] == c && j + u < t)) ? 1 : 0;
    }
    for (; j < n; ++j) {
      const uint32_t d = cs[j];
      rank += (d > c || (d == c && j < t)) ? 1 : 0;
    }
    const int round = rank / W, k = rank - round * W;
    const bool full = (round + 1) * W <= n;
    const int pos = round * W + (((round & 1) && full) ? (W - 1 - k) : k);
    perm[base + pos] = (uint32_t)(base + t);
  }
}

// Super-chunk sums in a fixed order, one workgroup per segment row: segment
// g of super-chunk s sums chunks c0+g, c0+g+8, ... sequentially (workgroup
// 8 s + g, threads < 91 one product each, every chunk load in flight); the
// last workgroup to arrive adds the 8 segments of each super-chunk in order.
// Rows of super-chunks this rank does not own are zeros, so a SUM all-reduce
// over ranks is an exact gather.  The segment rows are handed over
// write-through (sc1 stores, drained before one agent-scope arrival per
// workgroup, sc1 loads by the last; MI355X_MICROARCH.md, inter-workgroup
// visibility).
// D > 0 (single-rank device-resident update): the last workgroup then runs
// the filter step (ikf_step) -- a pass plus its filter step is two launches.
// D == 0: super rows only (host-driven passes, multi-rank all-reduce).
template <int D>
__global__ __launch_bounds__(kSolveThreads) void k_super_sums(
    const double* __restrict__ chunk_part, int64_t C, int s_begin, int s_end, double* seg_out,
    double* super_out, IkfCtl* ctl, const IkfCtl* src, IkfCtl* hblk, uint32_t* cnt, double R, int iter,
    int maxit, const uint32_t* __restrict__ cost, uint32_t* __restrict__ perm, int64_t nblk, int W) {
  constexpr int NT = kSolveThreads;
  __shared__ union {
    double seg[kNSeg][SLIO_NPROD];  // the pass's 64 segment rows (D == 0)
    StepLds L;
  } sh;
  StepLds& L = sh.L;
  __shared__ int arr;
  const int b = blockIdx.x;  // segment row b = 8 s + g
  const int s = b / kSuperSeg, g = b - s * kSuperSeg;
  const int t = threadIdx.x;
  if (D && b == 0) SSTAMP(0);
  // the pass kernel before this one is complete: keep its number of far
  // queries (slio_far_queries), reset the queue's head and tail
  if (b == 0 && t == 0) {
    st_sc1_u32(cnt + 6, ld_sc1_u32(cnt + 5));
    st_sc1_u32(cnt + 4, 0u);
    st_sc1_u32(cnt + 5, 0u);
  }
  if (t < SLIO_NPROD) {
    const int64_t c0 = super_lo(C, s), c1 = super_lo(C, s + 1);
    const bool mine = s >= s_begin && s < s_end;
    const int64_t lim = mine ? (c1 - c0 - g + kSuperSeg - 1) / kSuperSeg : 0;
    const double* p = chunk_part + (c0 + g) * SLIO_NPROD + t;
    constexpr int kJ = 16;  // C2's 100k-point scan has <= 13 chunks per segment: one round trip
    double acc = 0.0;
    for (int64_t j0 = 0; j0 < lim; j0 += kJ) {
      double v[kJ];
#pragma unroll
      for (int j = 0; j < kJ; ++j)
        v[j] = (j0 + j < lim) ? p[(j0 + j) * (kSuperSeg * SLIO_NPROD)] : 0.0;
#pragma unroll
      for (int j = 0; j < kJ; ++j) acc = acc + v[j];
    }
    st_sc1(seg_out + b * SLIO_NPROD + t, acc);
  }
  drain_stores();
  __syncthreads();
  if (t == 0) arr = (int)arrive(cnt);
  __syncthreads();
  if (arr != kNSeg - 1) {
    // the next search pass's chunk order of XCD x = arrival index: the
    // first 8 to arrive (never the last) cover all 8 ranges every pass
    if (perm && arr < 8) chunk_order(cost, perm, nblk, arr, W, reinterpret_cast<uint32_t*>(&sh.seg[0][0]));
    return;
  }
  if (D) SSTAMP(2);
  if (t == 0) reset_counter(cnt);
  if constexpr (D > 0) {
    final_step<NT, D, false>(L, seg_out, super_out, ctl, src, hblk, R, iter, maxit);
  } else {
    constexpr int kR = (kNSeg * SLIO_NPROD + NT - 1) / NT;
    double rv[kR];
#pragma unroll
    for (int u = 0; u < kR; ++u) {
      const int e = t + u * NT;
      rv[u] = e < kNSeg * SLIO_NPROD ? ld_sc1(seg_out + e) : 0.0;
    }
#pragma unroll
    for (int u = 0; u < kR; ++u) {
      const int e = t + u * NT;
      if (e < kNSeg * SLIO_NPROD) (&sh.seg[0][0])[e] = rv[u];
    }
    __syncthreads();
    // thread k < 91: the 8 super rows of product k
    if (t < SLIO_NPROD) {
#pragma unroll
      for (int ss = 0; ss < SLIO_NSUPER; ++ss) {
        double a = sh.seg[ss * kSuperSeg][t];
#pragma unroll
        for (int q = 1; q < kSuperSeg; ++q) a = a + sh.seg[ss * kSuperSeg + q][t];
        super_out[ss * SLIO_NPROD + t] = a;
      }
    }
  }
}

// ---------------------------------------------------------------- device IKF
// Filter step after the multi-rank all-reduce: super sums from HBM.
template <int D>
__global__ __launch_bounds__(kSolveThreads) void k_ikf_solve(IkfCtl* ctl, const IkfCtl* src,
                                                             IkfCtl* hblk, const double* sup,
                                                             double R, int i, int maxit) {
  __shared__ StepLds L;
  step_load<kSolveThreads, D, SLIO_NSUPER * SLIO_NPROD>(L, &L.sup[0][0], sup, false, src, ctl);
  __syncthreads();
  step_totals(L, R);
  __syncthreads();
  if (src == ctl && L.fl[F_DONE]) return;
  ikf_step<kSolveThreads, D>(ctl, hblk, R, i, maxit, L);
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
  uint32_t* nbr_pos = nullptr;
  PoseDev* nbr_pose = nullptr;  // pose of the last search pass (device)
  bool nbr_lazy = false;        // nbr_idx / nbr_sqd not yet derived from nbr_pos
  bool nbr_stale = false;       // ... and no longer derivable: another handle rebuilt the shared map
  uint64_t search_version = 0;  // map version the last search pass ran on
  uint64_t seen_epoch = 0;      // the map's last change this handle's stream is ordered after
  hipEvent_t map_ev = nullptr;  // recorded on this stream by another user's map change
  float* wbx = nullptr;  // scan-to-map: the scan in the map frame
  float* wby = nullptr;
  float* wbz = nullptr;
  int s2m_kind = -1;
  float* nbr_sqd = nullptr;
  float4* plane = nullptr;
  uint8_t* sel = nullptr;
  float* resid = nullptr;
  double* chunk_part = nullptr;
  uint32_t* chunk_cost = nullptr;  // per chunk of the last search pass (chunk_order)
  // kNN certificates of the device-resident update (k_search_pass): per point
  // query + bound (the 5 positions are nbr_pos); per chunk the update epoch
  float4* kq = nullptr;
  uint32_t* k6 = nullptr;
  uint32_t* kepoch = nullptr;
  uint32_t kc_next = 0;       // last epoch handed out
  uint32_t kc_epoch = 0;      // the running update's (0: certificates off)
  uint64_t kc_version = 0;    // map version of the update's first pass
  bool kc_stats = false;      // count certified / searched queries (slio_debug_knn_cert): two
                              // same-address atomics per workgroup, off the product path
  uint32_t* chunk_perm = nullptr;  // search order for the next device-resident pass
  int cus_per_xcd = 0;             // CUs per XCD (0: chunk_order off)
  // far queue (deferred queries, see far_search)
  double* d_super = nullptr;
  double* d_super_own = nullptr;
  double* d_seg = nullptr;    // the pass's 64 segment rows (k_super_sums hand-off)
  void* comm = nullptr;        // RCCL communicator of the rank group (slio_comm_init / slio_create_group)
  int group_reduce = 0;        // slio_create_group: 1 RCCL communicator, 2 in-device reduce (k_group_reduce)
  hipEvent_t grp_ev = nullptr; // in-device reduce: end of this rank's pass / of the reduce (rank 0)
  double* gsup = nullptr;      // fused group pass (rank 0): the group's 8 super rows
  uint32_t* garrive = nullptr; // ... and the ranks' arrival counter
  int32_t group_seq = 0;       // fused group pass: the running update's sequence number (0: none)
  int32_t upd_seq = 0;         // (rank 0) last sequence number handed out
  uint32_t* count = nullptr;  // [0] k_super_sums arrival counter, [4..5] far-queue head / tail,
  MapDev::Buf inc[7];         // map_incremental temporaries, kept across scans
                              // (zero between launches)
  MapDev::Buf pre[16];        // undistortion / VoxelGrid temporaries, kept across scans
                              // (per-call hipMalloc + hipFree cost more than the kernels)
  IkfCtl* ctl = nullptr;    // device-resident update state (HBM)
  IkfCtl* h_ctl = nullptr;  // mapped, coherent host block: update input and output
  IkfCtl* d_hctl = nullptr; // its device view
  hipEvent_t done_ev = nullptr;  // end of a device-resident update (polled)
  double* h_super = nullptr;  // pinned
  bool searched = false;
  // profiling: event pairs pending per kind, accumulated time
  bool prof = false;
  int prof_mask = 0;  // bit k: time kernel kind k
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pending[3];
  std::vector<std::pair<hipEvent_t, hipEvent_t>> pool;
  double prof_ms[3] = {0, 0, 0};
  int64_t prof_n[3] = {0, 0, 0};
  // diagnostic switches of the update path, read from the environment once
  // per handle (slio_create, slio_debug_reload_switches): no getenv on the
  // host turnaround between updates
  struct Switches {
    bool no_fuse = false;     // SLIO_NO_FUSE: two launches per pass
    bool no_fuse0 = false;    // SLIO_NO_FUSE0: two launches for the first pass
    bool no_mfma = false;     // SLIO_NO_MFMA: VALU chunk products
    bool event_wait = false;  // SLIO_EVENT_WAIT: wait on a completion event
    bool no_kc = false;       // SLIO_NO_KNN_CERT: every pass searches in full
    bool persist = false;     // SLIO_PERSIST: one persistent launch per update (k_update_persist)
  } sw;
  // persistent update (k_update_persist): the flag replicas, the CU count and
  // the workgroups the device holds at once (-1: not yet queried)
  uint64_t* goflag = nullptr;
  int ncu = 0;
  int64_t persist_cap = -1;
  int last_path = 0;  // the last device-resident update: 1 persistent launch, 0 a launch per pass
  bool dev_counted = false;  // counted in dev_users (slio_create succeeded)
  uint64_t wait_ticks = 0;  // device-side waits give up after this many 100 MHz ticks (0: 1 s;
                            // slio_debug_wait_limit)
  // host clock stamps (CLOCK_MONOTONIC ns) of the last device-resident update
  // (slio_debug_host_stamps)
  bool hstamp = false;
  int64_t hst[8] = {};
};

int dev_users(int device, int delta) {
  static std::atomic<int> users[256];
  if (device < 0 || device >= 256) return 0;
  return users[device].fetch_add(delta) + delta;
}

static bool env_on(const char* name) {
  const char* e = std::getenv(name);
  return e && e[0] && e[0] != '0';
}
static void load_switches(Ctx& c) {
  c.sw.no_fuse = env_on("SLIO_NO_FUSE");
  c.sw.no_fuse0 = env_on("SLIO_NO_FUSE0");
  c.sw.no_mfma = env_on("SLIO_NO_MFMA");
  c.sw.event_wait = env_on("SLIO_EVENT_WAIT");
  c.sw.no_kc = env_on("SLIO_NO_KNN_CERT");
  c.sw.persist = env_on("SLIO_PERSIST");
}
static inline int64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (int64_t)ts.tv_sec * 1000000000LL + ts.tv_nsec;
}
#define SLIO_HSTAMP(c, k) \
  do {                    \
    if ((c).hstamp) (c).hst[k] = mono_ns(); \
  } while (0)

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

// Map sharing: stream ordering of changes and reads (MapDev::mu held by the
// caller: exclusively for map_write_begin / _end, either way for
// map_read_sync).
static int map_write_begin(Ctx& c) {
  MapDev& m = *c.map;
  for (Ctx* u : m.users) {
    if (u == &c || u->stream == c.stream) continue;
    if (!u->map_ev) SLIO_HIP(hipEventCreateWithFlags(&u->map_ev, hipEventDisableTiming));
    SLIO_HIP(hipEventRecord(u->map_ev, u->stream));
    SLIO_HIP(hipStreamWaitEvent(c.stream, u->map_ev, 0));
  }
  if (m.ready && c.seen_epoch != m.epoch) SLIO_HIP(hipStreamWaitEvent(c.stream, m.ready, 0));
  return SLIO_OK;
}
static int map_write_end(Ctx& c) {
  MapDev& m = *c.map;
  if (!m.ready) SLIO_HIP(hipEventCreateWithFlags(&m.ready, hipEventDisableTiming));
  SLIO_HIP(hipEventRecord(m.ready, c.stream));
  c.seen_epoch = ++m.epoch;
  return SLIO_OK;
}
static int map_read_sync(Ctx& c) {
  MapDev& m = *c.map;
  if (c.seen_epoch != m.epoch) {
    if (m.ready) SLIO_HIP(hipStreamWaitEvent(c.stream, m.ready, 0));
    c.seen_epoch = m.epoch;
  }
  if (m.broken) {
    set_error("slio map: an index rebuild failed part-way; upload the map again");
    return SLIO_EDEVICE;
  }
  return SLIO_OK;
}
// attach c to map m (nullptr: detach), keeping the users list
static void map_attach(Ctx& c, std::shared_ptr<MapDev> m) {
  if (c.map) {
    std::unique_lock<std::shared_mutex> lk(c.map->mu);
    auto& u = c.map->users;
    u.erase(std::remove(u.begin(), u.end(), &c), u.end());
  }
  c.map = std::move(m);
  c.seen_epoch = 0;  // the new map's last change is not yet waited for
  if (c.map) {
    std::unique_lock<std::shared_mutex> lk(c.map->mu);
    c.map->users.push_back(&c);
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
  (void)hipFree(c->nbr_pos);
  c->nbr_pos = nullptr;
  (void)hipFree(c->nbr_pose);
  c->nbr_pose = nullptr;
  c->nbr_lazy = false;
  (void)hipFree(c->wbx);
  (void)hipFree(c->wby);
  (void)hipFree(c->wbz);
  c->wbx = c->wby = c->wbz = nullptr;
  (void)hipFree(c->nbr_sqd);
  (void)hipFree(c->plane);
  (void)hipFree(c->sel);
  (void)hipFree(c->resid);
  (void)hipFree(c->chunk_part);
  (void)hipFree(c->chunk_cost);
  (void)hipFree(c->chunk_perm);
  c->chunk_cost = c->chunk_perm = nullptr;
  (void)hipFree(c->kq);
  (void)hipFree(c->k6);
  (void)hipFree(c->kepoch);
  c->kq = nullptr;
  c->k6 = nullptr;
  c->kepoch = nullptr;
  c->bx = c->by = c->bz = nullptr;
  c->nbr_idx = nullptr;
  c->nbr_sqd = nullptr;
  c->plane = nullptr;
  c->sel = nullptr;
  c->resid = nullptr;
  c->chunk_part = nullptr;
}

// Enqueue one measurement pass (+ super-chunk sums) on the handle's stream.
// Host mode: pose P by value, search iff which == 1.  Device mode (ctl != 0):
// the pose and the search/reuse choice come from the control block in HBM;
// which == 2 launches both kernels (each exits unless selected).
// Wait for everything enqueued on the handle's stream by polling an event: a
// blocking stream sync sleeps and wakes ~10-20 us late, a large share of a
// ~60 us IKF iteration.
static hipError_t wait_stream(Ctx& c) {
  hipError_t e;
  if (!c.done_ev && (e = hipEventCreateWithFlags(&c.done_ev, hipEventDisableTiming))) return e;
  if ((e = hipEventRecord(c.done_ev, c.stream))) return e;
  while ((e = hipEventQuery(c.done_ev)) == hipErrorNotReady) {
  }
  return e;
}

// The same polled wait for any stream (the map maintenance, scan VoxelGrid
// and scan-to-map paths read counts and boxes back several times per scan):
// one event per device and host thread.
static hipError_t spin_sync(hipStream_t st) {
  thread_local hipEvent_t evs[16] = {};
  hipDevice_t dev = 0;
  hipError_t e = hipStreamGetDevice(st, &dev);
  if (e != hipSuccess || dev < 0 || dev >= 16) {
    (void)hipGetLastError();
    return hipStreamSynchronize(st);
  }
  if (!evs[dev]) {
    int cur = 0;
    (void)hipGetDevice(&cur);
    if (cur != dev) (void)hipSetDevice(dev);
    e = hipEventCreateWithFlags(&evs[dev], hipEventDisableTiming);
    if (cur != dev) (void)hipSetDevice(cur);
    if (e) return e;
  }
  if ((e = hipEventRecord(evs[dev], st))) return e;
  while ((e = hipEventQuery(evs[dev])) == hipErrorNotReady) __builtin_ia32_pause();
  return e;
}

// Small device -> host reads (scan totals, counters, boxes) through a pinned
// staging buffer of the calling thread, then one polled wait: a copy into
// pageable host memory waits inside the runtime, and a blocking stream
// synchronisation wakes ~10-20 us late.
struct Rb {
  void* dst;
  const void* src;
  size_t n;
};
static hipError_t readback(hipStream_t st, const Rb* rb, int k) {
  thread_local uint8_t* pin = nullptr;
  thread_local size_t cap = 0;
  size_t tot = 0;
  for (int j = 0; j < k; ++j) tot += (rb[j].n + 15) & ~(size_t)15;
  if (tot > cap) {
    if (pin) (void)hipHostFree(pin);
    pin = nullptr;
    cap = 0;
    const size_t want = std::max<size_t>(tot, 4096);
    if (hipHostMalloc((void**)&pin, want) != hipSuccess) {
      (void)hipGetLastError();
      pin = nullptr;
    } else {
      cap = want;
    }
  }
  hipError_t e = hipSuccess;
  if (!pin) {  // (no pinned buffer: the plain copies)
    for (int j = 0; j < k && !e; ++j) e = hipMemcpyAsync(rb[j].dst, rb[j].src, rb[j].n, hipMemcpyDeviceToHost, st);
    return e ? e : hipStreamSynchronize(st);
  }
  size_t off = 0;
  for (int j = 0; j < k && !e; ++j) {
    e = hipMemcpyAsync(pin + off, rb[j].src, rb[j].n, hipMemcpyDeviceToHost, st);
    off += (rb[j].n + 15) & ~(size_t)15;
  }
  if (!e) e = spin_sync(st);
  if (e) return e;
  off = 0;
  for (int j = 0; j < k; ++j) {
    std::memcpy(rb[j].dst, pin + off, rb[j].n);
    off += (rb[j].n + 15) & ~(size_t)15;
  }
  return hipSuccess;
}

// Wait for the device-resident update to publish its result in the mapped
// host block (one release store after x, P and the flags), which the host
// sees ~1 us after it happens; the stream's completion event is polled now
// and then so that a failed launch (no publication) still ends the wait.
// Kernels of the update still queued behind the publication exit at once
// (ctl->done) and touch neither the mapped block nor the caller's buffers.
static hipError_t wait_published(Ctx& c) {
  hipError_t e;
  // the stream itself is queried now and then (a failed or early-exiting
  // launch still ends the wait): no completion-event packet behind the
  // update's kernels (SLIO_EVENT_WAIT=1: the round-2 event record + query)
  const bool use_event = c.sw.event_wait;
  if (use_event) {
    if (!c.done_ev && (e = hipEventCreateWithFlags(&c.done_ev, hipEventDisableTiming))) return e;
    if ((e = hipEventRecord(c.done_ev, c.stream))) return e;
  }
  volatile int32_t* pub = &c.h_ctl->published;
  for (uint32_t it = 1;; ++it) {
    if (*pub) break;
    if ((it & 255) == 0) {
      e = use_event ? hipEventQuery(c.done_ev) : hipStreamQuery(c.stream);
      if (e != hipErrorNotReady) {
        if (e != hipSuccess) return e;
        break;  // all work done: the flags tell whether it published
      }
    }
    __builtin_ia32_pause();
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  return hipSuccess;
}

// After an update that did not complete (a device-side wait gave up, or a
// launch failed): wait for the handle's stream to drain, then zero the
// arrival counters (segment rows, passes, far queue), the persistent update's
// flag replicas and, on a group's rank 0, the ranks' arrival word and gate
// flag, so that the next update's last arriver is the right one.
static void reset_update_counters(Ctx& c) {
  (void)hipStreamSynchronize(c.stream);
  if (c.count) (void)hipMemsetAsync(c.count, 0, sizeof(uint32_t) * kCountWords, c.stream);
  if (c.goflag) (void)hipMemsetAsync(c.goflag, 0, sizeof(uint64_t) * 8 * kGoFlagStride, c.stream);
  if (c.garrive) (void)hipMemsetAsync(c.garrive, 0, 4 * sizeof(uint32_t), c.stream);
  (void)hipStreamSynchronize(c.stream);
  (void)hipGetLastError();
}

// Fused filter step of a single-rank device-resident update.
struct SolveArgs {
  int on;        // run the filter step in the super-sum kernel (single rank)
  int dim;       // D of the filter step: 6 without extrinsic estimation, 12 with
  int pass_idx;  // ctl->passes this pass belongs to
  int iter, maxit;
  double R;
  const IkfCtl* src;  // control block source: the mapped host block on pass 0, else ctl
  IkfCtl* hblk;       // mapped host block (device view): update output
};

static void enqueue_super(Ctx& c, IkfCtl* ctl, const SolveArgs* sa);
static int map_refresh(Ctx& c, bool adds_only = false);
static int map_refresh_locked(Ctx& c, bool adds_only);
static int nbr_settle_shared(Ctx& c);
static int build_blk(MapDev& m, hipStream_t st, const char* who);

static int enqueue_pass(Ctx& c, const PoseDev* Parg, IkfCtl* ctl, int which,
                        int extrinsic_est, const SolveArgs* sa = nullptr,
                        bool with_super = true, bool knn_only = false, const ScanDev* sd = nullptr,
                        const FuseArgs* fuse = nullptr, int persist = 0) {
  if (!c.map) {
    set_error("slio pass: no map uploaded");
    return SLIO_ESTATE;
  }
  if (!c.bx && c.n > 0) {
    set_error("slio pass: no scan uploaded");
    return SLIO_ESTATE;
  }
  if (which == 0 && !c.searched) {
    set_error("slio pass: reuse pass before any search pass");
    return SLIO_ESTATE;
  }
  int64_t c0, c1;
  rank_chunks(c.n, c.prm.rank, c.prm.nranks, &c0, &c1);
  // pose: by value (host-driven passes and the first pass of a device-resident
  // update) or from the control block in HBM (later device-resident passes)
  const bool devpose = ctl && !Parg;
  PassCfg cfg;
  cfg.ctl = (devpose || persist) ? ctl : nullptr;
  cfg.want_search = 1;
  cfg.plane_thr = c.prm.plane_threshold;
  cfg.max_sqd = c.prm.max_match_sqd;
  {
    // the first sphere must sit inside the 5x5x5 cube: rho0 < 2h
    const float rho = std::min(c.prm.search_radius, 1.99f * c.map->g.h);
    cfg.radius_sq = rho > 0.0f ? rho * rho : 0.0f;
  }
  cfg.far_sq = c.prm.far_query_margin > 0.0f ? c.prm.far_query_margin * c.prm.far_query_margin : 0.0f;
  cfg.extrinsic = extrinsic_est ? 1 : 0;
  cfg.c_begin = c0;
  cfg.c_end = c1;
  cfg.pass_idx = sa ? sa->pass_idx : 0;
  cfg.knn_only = knn_only ? 1 : 0;
  cfg.mfma = !c.sw.no_mfma;
  // later passes of a device-resident update take their chunks in the order
  // the previous pass's costs call for (chunk_order; pass 0 in index order)
  static const bool no_order = std::getenv("SLIO_NO_CHUNK_ORDER") != nullptr;
  // (fused passes compute no order: c.chunk_perm may be another scan's)
  cfg.perm = (devpose && !fuse && c.cus_per_xcd > 0 && !no_order) ? c.chunk_perm : nullptr;
  if (int rc = map_refresh(c); rc) return rc;
  if (which != 0 && c.map->blk_deferred) {
    std::unique_lock<std::shared_mutex> lk(c.map->mu);
    if (c.map->blk_deferred && (c.map->stable_passes += (persist > 0 ? persist : 1)) > kBlkAfterPasses) {
      if (int rc = map_write_begin(c)) return rc;
      if (int rc = build_blk(*c.map, c.stream, "slio map"); rc) return rc;
      if (int rc = map_write_end(c)) return rc;
    }
  }
  // the views are read and the kernels launched under the shared lock: a
  // change by another handle waits for these launches (map_write_begin)
  std::shared_lock<std::shared_mutex> map_lock(c.map->mu);
  if (int rc = map_read_sync(c)) return rc;
  // kNN certificates: only a device-resident pass after the update's first,
  // on the map that pass ran on (another handle sharing the map may have
  // rebuilt it in between)
  if (!devpose) c.kc_version = c.map->version;
  cfg.kc_epoch = ((devpose || persist) && c.kq && c.map->version == c.kc_version) ? c.kc_epoch : 0;
  cfg.seq = fuse ? c.group_seq : 0;
  PassOut o{c.nbr_idx,    c.nbr_pos,    c.nbr_sqd,   c.plane,  c.sel,    c.resid,
            c.chunk_part, c.count + 4, c.nbr_pose, c.chunk_cost, c.kq, c.k6,
            c.kepoch,     c.kc_stats ? c.count + kKcCount : nullptr};
  ScanDev s = sd ? *sd : ScanDev{c.bx, c.by, c.bz, c.n};
  const PoseDev P = Parg ? *Parg : PoseDev{};
  const int64_t nblk = c1 - c0;
  if (c.prof && (c.pending[0].size() + c.pending[1].size()) > 256) prof_drain(c);
  // (a fused pass is one launch of the search kernel, which also runs the
  // reuse pass when the update asks for one)
  const bool run_search = which != 0, run_reuse = which != 1 && !fuse;
  // Profiled launches carry their start/stop events inside the dispatch
  // packet (hipExtLaunchKernelGGL): no separate marker packets, so timing
  // does not open gaps between the dependent kernels.
  auto timing = [&](int kind) {
    std::pair<hipEvent_t, hipEvent_t> ev{nullptr, nullptr};
    if (c.prof && (c.prof_mask & (1 << kind))) {
      ev = prof_pair(c);
      c.pending[kind].push_back(ev);
    }
    return ev;
  };
  if (nblk > 0 && run_search) {
    const auto ev = timing(SLIO_KERNEL_SEARCH);
    const CoarseView cv{c.map->cg, c.map->clo, c.map->chi};
    const MapView mv{c.map->g,   c.map->n,    c.map->pts,    c.map->start, c.map->blk,
                     c.map->bstart, c.map->nblk, c.map->ncells, cv};
    const bool sph = cfg.radius_sq > 0.0f;
    const dim3 nb((unsigned)nblk);
#define SLIO_LAUNCH(L, SPH, DEV)                                                                   \
  hipExtLaunchKernelGGL(k_search_pass<L, SLIO_SEARCH_U, SPH, DEV>, nb, dim3(search_block<L>()), 0, c.stream, \
                        ev.first, ev.second, 0, mv, s, P, cfg, o, FuseArgs{})
#define SLIO_LAUNCH2(L, SPH) \
  do {                        \
    if (devpose)              \
      SLIO_LAUNCH(L, SPH, true); \
    else                      \
      SLIO_LAUNCH(L, SPH, false); \
  } while (0)
    if (fuse) {
      // fused pass (fusable() checked the configuration): the filter step
      // (D = 6, or 12 with extrinsic estimation) runs in this launch, no
      // k_super_sums; a later pass is a search or a reuse pass as the update
      // decides on the device
#define SLIO_LAUNCH_FUSED(DEV, D)                                                                           \
  hipExtLaunchKernelGGL(k_search_pass<2, SLIO_SEARCH_U, false, DEV, true, D>, nb, dim3(kSolveThreads), 0, \
                        c.stream, ev.first, ev.second, 0, mv, s, P, cfg, o, *fuse)
#define SLIO_LAUNCH_PERSIST(D)                                                                    \
  hipExtLaunchKernelGGL(k_update_persist<SLIO_SEARCH_U, D>, nb, dim3(kSolveThreads), 0, c.stream, ev.first, \
                        ev.second, 0, mv, s, P, cfg, o, *fuse, persist)
      if (persist > 0) {
        if (sa && sa->dim == 12)
          SLIO_LAUNCH_PERSIST(12);
        else
          SLIO_LAUNCH_PERSIST(6);
      } else if (sa && sa->dim == 12) {
        if (devpose)
          SLIO_LAUNCH_FUSED(true, 12);
        else
          SLIO_LAUNCH_FUSED(false, 12);
      } else {
        if (devpose)
          SLIO_LAUNCH_FUSED(true, 6);
        else
          SLIO_LAUNCH_FUSED(false, 6);
      }
#undef SLIO_LAUNCH_FUSED
#undef SLIO_LAUNCH_PERSIST
    } else
    switch (c.prm.lanes_per_query * 2 + (sph ? 1 : 0)) {
      case 2: SLIO_LAUNCH2(1, false); break;
      case 3: SLIO_LAUNCH2(1, true); break;
      case 8: SLIO_LAUNCH2(4, false); break;
      case 9: SLIO_LAUNCH2(4, true); break;
      case 16: SLIO_LAUNCH2(8, false); break;
      case 17: SLIO_LAUNCH2(8, true); break;
      case 5: SLIO_LAUNCH2(2, true); break;
      default: SLIO_LAUNCH2(2, false); break;
    }
#undef SLIO_LAUNCH2
#undef SLIO_LAUNCH
    c.nbr_lazy = !knn_only;
    c.nbr_stale = false;
  }
  if (nblk > 0 && run_reuse) {
    const auto ev = timing(SLIO_KERNEL_REUSE);
    PassCfg rcfg = cfg;
    rcfg.want_search = 0;
    const dim3 nb((unsigned)nblk), bs(256);
    if (devpose)
      hipExtLaunchKernelGGL(k_reuse_pass<true>, nb, bs, 0, c.stream, ev.first, ev.second, 0, s, P,
                            rcfg, o);
    else
      hipExtLaunchKernelGGL(k_reuse_pass<false>, nb, bs, 0, c.stream, ev.first, ev.second, 0, s, P,
                            rcfg, o);
  }
  if (with_super && !fuse) enqueue_super(c, ctl, sa);
  SLIO_HIP(hipGetLastError());
  if (which != 0) {
    c.searched = true;
    c.search_version = c.map->version;
  }
  return SLIO_OK;
}

// Derive the last search pass's Nearest_Points ids and pointSearchSqDis
// (k_nbr_derive) while its scan, map and pose are still the handle's: called
// before they change and before the results are read.
static int nbr_settle(Ctx& c) {
  if (!c.nbr_lazy) return SLIO_OK;
  c.nbr_lazy = false;
  // another handle sharing the map rebuilt it since this handle's last
  // search pass: the stored positions point into moved points
  if (!c.map || c.search_version != c.map->version) {
    c.nbr_stale = true;
    return SLIO_OK;
  }
  int64_t c0, c1;
  rank_chunks(c.n, c.prm.rank, c.prm.nranks, &c0, &c1);
  const int64_t b = c0 * SLIO_CHUNK, e = std::min(c1 * SLIO_CHUNK, c.n);
  if (e <= b || !c.map) return SLIO_OK;
  k_nbr_derive<<<(unsigned)((e - b + 255) / 256), 256, 0, c.stream>>>(ScanDev{c.bx, c.by, c.bz, c.n}, c.map->pts,
                                                         c.nbr_pos, c.nbr_pose, b, e, c.nbr_idx,
                                                         c.nbr_sqd);
  SLIO_HIP(hipGetLastError());
  return SLIO_OK;
}

// nbr_settle from outside any map lock (before the handle's scan or map is
// replaced, or its neighbours are read)
static int nbr_settle_shared(Ctx& c) {
  if (!c.nbr_lazy) return SLIO_OK;
  if (!c.map) return nbr_settle(c);
  std::shared_lock<std::shared_mutex> lk(c.map->mu);
  if (int rc = map_read_sync(c)) return rc;
  return nbr_settle(c);
}

// Super-chunk sums of the pass just enqueued (+ the filter step of a
// single-rank device-resident update).
static void enqueue_super(Ctx& c, IkfCtl* ctl, const SolveArgs* sa) {
  const int64_t C = num_chunks(c.n);
  int64_t c0, c1;
  rank_chunks(c.n, c.prm.rank, c.prm.nranks, &c0, &c1);
  const int per = SLIO_NSUPER / c.prm.nranks;
  std::pair<hipEvent_t, hipEvent_t> ev{nullptr, nullptr};
  if (c.prof && (c.prof_mask & (1 << SLIO_KERNEL_SUPER))) {
    ev = prof_pair(c);
    c.pending[SLIO_KERNEL_SUPER].push_back(ev);
  }
  const bool fuse = sa && sa->on;
  const auto kern = !fuse ? k_super_sums<0> : (sa->dim == 12 ? k_super_sums<12> : k_super_sums<6>);
  hipExtLaunchKernelGGL(kern, dim3(kNSeg), dim3(kSolveThreads), 0, c.stream, ev.first, ev.second, 0,
                        (const double*)c.chunk_part, C, c.prm.rank * per, (c.prm.rank + 1) * per,
                        c.d_seg, c.d_super, fuse ? ctl : (IkfCtl*)nullptr,
                        fuse ? sa->src : (const IkfCtl*)nullptr, fuse ? sa->hblk : (IkfCtl*)nullptr,
                        c.count, fuse ? sa->R : 0.0, fuse ? sa->iter : 0, fuse ? sa->maxit : 0,
                        (const uint32_t*)c.chunk_cost, c.chunk_perm, c1 - c0, c.cus_per_xcd);
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

#ifdef SLIO_ABL_STAMP
int slio_debug_clear_stamps(void) {
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_rstamps)) != hipSuccess) return -3;
  return hipMemset(p, 0, sizeof(g_rstamps)) == hipSuccess ? 0 : -3;
}
int slio_debug_stamps(unsigned long long* out, int nblocks) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 8 * nblocks) ==
                 hipSuccess
             ? 0
             : -3;
}
int slio_debug_wstamps(unsigned long long* out, int nblocks) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wstamps), sizeof(unsigned long long) * 16 * nblocks) ==
                 hipSuccess
             ? 0
             : -3;
}
int slio_debug_fstamps(unsigned long long* out, int nblocks) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fstamps), sizeof(unsigned long long) * 6 * nblocks) ==
                 hipSuccess
             ? 0
             : -3;
}
int slio_debug_rstamps(unsigned long long* out, int nblocks) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rstamps), sizeof(unsigned long long) * 6 * nblocks) ==
                 hipSuccess
             ? 0
             : -3;
}
int slio_debug_hwid(uint32_t* out, int nblocks) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_hwid), sizeof(uint32_t) * 2 * nblocks) == hipSuccess
             ? 0
             : -3;
}
#endif

const char* slio_last_error(void) { return g_err.c_str(); }
#ifndef SLIO_SOURCE_HASH
#define SLIO_SOURCE_HASH "unknown"
#endif
const char* slio_build_id(void) { return SLIO_SOURCE_HASH; }

int slio_params_default(slio_params* p) {
  if (!p) return SLIO_EINVAL;
  std::memset(p, 0, sizeof(*p));
  p->device = 0;
  p->max_points = 100000;
  p->rank = 0;
  p->nranks = 1;
  p->grid_cell = 0.0f;       // auto: 1.0 m, or 1.25 m for a grid of more than 2^27 cells
  p->search_radius = 0.0f;   // 3x3x3 block first (tuned); > 0 selects the sphere search
  p->plane_threshold = 0.1f;
  p->max_match_sqd = 5.0f;
  p->max_grid_cells = (int64_t)1 << 29;
  p->far_query_margin = 0.0f;  // exact everywhere (ikd-Tree has no cut)
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
  if (!(p->far_query_margin >= 0.0f) || !(p->search_radius >= 0.0f)) {
    set_error("slio_create: far_query_margin / search_radius must be >= 0");
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
  if (!(h->c.prm.grid_cell > 0.0f)) h->c.prm.grid_cell = 0.0f;  // auto (build_index)
  if (h->c.prm.max_grid_cells <= 0) h->c.prm.max_grid_cells = (int64_t)1 << 29;
  {
    const int l = h->c.prm.lanes_per_query;
    if (l != 1 && l != 2 && l != 4 && l != 8) h->c.prm.lanes_per_query = kDefaultLPQ;
  }
  if (hipStreamCreateWithFlags(&h->c.own_stream, hipStreamNonBlocking) != hipSuccess) {
    delete h;
    set_error("slio_create: hipStreamCreate failed");
    return SLIO_EDEVICE;
  }
  h->c.stream = h->c.own_stream;
  load_switches(h->c);
  {
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, p->device) == hipSuccess &&
        ncu > 0 && ncu % 8 == 0)
      h->c.cus_per_xcd = ncu / 8;
    h->c.ncu = ncu;
  }
  if (hipMalloc(&h->c.d_super_own, sizeof(double) * SLIO_NSUPER * SLIO_NPROD) != hipSuccess ||
      hipMalloc(&h->c.d_seg, sizeof(double) * kNSeg * SLIO_NPROD) != hipSuccess ||
      hipHostMalloc(&h->c.h_super, sizeof(double) * SLIO_NSUPER * SLIO_NPROD) != hipSuccess ||
      hipMalloc(&h->c.count, sizeof(uint32_t) * kCountWords) != hipSuccess ||
      hipMemset(h->c.count, 0, sizeof(uint32_t) * kCountWords) != hipSuccess ||
      hipMalloc(&h->c.goflag, sizeof(uint64_t) * 8 * kGoFlagStride) != hipSuccess ||
      hipMemset(h->c.goflag, 0, sizeof(uint64_t) * 8 * kGoFlagStride) != hipSuccess ||
      false) {
    set_error("slio_create: allocation failed");
    slio_destroy(h);
    return SLIO_ENOMEM;
  }
  h->c.d_super = h->c.d_super_own;
  h->c.dev_counted = true;
  dev_users(p->device, +1);
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
  (void)hipFree(h->c.d_seg);
  (void)hipFree(h->c.count);
  (void)hipFree(h->c.goflag);
  for (auto& b : h->c.inc)
    if (b.p) (void)hipFree(b.p);
  for (auto& b : h->c.pre)
    if (b.p) (void)hipFree(b.p);
  if (h->c.comm) (void)ncclCommDestroy((ncclComm_t)h->c.comm);
  if (h->c.grp_ev) (void)hipEventDestroy(h->c.grp_ev);
  (void)hipFree(h->c.gsup);
  (void)hipFree(h->c.garrive);
  (void)hipFree(h->c.ctl);
  (void)hipHostFree(h->c.h_ctl);
  if (h->c.done_ev) (void)hipEventDestroy(h->c.done_ev);
  (void)hipHostFree(h->c.h_super);
  map_attach(h->c, nullptr);
  if (h->c.map_ev) (void)hipEventDestroy(h->c.map_ev);
  if (h->c.own_stream) (void)hipStreamDestroy(h->c.own_stream);
  if (h->c.dev_counted) dev_users(h->c.prm.device, -1);
  delete h;
  return SLIO_OK;
}

int slio_set_stream(slio_handle h, void* s) {
  SLIO_CHECK_H(h);
  h->c.stream = s ? (hipStream_t)s : h->c.own_stream;
  return SLIO_OK;
}

int slio_debug_reload_switches(slio_handle h) {
  if (!h) return SLIO_EINVAL;
  load_switches(h->c);
  return SLIO_OK;
}

int slio_debug_knn_cert(slio_handle h, uint32_t out[2]) {
  SLIO_CHECK_H(h);
  if (!out) return SLIO_EINVAL;
  h->c.kc_stats = true;  // counting starts with the first call
  SLIO_HIP(hipStreamSynchronize(h->c.stream));
  SLIO_HIP(hipMemcpy(out, h->c.count + kKcCount, 8, hipMemcpyDeviceToHost));
  return SLIO_OK;
}

int slio_debug_host_stamps(slio_handle h, int enable, int64_t out[8]) {
  if (!h) return SLIO_EINVAL;
  if (out) std::memcpy(out, h->c.hst, sizeof(h->c.hst));
  if (enable >= 0) h->c.hstamp = enable != 0;
  return SLIO_OK;
}

int slio_debug_wait_limit(slio_handle h, int64_t ticks) {
  SLIO_CHECK_H(h);
  if (ticks < 0) {
    set_error("slio_debug_wait_limit: ticks < 0");
    return SLIO_EINVAL;
  }
  h->c.wait_ticks = (uint64_t)ticks;
  return SLIO_OK;
}

int slio_debug_update_path(slio_handle h) {
  if (!h) return SLIO_EINVAL;
  return h->c.last_path;
}

}  // extern "C"

// ---------------------------------------------------------------- map index build
namespace slio {

__global__ void k_pack_ids(const float* __restrict__ x, const float* __restrict__ y,
                           const float* __restrict__ z, int64_t n, uint32_t id0, float4* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = make_float4(x[i], y[i], z[i], __uint_as_float(id0 + (uint32_t)i));
}

// sort key (cell << idbits) | id: the cell-sorted map keeps ascending ids
// inside a cell (the tie order of the kNN keys), whatever order the points
// come in
__global__ void k_cell_keys64(const float4* __restrict__ in, int64_t n, GridGeom g, int idbits,
                              uint64_t* __restrict__ keys, uint32_t* __restrict__ vals) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 p = in[i];
  const int cx = min(max(cell_coord(p.x, g.ox, g.inv_h), 0), g.dx - 1);
  const int cy = min(max(cell_coord(p.y, g.oy, g.inv_h), 0), g.dy - 1);
  const int cz = min(max(cell_coord(p.z, g.oz, g.inv_h), 0), g.dz - 1);
  const uint64_t cell = ((uint64_t)cz * (uint64_t)g.dy + (uint64_t)cy) * (uint64_t)g.dx + (uint64_t)cx;
  keys[i] = (cell << idbits) | (uint64_t)__float_as_uint(p.w);
  vals[i] = (uint32_t)i;
}

__global__ void k_gather4(const float4* __restrict__ in, const uint32_t* __restrict__ order, int64_t n,
                          float4* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = in[order[i]];
}

// order-preserving float keys for atomic min / max
__device__ __forceinline__ int32_t fkey(float f) {
  const int32_t b = __float_as_int(f);
  return b >= 0 ? b : b ^ 0x7FFFFFFF;
}
static inline float fkey_inv(int32_t k) {
  const int32_t b = k >= 0 ? k : k ^ 0x7FFFFFFF;
  float f;
  std::memcpy(&f, &b, 4);
  return f;
}

// bounding box: out[0..2] min keys, out[3..5] max keys; out[6] = 1 if a
// coordinate is not finite
__global__ void k_bbox4(const float4* __restrict__ in, int64_t n, int32_t* __restrict__ out) {
  int32_t lo[3] = {INT32_MAX, INT32_MAX, INT32_MAX}, hi[3] = {INT32_MIN, INT32_MIN, INT32_MIN};
  int bad = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 p = in[i];
    const float c[3] = {p.x, p.y, p.z};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      bad |= !isfinite(c[a]);
      const int32_t k = fkey(c[a]);
      lo[a] = min(lo[a], k);
      hi[a] = max(hi[a], k);
    }
  }
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    for (int d = 32; d > 0; d >>= 1) {
      lo[a] = min(lo[a], __shfl_xor(lo[a], d, 64));
      hi[a] = max(hi[a], __shfl_xor(hi[a], d, 64));
    }
  }
  bad = __any(bad);
  // one set of atomics per workgroup: the 6 counters are shared by the
  // whole grid, and same-address atomics serialise (one per wavefront of a
  // 2048-block grid took 0.58 ms on a 10M-point map)
  __shared__ int32_t wl[3][4], wh[3][4];
  __shared__ int wb[4];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      wl[a][w] = lo[a];
      wh[a][w] = hi[a];
    }
    wb[w] = bad;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    const int a = threadIdx.x;
    int32_t l = wl[a][0], h = wh[a][0];
    for (int q = 1; q < (int)(blockDim.x >> 6); ++q) {
      l = min(l, wl[a][q]);
      h = max(h, wh[a][q]);
    }
    atomicMin(out + a, l);
    atomicMax(out + 3 + a, h);
  } else if (threadIdx.x == 3) {
    int b = 0;
    for (int q = 0; q < (int)(blockDim.x >> 6); ++q) b |= wb[q];
    if (b) atomicOr(out + 6, 1);
  }
}

__global__ void k_iota_u32(uint32_t* __restrict__ p, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = (uint32_t)i;
}

__global__ void k_fill_u8(uint8_t* __restrict__ p, int64_t n, uint8_t v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

__global__ void k_widen_flags(const uint8_t* __restrict__ k, int64_t n, uint32_t* __restrict__ f) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) f[i] = k[i] ? 1u : 0u;
}

static int grid_blocks(int64_t n) { return (int)std::max<int64_t>(1, (n + 255) / 256); }

// ---- survivor ranks straight from the keep bytes (the merge rebuild's
// exclusive prefix count of the stored points): per-tile counts, one
// workgroup's scan of the tile counts, then each tile's ranks -- 10 + 10 MB
// read and 40 MB written for the 10M map (the flags widened to 32 bits and a
// device-wide scan moved ~170 MB in ~110 us)
constexpr int kRankTile = 4096;  // keep bytes per workgroup: 256 threads x 16
__device__ __forceinline__ uint32_t nz_bytes(uint32_t w) {  // per byte: 0x80 when non-zero
  return (((w & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | w) & 0x80808080u;
}
__device__ __forceinline__ uint4 load_keep16(const uint8_t* __restrict__ keep, int64_t i, int64_t n) {
  if (i + 16 <= n) return *reinterpret_cast<const uint4*>(keep + i);
  uint32_t w[4] = {0, 0, 0, 0};
  for (int b = 0; b < 16 && i + b < n; ++b) w[b >> 2] |= (uint32_t)(keep[i + b] != 0) << (8 * (b & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}
// block-wide exclusive sum of one value per thread (256 threads); *total gets the sum
__device__ __forceinline__ uint32_t block_excl_256(uint32_t v, uint32_t* total) {
  __shared__ uint32_t ws[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t s = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t u = __shfl_up(s, d, 64);
    if (lane >= d) s += u;
  }
  if (lane == 63) ws[w] = s;
  __syncthreads();
  uint32_t off = 0;
  for (int k = 0; k < w; ++k) off += ws[k];
  if (total) *total = ws[0] + ws[1] + ws[2] + ws[3];
  __syncthreads();
  return off + s - v;
}
// tcnt[t] = tile t's survivors; tcnt[nt + 1], tcnt[nt + 2] zeroed (k_merge_keys'
// live count and edge flag)
__global__ __launch_bounds__(256) void k_keep_tiles(const uint8_t* __restrict__ keep, int64_t n, int64_t nt,
                                                    uint32_t* __restrict__ tcnt) {
  const uint4 v = load_keep16(keep, (int64_t)blockIdx.x * kRankTile + threadIdx.x * 16, n);
  const uint32_t c = __popc(nz_bytes(v.x)) + __popc(nz_bytes(v.y)) + __popc(nz_bytes(v.z)) + __popc(nz_bytes(v.w));
  uint32_t tot;
  (void)block_excl_256(c, &tot);
  if (threadIdx.x == 0) tcnt[blockIdx.x] = tot;
  if (blockIdx.x == 0 && threadIdx.x < 2) tcnt[nt + 1 + threadIdx.x] = 0;
}
// in place: tcnt[0..nt) -> exclusive prefix, tcnt[nt] = the total (one
// workgroup: O(nt); summing the earlier tiles' counts in every rank
// workgroup instead was O(nt^2) -- 73M loads for a 50M map)
__global__ __launch_bounds__(256) void k_tile_scan(uint32_t* __restrict__ tcnt, int64_t nt) {
  const int64_t per = (nt + 255) / 256, a = min((int64_t)threadIdx.x * per, nt), b = min(a + per, nt);
  uint32_t s = 0;
  for (int64_t i = a; i < b; ++i) s += tcnt[i];
  uint32_t tot;
  uint32_t run = block_excl_256(s, &tot);
  for (int64_t i = a; i < b; ++i) {
    const uint32_t v = tcnt[i];
    tcnt[i] = run;
    run += v;
  }
  if (threadIdx.x == 0) tcnt[nt] = tot;
}
// rank[i] = survivors before i: the tile's base plus the exclusive count
// within the tile
__global__ __launch_bounds__(256) void k_keep_rank(const uint8_t* __restrict__ keep, int64_t n,
                                                   const uint32_t* __restrict__ tbase, uint32_t* __restrict__ rank) {
  const int64_t i0 = (int64_t)blockIdx.x * kRankTile + threadIdx.x * 16;
  const uint4 v = load_keep16(keep, i0, n);
  const uint32_t m[4] = {nz_bytes(v.x), nz_bytes(v.y), nz_bytes(v.z), nz_bytes(v.w)};
  const uint32_t c = __popc(m[0]) + __popc(m[1]) + __popc(m[2]) + __popc(m[3]);
  uint32_t r = tbase[blockIdx.x] + block_excl_256(c, nullptr);
  uint32_t o[16];
#pragma unroll
  for (int b = 0; b < 16; ++b) {
    o[b] = r;
    r += (m[b >> 2] >> (8 * (b & 3) + 7)) & 1u;
  }
  if (i0 + 16 <= n) {
    uint4* d = reinterpret_cast<uint4*>(rank + i0);
#pragma unroll
    for (int q = 0; q < 4; ++q) d[q] = make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
  } else {
    for (int b = 0; b < 16 && i0 + b < n; ++b) rank[i0 + b] = o[b];
  }
}

// Build the grid index of m from the n points in `in` (device, x y z
// bits(id), any order, all ids distinct) with bounding box mn / mx: the cell
// table, the cell-sorted points, the coarse level and (speed only) the
// block rows; keep flags all set.  m's index arrays must be empty.
// block rows wanted: not disabled, positions fit 32 bits
static bool block_rows_wanted(const MapDev& m) {
  const char* nb9 = std::getenv("SLIO_NO_BLOCK_ROWS");
  return !(nb9 && nb9[0] && nb9[0] != '0') && m.n > 0 && 9 * m.n < (int64_t)0xFFFFFFF0ll;
}

// Block rows of m's current index (speed only: on any failure the map just
// goes without them).  The views are published after the stream has
// finished them, so a handle sharing the map sees either no block rows or
// complete ones.
static int build_blk(MapDev& m, hipStream_t st, const char* who) {
  m.blk_deferred = false;
  const GridGeom g = m.g;
  const int64_t nseg = (int64_t)((g.dx + kBlkSeg - 1) / kBlkSeg) * g.dy * g.dz;
  size_t t3 = 0;
  hipError_t e;
  if ((e = hipcub::DeviceScan::ExclusiveSum(nullptr, t3, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                            (int)(m.ncells + 1), st)) ||
      (e = m.take(m.b_tmp[6], 4 * (m.ncells + 1))) || (e = m.take(m.b_tmp[7], t3)) ||
      (e = m.take(m.b_bstart, sizeof(uint32_t) * (m.ncells + 1)))) {
    (void)hipGetLastError();
    return SLIO_OK;
  }
  uint32_t* cnt = (uint32_t*)m.b_tmp[6].p;
  uint32_t* bstart = (uint32_t*)m.b_bstart.p;
  if ((e = m.take(m.b_tmp[5], 2 * nseg))) {
    (void)hipGetLastError();
    return SLIO_OK;
  }
  uint16_t* live = (uint16_t*)m.b_tmp[5].p;
  if ((e = hipMemsetAsync(cnt + m.ncells, 0, 4, st))) {
    set_error(std::string(who) + ": block rows: " + hipGetErrorString(e));
    return SLIO_EDEVICE;
  }
  k_blk_live<<<grid_blocks(nseg), 256, 0, st>>>(m.start, g, nseg, live);
  k_blk_count<<<grid_blocks(m.ncells), 256, 0, st>>>(m.start, live, g, m.ncells, cnt);
  size_t tb = m.b_tmp[7].cap;
  if ((e = hipcub::DeviceScan::ExclusiveSum(m.b_tmp[7].p, tb, cnt, bstart, (int)(m.ncells + 1), st))) {
    set_error(std::string(who) + ": block-row scan: " + hipGetErrorString(e));
    return SLIO_EDEVICE;
  }
  uint32_t total = 0;  // <= 9 n < 2^32 (block_rows_wanted): the scan cannot wrap
  if ((e = hipMemcpyAsync(&total, bstart + m.ncells, sizeof(uint32_t), hipMemcpyDeviceToHost, st)) ||
      (e = hipStreamSynchronize(st))) {
    set_error(std::string(who) + ": block-row total: " + hipGetErrorString(e));
    return SLIO_EDEVICE;
  }
  if (m.take(m.b_blk, sizeof(float4) * std::max<uint32_t>(total, 1u))) {
    (void)hipGetLastError();
    return SLIO_OK;
  }
  k_blk_fill<<<grid_blocks(m.ncells), 256, 0, st>>>(m.pts, m.start, live, bstart, g, m.ncells,
                                                     (float4*)m.b_blk.p);
  if ((e = hipGetLastError()) || (e = hipStreamSynchronize(st))) {
    set_error(std::string(who) + ": block-row kernels: " + hipGetErrorString(e));
    return SLIO_EDEVICE;
  }
  m.bstart = bstart;
  m.nblk = (int64_t)total;
  m.blk = (float4*)m.b_blk.p;
  return SLIO_OK;
}

// in_id_order: `in` is the map's previous cell-sorted points (survivors, in
// their stored order) followed by points with larger ids in id order -- then,
// when the grid comes out the same as before (or the map was empty), a STABLE
// sort by cell alone yields (cell, id) order, and the 32-bit cell key needs
// about half the radix passes of the 64-bit (cell, id) key.
static int build_index(MapDev& m, const float4* in, int64_t n, const float mn[3], const float mx[3],
                       hipStream_t st, const char* who, bool with_blk = true, bool in_id_order = false,
                       bool had_points = false) {
  m.blk_deferred = false;
  const GridGeom g_old = m.g;
  GridGeom g;
  // cell edge: the caller's, or auto (cell0 == 0): 1.0 m -- the best edge for the
  // 10M-point, 0.5 m map (cell edge) -- unless that grid has more
  // than 2^27 cells, whose tables overflow the Infinity Cache and slow every
  // query's first loads: then 1.25 m (the 50M-point map's best)
  const bool auto_cell = !(m.cell0 > 0.0f);
  float hcell = auto_cell ? 1.0f : m.cell0;
  // kGridPad empty cells around the map's bounding box: scan points just
  // outside it (ground returns below a flat map's lowest point, range noise)
  // still get a query cell inside the grid, so they take the 3x3x3 fast path
  // A rebuild keeps the previous grid while the points still lie at least one
  // cell inside it (the grid need not be tight: every bound is conservative),
  // so the cell-only sort below applies; when they do not, the new grid gets
  // twice the padding, and a map growing slowly at an edge re-grids rarely.
  const int kGridPad = in_id_order ? 4 : 2;
  bool keep_grid = in_id_order && had_points;
  if (keep_grid) {
    const float o[3] = {g_old.ox, g_old.oy, g_old.oz};
    const int d[3] = {g_old.dx, g_old.dy, g_old.dz};
    for (int a = 0; a < 3; ++a)
      keep_grid = keep_grid && mn[a] >= o[a] + g_old.h && mx[a] <= o[a] + (float)(d[a] - 1) * g_old.h;
  }
  for (; !keep_grid;) {
    g.ox = mn[0] - kGridPad * hcell;
    g.oy = mn[1] - kGridPad * hcell;
    g.oz = mn[2] - kGridPad * hcell;
    g.h = hcell;
    g.inv_h = 1.0f / hcell;
    g.dx = cell_coord(mx[0], g.ox, g.inv_h) + 1 + kGridPad;
    g.dy = cell_coord(mx[1], g.oy, g.inv_h) + 1 + kGridPad;
    g.dz = cell_coord(mx[2], g.oz, g.inv_h) + 1 + kGridPad;
    const int64_t nc = (int64_t)g.dx * g.dy * g.dz;
    if (auto_cell && hcell == 1.0f && nc > ((int64_t)1 << 27)) {
      hcell = 1.25f;
      continue;
    }
    if (nc <= m.max_cells && nc < (int64_t)0xFFFFFFF0ll) break;
    hcell *= 1.25f;  // grow cells until the dense table fits the budget
  }
  if (keep_grid) g = g_old;
  // largest |coordinate| a cell face can have: |origin| + dims * h per axis
  // (kept grid: the same tol as before)
  const float mag = std::max(std::fabs(g.ox) + (float)g.dx * g.h,
                             std::max(std::fabs(g.oy) + (float)g.dy * g.h, std::fabs(g.oz) + (float)g.dz * g.h));
  g.tol = mag * 3.814697265625e-06f + 1.0e-5f;  // 2^-18 relative: >= 64 ulps
  const bool cell_only =
      in_id_order && (!had_points || (g.ox == g_old.ox && g.oy == g_old.oy && g.oz == g_old.oz &&
                                      g.h == g_old.h && g.dx == g_old.dx && g.dy == g_old.dy &&
                                      g.dz == g_old.dz));
  if (in_id_order && std::getenv("SLIO_DEBUG_REBUILD"))
    std::fprintf(stderr, "slio rebuild: n %lld cell_only %d grid %d %d %d (was %d %d %d) origin %.6g %.6g %.6g (was %.6g %.6g %.6g)\n",
                 (long long)n, (int)cell_only, g.dx, g.dy, g.dz, g_old.dx, g_old.dy, g_old.dz, g.ox, g.oy, g.oz,
                 g_old.ox, g_old.oy, g_old.oz);
  m.g = g;
  m.n = n;
  m.ncells = (int64_t)g.dx * g.dy * g.dz;
  // coarse level geometry (cells of edge 4h on the same origin)
  GridGeom cg = g;
  cg.h = 4.0f * g.h;
  cg.inv_h = 1.0f / cg.h;
  cg.dx = (g.dx + 3) / 4;
  cg.dy = (g.dy + 3) / 4;
  cg.dz = (g.dz + 3) / 4;
  m.cg = cg;
  m.nccells = (int64_t)cg.dx * cg.dy * cg.dz;

  auto fail = [&](const char* what, hipError_t e) {
    set_error(std::string(who) + ": " + what + ": " + hipGetErrorString(e));
    return e == hipErrorOutOfMemory ? SLIO_ENOMEM : SLIO_EDEVICE;
  };
  hipError_t e;
  if ((e = m.take(m.b_start, sizeof(uint32_t) * (m.ncells + 1))) ||
      (e = m.take(m.b_clo, sizeof(float4) * m.nccells)) || (e = m.take(m.b_chi, sizeof(float4) * m.nccells)))
    return fail("hipMalloc", e);
  m.start = (uint32_t*)m.b_start.p;
  m.clo = (float4*)m.b_clo.p;
  m.chi = (float4*)m.b_chi.p;
  if (n == 0) {
    if ((e = hipMemsetAsync(m.start, 0, sizeof(uint32_t) * (m.ncells + 1), st)) ||
        (e = hipMemsetAsync(m.clo, 0, sizeof(float4) * m.nccells, st)) || (e = hipStreamSynchronize(st)))
      return fail("empty map", e);
    return SLIO_OK;
  }
  if ((e = m.take(m.b_pts, sizeof(float4) * n)) || (e = m.take(m.b_keep, n)))
    return fail("hipMalloc", e);
  m.pts = (float4*)m.b_pts.p;
  m.keep = (uint8_t*)m.b_keep.p;
  uint64_t *k0 = nullptr, *k1 = nullptr;
  uint32_t *v0 = nullptr, *v1 = nullptr, *cnt = nullptr, *c0 = nullptr, *c1 = nullptr;
  void* tmp = nullptr;
  int rc = SLIO_OK;
  const int64_t maxc = std::max(m.ncells, m.nccells) + 1;
  do {
    if ((e = m.take(m.b_tmp[0], 8 * n)) || (e = m.take(m.b_tmp[1], 8 * n)) || (e = m.take(m.b_tmp[2], 4 * n)) ||
        (e = m.take(m.b_tmp[3], 4 * n)) || (e = m.take(m.b_tmp[4], 4 * n)) || (e = m.take(m.b_tmp[5], 4 * n)) ||
        (e = m.take(m.b_tmp[6], 4 * maxc))) {
      rc = fail("hipMalloc", e);
      break;
    }
    k0 = (uint64_t*)m.b_tmp[0].p;
    k1 = (uint64_t*)m.b_tmp[1].p;
    v0 = (uint32_t*)m.b_tmp[2].p;
    v1 = (uint32_t*)m.b_tmp[3].p;
    c0 = (uint32_t*)m.b_tmp[4].p;
    c1 = (uint32_t*)m.b_tmp[5].p;
    cnt = (uint32_t*)m.b_tmp[6].p;
    int idbits = 1;
    while (idbits < 32 && ((int64_t)1 << idbits) <= (int64_t)m.next_id) ++idbits;
    int cbits = 1;
    while (cbits < 32 && ((int64_t)1 << cbits) < m.ncells) ++cbits;
    int ccbits = 1;
    while (ccbits < 32 && ((int64_t)1 << ccbits) < m.nccells) ++ccbits;
    size_t t1 = 0, t2 = 0, t3 = 0, t4 = 0, t5 = 0;
    if ((e = hipcub::DeviceRadixSort::SortPairs(nullptr, t1, k0, k1, v0, v1, (int)n, 0, idbits + cbits, st)) ||
        (e = hipcub::DeviceRadixSort::SortPairs(nullptr, t2, c0, c1, v0, v1, (int)n, 0, ccbits, st)) ||
        (e = hipcub::DeviceRadixSort::SortPairs(nullptr, t5, c0, c1, v0, v1, (int)n, 0, cbits, st)) ||
        (e = hipcub::DeviceScan::ExclusiveSum(nullptr, t3, cnt, m.start, (int)maxc, st))) {
      rc = fail("sort size", e);
      break;
    }
    t4 = std::max(std::max(std::max(t1, t2), t3), t5);
    if ((e = m.take(m.b_tmp[7], t4))) {
      rc = fail("hipMalloc tmp", e);
      break;
    }
    tmp = m.b_tmp[7].p;
    const int nb = grid_blocks(n);
    if (cell_only) {
      k_coarse_keys<<<nb, 256, 0, st>>>(in, n, g, c0, v0);  // fine cell keys (same formula)
      if ((e = hipcub::DeviceRadixSort::SortPairs(tmp, t4, c0, c1, v0, v1, (int)n, 0, cbits, st)) ||
          (e = hipMemsetAsync(cnt, 0, 4 * (m.ncells + 1), st))) {
        rc = fail("sort", e);
        break;
      }
      k_cell_hist_sorted<uint32_t><<<nb, 256, 0, st>>>(c1, n, 0, cnt);
    } else {
      k_cell_keys64<<<nb, 256, 0, st>>>(in, n, g, idbits, k0, v0);
      if ((e = hipcub::DeviceRadixSort::SortPairs(tmp, t4, k0, k1, v0, v1, (int)n, 0, idbits + cbits, st)) ||
          (e = hipMemsetAsync(cnt, 0, 4 * (m.ncells + 1), st))) {
        rc = fail("sort", e);
        break;
      }
      k_cell_hist_sorted<uint64_t><<<nb, 256, 0, st>>>(k1, n, idbits, cnt);
    }
    if ((e = hipcub::DeviceScan::ExclusiveSum(tmp, t4, cnt, m.start, (int)(m.ncells + 1), st))) {
      rc = fail("scan", e);
      break;
    }
    k_gather4<<<nb, 256, 0, st>>>(in, v1, n, m.pts);
    k_fill_u8<<<nb, 256, 0, st>>>(m.keep, n, 1);
    // coarse level from the fine cell table (k_coarse_count / k_coarse_boxes:
    // no sort), tight boxes
    k_coarse_count<<<grid_blocks(m.nccells), 256, 0, st>>>(m.start, g, cg, m.nccells, cnt);
    k_coarse_boxes<<<grid_blocks(m.nccells), 256, 0, st>>>(m.pts, m.start, g, cg, cnt, m.nccells, m.clo,
                                                                   m.chi);
    m.del_loose = 0;
    if ((e = hipGetLastError()) || (e = hipStreamSynchronize(st))) {
      rc = fail("build kernels", e);
      break;
    }
    // block rows (speed only): now for an uploaded map; a map rebuilt by
    // the live-map maintenance gets them once it has stopped changing
    m.blk_deferred = block_rows_wanted(m);
    m.stable_passes = 0;
    if (with_blk && m.blk_deferred) rc = build_blk(m, st, who);
  } while (0);
#ifdef SLIO_BOUNDS_CHECK
  if (!rc) {
    const int64_t nc = m.ncells;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(c_dbg_npts), &n, sizeof(n));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(c_dbg_ncells), &nc, sizeof(nc));
  }
#endif
  return rc;
}

static int ensure_scan_buffers(Ctx& c) {
  if (!c.bx) {
    const int64_t cap = c.prm.max_points;
    const int64_t capc = num_chunks(cap) + 1;
    hipError_t e;
    if ((e = hipMalloc(&c.bx, 4 * cap)) || (e = hipMalloc(&c.by, 4 * cap)) ||
        (e = hipMalloc(&c.bz, 4 * cap)) || (e = hipMalloc(&c.nbr_idx, 4 * 5 * cap)) ||
        (e = hipMalloc(&c.nbr_pos, 4 * 5 * cap)) || (e = hipMalloc(&c.nbr_pose, sizeof(PoseDev))) ||
        (e = hipMalloc(&c.nbr_sqd, 4 * 5 * cap)) || (e = hipMalloc(&c.plane, 16 * cap)) ||
        (e = hipMalloc(&c.sel, cap)) || (e = hipMalloc(&c.resid, 4 * cap)) ||
        (e = hipMalloc(&c.chunk_part, 8 * SLIO_NPROD * capc)) ||
        (e = hipMalloc(&c.chunk_cost, 4 * capc)) || (e = hipMalloc(&c.chunk_perm, 4 * capc)) ||
        (e = hipMalloc(&c.kq, 16 * cap)) || (e = hipMalloc(&c.k6, 4 * cap)) ||
        (e = hipMalloc(&c.kepoch, 4 * capc)) || (e = hipMemset(c.kepoch, 0, 4 * capc))) {
      free_scan(&c);
      set_error(std::string("slio scan buffers: hipMalloc: ") + hipGetErrorString(e));
      return SLIO_ENOMEM;
    }
    k_iota_u32<<<grid_blocks(capc), 256, 0, c.stream>>>(c.chunk_perm, capc);
    SLIO_HIP(hipMemsetAsync(c.chunk_cost, 0, 4 * capc, c.stream));
  }
  return SLIO_OK;
}

// ---------------------------------------------------------------- map maintenance
// Device mirror of the map changes laserMapping makes every scan
// (map_incremental laserMapping.cpp:382-433, KD_TREE::Add_Points
// ikd_Tree.cpp:419-512, Delete_Point_Boxes ikd_Tree.cpp:559-579), with the
// set semantics the oracle (oracle/map_oracle.cpp) restates.

__device__ __forceinline__ float map_dist(float ax, float ay, float az, float bx, float by, float bz) {
  // calc_dist (ikd_Tree.cpp:1539-1544, common_lib.h:86-90)
  return (ax - bx) * (ax - bx) + (ay - by) * (ay - by) + (az - bz) * (az - bz);
}
__device__ __forceinline__ bool map_same(float ax, float ay, float az, float bx, float by, float bz) {
  // same_point (ikd_Tree.cpp:1533-1536), EPSS 1e-6
  return fabsf(ax - bx) < 1e-6 && fabsf(ay - by) < 1e-6 && fabsf(az - bz) < 1e-6;
}

// Delete_Point_Boxes: half-open boxes [min, max) (the Delete_by_range
// predicate); boxes in constant-size batches
struct Boxes8 {
  float b[8][6];
  int n;
};
__global__ void k_map_delete(const float4* __restrict__ pts, uint8_t* __restrict__ keep, int64_t n, Boxes8 bx,
                             unsigned long long* __restrict__ count) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool del = false;
  if (i < n && keep[i]) {
    const float4 p = pts[i];
    for (int k = 0; k < bx.n; ++k) {
      const float* b = bx.b[k];
      if (b[0] <= p.x && b[3] > p.x && b[1] <= p.y && b[4] > p.y && b[2] <= p.z && b[5] > p.z) del = true;
    }
    if (del) keep[i] = 0;
  }
  const unsigned long long m = __ballot(del);
  if ((threadIdx.x & 63) == 0 && m) atomicAdd(count, (unsigned long long)__popcll(m));
}

// downsample voxel key of a point: the three floor(p / ds) (ikd_Tree.cpp:430-441)
__device__ __forceinline__ uint64_t ds_key(int64_t kx, int64_t ky, int64_t kz) {
  return ((uint64_t)((kx + (1 << 20)) & 0x1FFFFF) << 42) | ((uint64_t)((ky + (1 << 20)) & 0x1FFFFF) << 21) |
         (uint64_t)((kz + (1 << 20)) & 0x1FFFFF);
}

// the call's voxel-key range per axis (atomic min / max of floor(p / ds),
// reduced per wavefront first)
__global__ void k_ds_range(const float4* __restrict__ in, int64_t n, float ds, int32_t* __restrict__ rg) {
  int32_t lo[3] = {INT32_MAX, INT32_MAX, INT32_MAX}, hi[3] = {INT32_MIN, INT32_MIN, INT32_MIN};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 p = in[i];
    const int32_t k[3] = {(int32_t)floorf(p.x / ds), (int32_t)floorf(p.y / ds), (int32_t)floorf(p.z / ds)};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      lo[a] = min(lo[a], k[a]);
      hi[a] = max(hi[a], k[a]);
    }
  }
#pragma unroll
  for (int a = 0; a < 3; ++a)
    for (int d = 32; d > 0; d >>= 1) {
      lo[a] = min(lo[a], __shfl_xor(lo[a], d, 64));
      hi[a] = max(hi[a], __shfl_xor(hi[a], d, 64));
    }
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      atomicMin(&rg[a], lo[a]);
      atomicMax(&rg[3 + a], hi[a]);
    }
}
// keys packed relative to the call's range (groups by equality only)
struct DsPack {
  int32_t mx, my, mz;
  int sy, sz;  // shifts of the x and y fields
};
__global__ void k_ds_keys_packed(const float4* __restrict__ in, int64_t n, float ds, DsPack pk,
                                 uint64_t* __restrict__ keys, uint32_t* __restrict__ vals) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 p = in[i];
  const uint64_t kx = (uint64_t)((int64_t)(int32_t)floorf(p.x / ds) - pk.mx);
  const uint64_t ky = (uint64_t)((int64_t)(int32_t)floorf(p.y / ds) - pk.my);
  const uint64_t kz = (uint64_t)((int64_t)(int32_t)floorf(p.z / ds) - pk.mz);
  keys[i] = (kx << pk.sy) | (ky << pk.sz) | kz;
  vals[i] = (uint32_t)i;
}

__global__ void k_ds_keys(const float4* __restrict__ in, int64_t n, float ds, uint64_t* __restrict__ keys,
                          uint32_t* __restrict__ vals) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 p = in[i];
  const int64_t kx = (int64_t)floorf(p.x / ds), ky = (int64_t)floorf(p.y / ds), kz = (int64_t)floorf(p.z / ds);
  keys[i] = ds_key(kx, ky, kz);
  vals[i] = (uint32_t)i;
}

// The downsample box of key (kx, ky, kz): [floor * ds, floor * ds + ds) per
// axis in float, as Add_Points forms it from a point of that key
// (ikd_Tree.cpp:430-441); Search_by_range's predicate is half-open
// (:1127-1128).  For a downsample size that is not a power of two,
// neighbouring float boxes can overlap by an ulp (or leave an ulp gap).
struct DsBox {
  float lo[3], hi[3];
};
__device__ __forceinline__ DsBox ds_box(int64_t kx, int64_t ky, int64_t kz, float ds) {
  DsBox b;
  const int64_t k[3] = {kx, ky, kz};
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    b.lo[a] = (float)k[a] * ds;
    b.hi[a] = b.lo[a] + ds;
  }
  return b;
}
__device__ __forceinline__ bool ds_inside(const DsBox& b, float x, float y, float z) {
  return b.lo[0] <= x && b.hi[0] > x && b.lo[1] <= y && b.hi[1] > y && b.lo[2] <= z && b.hi[2] > z;
}
__device__ __forceinline__ int64_t ds_find(const uint64_t* __restrict__ keys, int64_t n, uint64_t k) {
  int64_t a = 0, b = n;  // first index with keys[i] >= k
  while (a < b) {
    const int64_t m = (a + b) >> 1;
    if (keys[m] < k) a = m + 1; else b = m;
  }
  return (a < n && keys[a] == k) ? a : -1;
}
// p lies in the box of a key other than `own` that this call also holds a
// point of (the boxes of the 27 keys around p's own key)
__device__ __forceinline__ bool ds_shared(float x, float y, float z, uint64_t own, float ds,
                                          const uint64_t* __restrict__ keys, int64_t n) {
  const int64_t kx = (int64_t)floorf(x / ds), ky = (int64_t)floorf(y / ds), kz = (int64_t)floorf(z / ds);
  for (int dz = -1; dz <= 1; ++dz)
    for (int dy = -1; dy <= 1; ++dy)
      for (int dx = -1; dx <= 1; ++dx) {
        const uint64_t k = ds_key(kx + dx, ky + dy, kz + dz);
        if (k == own || !ds_inside(ds_box(kx + dx, ky + dy, kz + dz, ds), x, y, z)) continue;
        if (ds_find(keys, n, k) >= 0) return true;
      }
  return false;
}

// Groups are independent (k_ds_groups) unless some point -- stored and alive
// in a group's box, or one of the call's new points -- lies in the boxes of
// two keys of this call (float boxes overlapping by an ulp, or a new point
// past its own box's upper face inside the next box), or a new point lies
// outside its own box (an ulp gap): then the call's sequential order
// matters.  One thread per group; flag[0] = 1 on any.
__global__ void k_ds_conflicts(const float4* __restrict__ in, const uint64_t* __restrict__ keys,
                               const uint32_t* __restrict__ order, int64_t n, float ds, MapView map,
                               const uint8_t* __restrict__ keep, unsigned long long* __restrict__ flag) {
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i0 >= n || (i0 > 0 && keys[i0] == keys[i0 - 1])) return;
  const uint64_t own = keys[i0];
  bool hit = false;
  {
    const float4 q0 = in[order[i0]];
    const DsBox ob = ds_box((int64_t)floorf(q0.x / ds), (int64_t)floorf(q0.y / ds), (int64_t)floorf(q0.z / ds), ds);
    for (int64_t j = i0; j < n && keys[j] == own && !hit; ++j) {
      const float4 q = in[order[j]];
      // a new point outside its own box (an ulp gap past the upper face):
      // the group's later points do not see it (k_ds_groups assumes they do)
      hit = !ds_inside(ob, q.x, q.y, q.z) || ds_shared(q.x, q.y, q.z, own, ds, keys, n);
    }
  }
  if (!hit && map.n > 0) {
    const float4 q0 = in[order[i0]];
    const DsBox bx = ds_box((int64_t)floorf(q0.x / ds), (int64_t)floorf(q0.y / ds), (int64_t)floorf(q0.z / ds), ds);
    const GridGeom g = map.g;
    int ca[3], cb[3];
    const float og[3] = {g.ox, g.oy, g.oz};
    const int dg[3] = {g.dx, g.dy, g.dz};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      ca[a] = min(max(cell_coord(bx.lo[a], og[a], g.inv_h), 0), dg[a] - 1);
      cb[a] = min(max(cell_coord(bx.hi[a], og[a], g.inv_h), 0), dg[a] - 1);
    }
    for (int z = ca[2]; z <= cb[2] && !hit; ++z)
      for (int y = ca[1]; y <= cb[1] && !hit; ++y) {
        const uint32_t rb = ((uint32_t)z * (uint32_t)g.dy + (uint32_t)y) * (uint32_t)g.dx;
        for (uint32_t ps = map.start[rb + ca[0]]; ps < map.start[rb + cb[0] + 1] && !hit; ++ps) {
          if (!keep[ps]) continue;
          const float4 p = map.pts[ps];
          if (ds_inside(bx, p.x, p.y, p.z)) hit = ds_shared(p.x, p.y, p.z, own, ds, keys, n);
        }
      }
  }
  if (hit) atomicExch(flag, 1ull);
}

// The call's exact sequential Add_Points (ikd_Tree.cpp:428-512, the set
// restatement of oracle/map_oracle.cpp) by ONE thread, point by point in list
// order, for a call whose groups interact (k_ds_conflicts): stored points in
// storage order (ascending id), then this call's earlier survivors in list
// order; the new point wins ties, a stored one only when strictly nearer.
// Slow (one thread) and rare: only ulp-wide float overlaps of downsample
// boxes can interact, and only for a size that is not a power of two.
__global__ void k_ds_sequential(const float4* __restrict__ in, const uint64_t* __restrict__ keys,
                                const uint32_t* __restrict__ order, int64_t n, float ds, MapView map,
                                uint8_t* __restrict__ keep, uint32_t* __restrict__ surv,
                                unsigned long long* __restrict__ counter) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  const GridGeom g = map.g;
  const float og[3] = {g.ox, g.oy, g.oz};
  const int dg[3] = {g.dx, g.dy, g.dz};
  unsigned long long ops = 0;
  for (int64_t li = 0; li < n; ++li) {
    const float4 q = in[li];
    const int64_t kx = (int64_t)floorf(q.x / ds), ky = (int64_t)floorf(q.y / ds), kz = (int64_t)floorf(q.z / ds);
    const DsBox bx = ds_box(kx, ky, kz, ds);
    const float mx = (float)((double)bx.lo[0] + (double)(bx.hi[0] - bx.lo[0]) / 2.0);
    const float my = (float)((double)bx.lo[1] + (double)(bx.hi[1] - bx.lo[1]) / 2.0);
    const float mz = (float)((double)bx.lo[2] + (double)(bx.hi[2] - bx.lo[2]) / 2.0);
    int ca[3], cb[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      ca[a] = min(max(cell_coord(bx.lo[a], og[a], g.inv_h), 0), dg[a] - 1);
      cb[a] = min(max(cell_coord(bx.hi[a], og[a], g.inv_h), 0), dg[a] - 1);
    }
    // winner: the new point unless a storage entry is strictly nearer; among
    // entries, the first minimum in storage order
    int64_t cnt = 0;
    float bd = map_dist(q.x, q.y, q.z, mx, my, mz);
    int wk = 0;  // 0: the new point, 1: stored (bpos), 2: this call's earlier survivor (blj)
    uint32_t bid = 0;
    int64_t bpos = -1, blj = -1;
    float4 bp = q;
    if (map.n > 0)
      for (int z = ca[2]; z <= cb[2]; ++z)
        for (int y = ca[1]; y <= cb[1]; ++y) {
          const uint32_t rb = ((uint32_t)z * (uint32_t)g.dy + (uint32_t)y) * (uint32_t)g.dx;
          for (uint32_t ps = map.start[rb + ca[0]]; ps < map.start[rb + cb[0] + 1]; ++ps) {
            if (!keep[ps]) continue;
            const float4 p = map.pts[ps];
            if (!ds_inside(bx, p.x, p.y, p.z)) continue;
            ++cnt;
            const float d = map_dist(p.x, p.y, p.z, mx, my, mz);
            const uint32_t id = __float_as_uint(p.w);
            if (d < bd || (wk == 1 && d == bd && id < bid)) {
              bd = d;
              bid = id;
              bpos = ps;
              bp = p;
              wk = 1;
            }
          }
        }
    // earlier survivors of this call inside the box: their keys are among
    // the 27 around q's key; storage order after every stored point, in list order
    for (int dz = -1; dz <= 1; ++dz)
      for (int dy = -1; dy <= 1; ++dy)
        for (int dx = -1; dx <= 1; ++dx) {
          int64_t j = ds_find(keys, n, ds_key(kx + dx, ky + dy, kz + dz));
          if (j < 0) continue;
          const uint64_t k = keys[j];
          for (; j < n && keys[j] == k; ++j) {
            const uint32_t lj = order[j];
            if ((int64_t)lj >= li || !surv[lj]) continue;
            const float4 p = in[lj];
            if (!ds_inside(bx, p.x, p.y, p.z)) continue;
            ++cnt;
            const float d = map_dist(p.x, p.y, p.z, mx, my, mz);
            // strictly nearer than the best so far, or as near as the best
            // earlier survivor but earlier in list order (storage order)
            if (d < bd || (wk == 2 && d == bd && (int64_t)lj < blj)) {
              bd = d;
              blj = lj;
              bp = p;
              wk = 2;
            }
          }
        }
    if (cnt > 1 || map_same(q.x, q.y, q.z, bp.x, bp.y, bp.z)) {
      ++ops;
      // every storage entry but the winner goes
      if (map.n > 0)
        for (int z = ca[2]; z <= cb[2]; ++z)
          for (int y = ca[1]; y <= cb[1]; ++y) {
            const uint32_t rb = ((uint32_t)z * (uint32_t)g.dy + (uint32_t)y) * (uint32_t)g.dx;
            for (uint32_t ps = map.start[rb + ca[0]]; ps < map.start[rb + cb[0] + 1]; ++ps)
              if (keep[ps] && !(wk == 1 && (int64_t)ps == bpos) && ds_inside(bx, map.pts[ps].x, map.pts[ps].y,
                                                                                  map.pts[ps].z))
                keep[ps] = 0;
          }
      for (int dz = -1; dz <= 1; ++dz)
        for (int dy = -1; dy <= 1; ++dy)
          for (int dx = -1; dx <= 1; ++dx) {
            int64_t j = ds_find(keys, n, ds_key(kx + dx, ky + dy, kz + dz));
            if (j < 0) continue;
            const uint64_t k = keys[j];
            for (; j < n && keys[j] == k; ++j) {
              const uint32_t lj = order[j];
              if ((int64_t)lj >= li || !surv[lj] || (wk == 2 && (int64_t)lj == blj)) continue;
              if (ds_inside(bx, in[lj].x, in[lj].y, in[lj].z)) surv[lj] = 0;
            }
          }
      if (wk == 0) surv[li] = 1;
    }
  }
  counter[0] = ops;
}

// One thread per voxel group of the sorted list (the points of one
// Add_Points call that share a downsample box, in list order): the
// sequential rules of Add_Points on the box's stored points and the group's
// points.  Stored points in storage order = ascending id; a stored point
// wins only when strictly nearer the box centre (ties: the lower id).
// One downsample group (the points of one voxel key) against the stored
// map, in list order -- the sequential rules of Add_Points (ikd_Tree.cpp:
// 428-512) for a group no other group interacts with.  member(j) is the
// list index of the group's j-th point in list order, j < m.
template <typename Member>
__device__ __forceinline__ void ds_group(const float4* __restrict__ in, float ds, const MapView& map,
                                         uint8_t* __restrict__ keep, uint32_t* __restrict__ surv,
                                         unsigned long long* __restrict__ counter, int64_t m, Member member) {
  const uint32_t li0 = member(0);
  const float4 q0 = in[li0];
  float lo[3], hi[3];
  const float c0[3] = {q0.x, q0.y, q0.z};
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    lo[a] = floorf(c0[a] / ds) * ds;
    hi[a] = lo[a] + ds;
  }
  const float mx = (float)((double)lo[0] + (double)(hi[0] - lo[0]) / 2.0);
  const float my = (float)((double)lo[1] + (double)(hi[1] - lo[1]) / 2.0);
  const float mz = (float)((double)lo[2] + (double)(hi[2] - lo[2]) / 2.0);
  const GridGeom g = map.g;
  int ca[3], cb[3];
  const float og[3] = {g.ox, g.oy, g.oz};
  const int dg[3] = {g.dx, g.dy, g.dz};
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    ca[a] = min(max(cell_coord(lo[a], og[a], g.inv_h), 0), dg[a] - 1);
    cb[a] = min(max(cell_coord(hi[a], og[a], g.inv_h), 0), dg[a] - 1);
  }
  auto inside = [&](const float4& p) {
    return lo[0] <= p.x && hi[0] > p.x && lo[1] <= p.y && hi[1] > p.y && lo[2] <= p.z && hi[2] > p.z;
  };
  // stored points in the box: count and the one nearest the centre
  int64_t cnt = 0;
  float bd = 0.0f;
  uint32_t bid = 0xFFFFFFFFu;
  int64_t bpos = -1;
  float4 bp = make_float4(0, 0, 0, 0);
  if (map.n > 0)
    for (int z = ca[2]; z <= cb[2]; ++z)
      for (int y = ca[1]; y <= cb[1]; ++y) {
        const uint32_t rb = ((uint32_t)z * (uint32_t)g.dy + (uint32_t)y) * (uint32_t)g.dx;
        for (uint32_t ps = map.start[rb + ca[0]]; ps < map.start[rb + cb[0] + 1]; ++ps) {
          if (!keep[ps]) continue;
          const float4 p = map.pts[ps];
          if (!inside(p)) continue;
          ++cnt;
          const float d = map_dist(p.x, p.y, p.z, mx, my, mz);
          const uint32_t id = __float_as_uint(p.w);
          if (bpos < 0 || d < bd || (d == bd && id < bid)) {
            bd = d;
            bid = id;
            bpos = ps;
            bp = p;
          }
        }
      }
  // the group's points, in list order
  bool orig_all = true;       // every stored point still alive
  int64_t orig_keep = -1;     // else: the one stored point kept (or none)
  int64_t cur_new = -1;       // list index of this call's surviving new point
  bool best_new = false;
  unsigned long long ops = 0;
  for (int64_t j = 0; j < m; ++j) {
    const uint32_t li = j == 0 ? li0 : member(j);  // member() is called once per j, in order
    const float4 q = in[li];
    const float dq = map_dist(q.x, q.y, q.z, mx, my, mz);
    const bool stored_wins = cnt > 0 && bd < dq;
    const float4 w = stored_wins ? bp : q;
    if (cnt > 1 || map_same(q.x, q.y, q.z, w.x, w.y, w.z)) {
      ++ops;
      if (!stored_wins) {
        orig_all = false;
        orig_keep = -1;
        cur_new = li;
        best_new = true;
        bd = dq;
        bp = q;
      } else if (!best_new && orig_all) {
        orig_all = false;
        orig_keep = bpos;
      }
      cnt = 1;
    }
  }
  if (!orig_all && map.n > 0)
    for (int z = ca[2]; z <= cb[2]; ++z)
      for (int y = ca[1]; y <= cb[1]; ++y) {
        const uint32_t rb = ((uint32_t)z * (uint32_t)g.dy + (uint32_t)y) * (uint32_t)g.dx;
        for (uint32_t ps = map.start[rb + ca[0]]; ps < map.start[rb + cb[0] + 1]; ++ps)
          if (keep[ps] && (int64_t)ps != orig_keep && inside(map.pts[ps])) keep[ps] = 0;
      }
  if (cur_new >= 0) surv[cur_new] = 1;
  if (ops) atomicAdd(counter, ops);
}

// groups from the keys sorted stably (keys, order = list indices): one
// thread per group head
__global__ void k_ds_groups(const float4* __restrict__ in, const uint64_t* __restrict__ keys,
                            const uint32_t* __restrict__ order, int64_t n, float ds, MapView map,
                            uint8_t* __restrict__ keep, uint32_t* __restrict__ surv,
                            unsigned long long* __restrict__ counter) {
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i0 >= n || (i0 > 0 && keys[i0] == keys[i0 - 1])) return;
  if (counter[1]) return;  // interacting groups: k_ds_sequential instead
  int64_t m = 1;
  while (i0 + m < n && keys[i0 + m] == keys[i0]) ++m;
  ds_group(in, ds, map, keep, surv, counter, m, [&](int64_t j) { return order[i0 + j]; });
}

// Grouping without a sort (exact boxes: groups are independent and need no
// global order, only their own points in list order).  Open-addressing hash
// of the voxel key (ds_key) into H = 2^hb slots: each point claims or finds
// its key's slot (atomicCAS), takes a member position (atomicAdd) and stores
// its list index there (up to kDsInline per slot); a slot with more members
// rescans the list for its key (rare: a 0.5 m voxel of a downsampled scan).
// A key outside ds_key's 21-bit range sets *flag (counter[2] of the groups
// kernel): the caller then takes the sorting path.
constexpr int kDsInline = 16;
constexpr uint64_t kDsEmpty = ~0ull;
// (nl: when set, the list holds nl[0] + nl[1] points -- an exclusive scan's
// last rank and flag -- of the n it has room for)
__global__ void k_ds_hash(const float4* __restrict__ in, int64_t n, float ds, int hb, uint64_t* __restrict__ hkey,
                          uint32_t* __restrict__ hcnt, uint32_t* __restrict__ hmem,
                          unsigned long long* __restrict__ flag, const uint32_t* __restrict__ nl_rank = nullptr,
                          const uint32_t* __restrict__ nl_flag = nullptr) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (nl_rank ? (int64_t)(*nl_rank + *nl_flag) : n)) return;
  const float4 p = in[i];
  const int64_t kx = (int64_t)floorf(p.x / ds), ky = (int64_t)floorf(p.y / ds), kz = (int64_t)floorf(p.z / ds);
  constexpr int64_t kLim = (1 << 20) - 1;
  if (kx < -kLim || kx > kLim || ky < -kLim || ky > kLim || kz < -kLim || kz > kLim) {
    atomicExch(flag, 1ull);
    return;
  }
  const uint64_t key = ds_key(kx, ky, kz);
  const uint64_t mask = ((uint64_t)1 << hb) - 1;
  uint64_t h = (key * 0x9E3779B97F4A7C15ull) >> (64 - hb);
  for (;;) {
    const unsigned long long prev = atomicCAS((unsigned long long*)&hkey[h], kDsEmpty, key);
    if (prev == kDsEmpty || prev == key) break;
    h = (h + 1) & mask;
  }
  const uint32_t pos = atomicAdd(&hcnt[h], 1u);
  if (pos < (uint32_t)kDsInline) hmem[h * kDsInline + pos] = (uint32_t)i;
}

// the hash table emptied, survivor flags and counters zeroed: one launch
// (four fills were four launches in a row)
__global__ void k_ds_init(uint64_t* __restrict__ hkey, uint32_t* __restrict__ hcnt, int64_t H,
                          uint32_t* __restrict__ surv, int64_t n, unsigned long long* __restrict__ dcount) {
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, st = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = i0; i < H; i += st) {
    hkey[i] = kDsEmpty;
    hcnt[i] = 0;
  }
  for (int64_t i = i0; i < n; i += st) surv[i] = 0;
  if (i0 < 3) dcount[i0] = 0;
}

// one thread per occupied slot: its members sorted into list order, then
// ds_group
__global__ void k_ds_groups_hash(const float4* __restrict__ in, int64_t n, float ds, int hb,
                                 const uint64_t* __restrict__ hkey, const uint32_t* __restrict__ hcnt,
                                 const uint32_t* __restrict__ hmem, MapView map, uint8_t* __restrict__ keep,
                                 uint32_t* __restrict__ surv, unsigned long long* __restrict__ counter) {
  const int64_t h = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (h >= ((int64_t)1 << hb) || counter[2]) return;  // counter[2]: a key out of range
  const uint64_t key = hkey[h];
  if (key == kDsEmpty) return;
  const int64_t m = hcnt[h];
  if (m <= kDsInline) {
    uint32_t mem[kDsInline];
#pragma unroll
    for (int j = 0; j < kDsInline; ++j) mem[j] = j < m ? hmem[h * kDsInline + j] : 0xFFFFFFFFu;
    // insertion sort into list order (m is small)
    for (int j = 1; j < m; ++j) {
      const uint32_t v = mem[j];
      int k = j - 1;
      for (; k >= 0 && mem[k] > v; --k) mem[k + 1] = mem[k];
      mem[k + 1] = v;
    }
    ds_group(in, ds, map, keep, surv, counter, m, [&](int64_t j) { return mem[j]; });
  } else {
    // more members than the slot holds: the list in order, filtered by key
    int64_t next = 0;
    auto member = [&](int64_t j) {
      (void)j;  // called with j = 0, 1, ... in order
      for (;; ++next) {
        const float4 p = in[next];
        const uint64_t k = ds_key((int64_t)floorf(p.x / ds), (int64_t)floorf(p.y / ds), (int64_t)floorf(p.z / ds));
        if (k == key) return (uint32_t)next++;
      }
    };
    ds_group(in, ds, map, keep, surv, counter, m, member);
  }
}

// surviving points -> add4[base + rank] with id next_id + rank
__global__ void k_append(const float4* __restrict__ in, const uint32_t* __restrict__ surv,
                         const uint32_t* __restrict__ rank, int64_t n, float4* __restrict__ add4,
                         uint8_t* __restrict__ akeep, int64_t base, uint32_t next_id) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || (surv && !surv[i])) return;
  const uint32_t r = rank ? rank[i] : (uint32_t)i;
  const float4 p = in[i];
  add4[base + r] = make_float4(p.x, p.y, p.z, __uint_as_float(next_id + r));
  akeep[base + r] = 1;
}

// map_incremental's PointNoNeedDownsample after its PointToAdd survivors,
// both counts on the device: cnt = *cr + *cf points of `in`, placed after
// the *sr + *sf survivors at add4[base ...] with ids continuing next_id
__global__ void k_append_after(const float4* __restrict__ in, int64_t n, const uint32_t* __restrict__ cr,
                               const uint32_t* __restrict__ cf, const uint32_t* __restrict__ sr,
                               const uint32_t* __restrict__ sf, float4* __restrict__ add4,
                               uint8_t* __restrict__ akeep, int64_t base, uint32_t next_id) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || i >= (int64_t)(*cr + *cf)) return;
  const uint32_t r = *sr + *sf + (uint32_t)i;
  const float4 p = in[i];
  add4[base + r] = make_float4(p.x, p.y, p.z, __uint_as_float(next_id + r));
  akeep[base + r] = 1;
}
// the six scan totals (rank + flag of the last entry) map_incremental reads back
__global__ void k_inc_counts(const uint32_t* __restrict__ a0, const uint32_t* __restrict__ a1,
                             const uint32_t* __restrict__ b0, const uint32_t* __restrict__ b1,
                             const uint32_t* __restrict__ c0, const uint32_t* __restrict__ c1,
                             uint32_t* __restrict__ out) {
  if (threadIdx.x == 0) {
    out[0] = *a0 + *a1;
    out[1] = *b0 + *b1;
    out[2] = *c0 + *c1;
  }
}

// pointBodyToWorld (laserMapping.cpp:276-287) with the rotation matrices
// (Sophus SO3::matrix = Eigen toRotationMatrix) and map_incremental's
// classification (laserMapping.cpp:388-423): flag 1 = PointToAdd,
// 2 = PointNoNeedDownsample, 0 = not added.
struct WorldMat {
  double R[9], RL[9], pos[3], tli[3];
};
__global__ void k_map_classify(const float* __restrict__ bx, const float* __restrict__ by,
                               const float* __restrict__ bz, int64_t n, WorldMat W,
                               const uint32_t* __restrict__ nbr_pos, const float4* __restrict__ pts, double fs,
                               int ekf_inited, float4* __restrict__ wpts, uint32_t* __restrict__ f_add,
                               uint32_t* __restrict__ f_no) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double pb[3] = {(double)bx[i], (double)by[i], (double)bz[i]};
  double a[3], w[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) a[r] = ((W.RL[3 * r] * pb[0] + W.RL[3 * r + 1] * pb[1]) + W.RL[3 * r + 2] * pb[2]) + W.tli[r];
#pragma unroll
  for (int r = 0; r < 3; ++r) w[r] = ((W.R[3 * r] * a[0] + W.R[3 * r + 1] * a[1]) + W.R[3 * r + 2] * a[2]) + W.pos[r];
  const float px = (float)w[0], py = (float)w[1], pz = (float)w[2];
  wpts[i] = make_float4(px, py, pz, 0.0f);
  int nn = 0;
  float4 nb[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const uint32_t ps = nbr_pos[i * 5 + j];
    nb[j] = make_float4(0, 0, 0, 0);
    if (ps != 0xFFFFFFFFu && nn == j) {
      nb[j] = pts[ps];
      ++nn;
    }
  }
  uint32_t fa = 0, fn = 0;
  if (nn > 0 && ekf_inited) {
    const float mx = (float)(floor((double)px / fs) * fs + 0.5 * fs);
    const float my = (float)(floor((double)py / fs) * fs + 0.5 * fs);
    const float mz = (float)(floor((double)pz / fs) * fs + 0.5 * fs);
    const float dist = map_dist(px, py, pz, mx, my, mz);
    if ((double)fabsf(nb[0].x - mx) > 0.5 * fs && (double)fabsf(nb[0].y - my) > 0.5 * fs &&
        (double)fabsf(nb[0].z - mz) > 0.5 * fs) {
      fn = 1;
    } else {
      bool need_add = true;
      if (nn >= 5) {
#pragma unroll
        for (int j = 0; j < 5; ++j)
          if (need_add && map_dist(nb[j].x, nb[j].y, nb[j].z, mx, my, mz) < dist) need_add = false;
      }
      fa = need_add ? 1 : 0;
    }
  } else {
    fa = 1;
  }
  f_add[i] = fa;
  f_no[i] = fn;
}

__global__ void k_compact4(const float4* __restrict__ in, const uint32_t* __restrict__ flag,
                           const uint32_t* __restrict__ rank, int64_t n, float4* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && flag[i]) out[rank[i]] = in[i];
}

// ---------------------------------------------------------------- scan VoxelGrid
// downSizeFilterSurf (laserMapping.cpp:683-686, 737-739): pcl::VoxelGrid
// (PCL 1.10 voxel_grid.hpp applyFilter + CentroidPoint) on the device.
__global__ void k_vg_bbox(const float* __restrict__ x, const float* __restrict__ y, const float* __restrict__ z,
                          int64_t n, int32_t* __restrict__ out) {
  int32_t lo[3] = {INT32_MAX, INT32_MAX, INT32_MAX}, hi[3] = {INT32_MIN, INT32_MIN, INT32_MIN};
  int cnt = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float c[3] = {x[i], y[i], z[i]};
    if (!(isfinite(c[0]) && isfinite(c[1]) && isfinite(c[2]))) continue;  // getMinMax3D skips them
    ++cnt;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const int32_t k = fkey(c[a]);
      lo[a] = min(lo[a], k);
      hi[a] = max(hi[a], k);
    }
  }
#pragma unroll
  for (int a = 0; a < 3; ++a)
    for (int d = 32; d > 0; d >>= 1) {
      lo[a] = min(lo[a], __shfl_xor(lo[a], d, 64));
      hi[a] = max(hi[a], __shfl_xor(hi[a], d, 64));
    }
  for (int d = 32; d > 0; d >>= 1) cnt += __shfl_xor(cnt, d, 64);
  // one set of atomics per workgroup on a small grid (as k_bbox4): one per
  // wavefront of a 391-block grid serialised on the 7 counters' cache line,
  // 128 us for a 100k-point scan
  __shared__ int32_t wl[3][4], wh[3][4];
  __shared__ int wc[4];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      wl[a][w] = lo[a];
      wh[a][w] = hi[a];
    }
    wc[w] = cnt;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    const int a = threadIdx.x;
    int32_t l = wl[a][0], h = wh[a][0];
    for (int q = 1; q < (int)(blockDim.x >> 6); ++q) {
      l = min(l, wl[a][q]);
      h = max(h, wh[a][q]);
    }
    atomicMin(out + a, l);
    atomicMax(out + 3 + a, h);
  } else if (threadIdx.x == 3) {
    int c = 0;
    for (int q = 0; q < (int)(blockDim.x >> 6); ++q) c += wc[q];
    atomicAdd(out + 6, c);
  }
}

struct VgGeom {
  float inv[3];
  int minb[3];
  int mul[3];
};

// voxel index idx = ijk0 + ijk1 * div0 + ijk2 * div0 * div1, ijk =
// int(floor(p * inv) - float(min_b)); non-finite points sort last (dropped)
// PCL's geometry (voxel_grid.hpp applyFilter) from the bounding box keys, on
// the device (the same float arithmetic the host did after reading the box
// back): flags[0] = 1 when no point is finite (empty output), flags[1] = 1
// when the leaf is too small for the cloud (PCL passes the input through).
// With either flag set the keys below are meaningless and the caller,
// reading the flags with the voxel count, ignores them.
__global__ void k_vg_geom(const int32_t* __restrict__ bb, float leaf, VgGeom* __restrict__ G,
                          uint32_t* __restrict__ flags) {
  if (threadIdx.x != 0) return;
  VgGeom g;
  float mn[3], mx[3];
  int64_t dd[3];
  for (int a = 0; a < 3; ++a) {
    const int32_t lo = bb[a] >= 0 ? bb[a] : bb[a] ^ 0x7FFFFFFF, hi = bb[3 + a] >= 0 ? bb[3 + a] : bb[3 + a] ^ 0x7FFFFFFF;
    mn[a] = __int_as_float(lo);
    mx[a] = __int_as_float(hi);
    g.inv[a] = 1.0f / leaf;
    const float span = (mx[a] - mn[a]) * g.inv[a];
    dd[a] = isfinite(span) && span < 9.2e18f ? (int64_t)span + 1 : INT64_MAX / 4;
  }
  const bool empty = bb[6] == 0;
  bool pass = dd[0] > INT32_MAX || dd[1] > INT32_MAX || dd[2] > INT32_MAX;
  if (!pass) {
    const int64_t d01 = dd[0] * dd[1];  // (<= 2^62)
    pass = d01 > INT32_MAX || d01 * dd[2] > (int64_t)INT32_MAX;
  }
  pass = pass && !empty;
  int div[3] = {1, 1, 1};
  for (int a = 0; a < 3; ++a) {
    g.minb[a] = 0;
    if (!empty && !pass) {
      g.minb[a] = (int)floorf(mn[a] * g.inv[a]);
      div[a] = (int)floorf(mx[a] * g.inv[a]) - g.minb[a] + 1;
    }
  }
  g.mul[0] = 1;
  g.mul[1] = div[0];
  g.mul[2] = div[0] * div[1];
  *G = g;
  flags[0] = empty ? 1u : 0u;
  flags[1] = pass ? 1u : 0u;
}

__global__ void k_vg_keys(const float* __restrict__ x, const float* __restrict__ y, const float* __restrict__ z,
                          int64_t n, const VgGeom* __restrict__ Gp, uint32_t* __restrict__ keys,
                          uint32_t* __restrict__ vals) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const VgGeom G = *Gp;
  const float c[3] = {x[i], y[i], z[i]};
  uint32_t key = 0xFFFFFFFFu;
  if (isfinite(c[0]) && isfinite(c[1]) && isfinite(c[2])) {
    int ijk[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) ijk[a] = (int)(floorf(c[a] * G.inv[a]) - (float)G.minb[a]);
    key = (uint32_t)(ijk[0] * G.mul[0] + ijk[1] * G.mul[1] + ijk[2] * G.mul[2]);
  }
  keys[i] = key;
  vals[i] = (uint32_t)i;
}

__global__ void k_vg_heads(const uint32_t* __restrict__ keys, int64_t n, uint32_t* __restrict__ head) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  head[i] = keys[i] != 0xFFFFFFFFu && (i == 0 || keys[i] != keys[i - 1]) ? 1u : 0u;
}

// one thread per voxel: the centroid, summed in float in the sorted order
// (ascending point index inside a voxel), divided by the count (CentroidPoint
// AccumulatorXYZ: xyz += p; get: xyz / n)
__global__ void k_vg_centroids(const float* __restrict__ x, const float* __restrict__ y,
                               const float* __restrict__ z, const uint32_t* __restrict__ keys,
                               const uint32_t* __restrict__ order, const uint32_t* __restrict__ head,
                               const uint32_t* __restrict__ rank, int64_t n, float* __restrict__ ox,
                               float* __restrict__ oy, float* __restrict__ oz) {
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i0 >= n || !head[i0]) return;
  float sx = 0.0f, sy = 0.0f, sz = 0.0f;
  int64_t j = i0;
  for (; j < n && keys[j] == keys[i0]; ++j) {
    const uint32_t o = order[j];
    sx = sx + x[o];
    sy = sy + y[o];
    sz = sz + z[o];
  }
  const float cnt = (float)(j - i0);
  const uint32_t r = rank[i0];
  ox[r] = sx / cnt;
  oy[r] = sy / cnt;
  oz[r] = sz / cnt;
}

// exclusive scan of n flags into rank, enqueued on st (no readback)
static int scan_launch(const uint32_t* flag, uint32_t* rank, int64_t n, hipStream_t st) {
  size_t tb = 0;
  // scan temporaries cached per host thread AND device (no hipMalloc /
  // hipFree per call; one thread may drive handles on several GPUs, and a
  // device must never be handed another device's buffer).  Scans reusing
  // the buffer are ordered on one stream, and a buffer is replaced only
  // after the device is idle (hipFree synchronises).
  constexpr int kMaxDev = 64;
  static thread_local void* tmps[kMaxDev] = {};
  static thread_local size_t tcaps[kMaxDev] = {};
  int dev = 0;
  hipError_t e;
  if ((e = hipGetDevice(&dev)) || dev < 0 || dev >= kMaxDev) {
    set_error("slio map: scan: no current device");
    return SLIO_EDEVICE;
  }
  void*& tmp = tmps[dev];
  size_t& tcap = tcaps[dev];
  if ((e = hipcub::DeviceScan::ExclusiveSum(nullptr, tb, flag, rank, (int)n, st))) {
    set_error(std::string("slio map: scan: ") + hipGetErrorString(e));
    return SLIO_EDEVICE;
  }
  if (tb > tcap) {
    (void)hipFree(tmp);
    tmp = nullptr;
    tcap = 0;
    if ((e = hipMalloc(&tmp, tb + tb / 2))) {
      set_error(std::string("slio map: scan: ") + hipGetErrorString(e));
      return SLIO_ENOMEM;
    }
    tcap = tb + tb / 2;
  }
  if ((e = hipcub::DeviceScan::ExclusiveSum(tmp, tb, flag, rank, (int)n, st))) {
    set_error(std::string("slio map: scan: ") + hipGetErrorString(e));
    return SLIO_EDEVICE;
  }
  return SLIO_OK;
}

// exclusive scans of k flag arrays (n each) into ranks; totals read back
// with one synchronisation
static int scan_flags_k(int k, const uint32_t* const* flag, uint32_t* const* rank, int64_t n, hipStream_t st,
                        uint32_t* total) {
  for (int j = 0; j < k; ++j) total[j] = 0;
  if (n == 0) return SLIO_OK;
  uint32_t last[4] = {0, 0, 0, 0};
  Rb rb[4];
  for (int j = 0; j < k; ++j) {
    if (int rc = scan_launch(flag[j], rank[j], n, st)) return rc;
    rb[2 * j] = Rb{&last[2 * j], rank[j] + n - 1, 4};
    rb[2 * j + 1] = Rb{&last[2 * j + 1], flag[j] + n - 1, 4};
  }
  const hipError_t e = readback(st, rb, 2 * k);
  if (e) {
    set_error(std::string("slio map: scan total: ") + hipGetErrorString(e));
    return SLIO_EDEVICE;
  }
  for (int j = 0; j < k; ++j) total[j] = last[2 * j] + last[2 * j + 1];
  return SLIO_OK;
}

// exclusive scan of n flags into rank; returns the total
static int scan_flags(const uint32_t* flag, uint32_t* rank, int64_t n, hipStream_t st, uint32_t* total) {
  return scan_flags_k(1, &flag, &rank, n, st, total);
}

// two exclusive flag scans on one stream, one readback of both totals
static int scan_flags2(const uint32_t* f1, uint32_t* r1, const uint32_t* f2, uint32_t* r2, int64_t n,
                       hipStream_t st, uint32_t* t1, uint32_t* t2) {
  const uint32_t* f[2] = {f1, f2};
  uint32_t* r[2] = {r1, r2};
  uint32_t t[2];
  const int rc = scan_flags_k(2, f, r, n, st, t);
  *t1 = t[0];
  *t2 = t[1];
  return rc;
}

static int add_reserve(MapDev& m, int64_t more, hipStream_t st) {
  if (m.nadd + more <= m.add_cap) return SLIO_OK;
  const int64_t cap = std::max<int64_t>(2 * m.add_cap, m.nadd + more + 4096);
  float4* a = nullptr;
  uint8_t* k = nullptr;
  hipError_t e;
  if ((e = hipMalloc(&a, 16 * cap)) || (e = hipMalloc(&k, cap))) {
    (void)hipFree(a);
    set_error(std::string("slio map: hipMalloc adds: ") + hipGetErrorString(e));
    return SLIO_ENOMEM;
  }
  if (m.nadd > 0 && ((e = hipMemcpyAsync(a, m.add4, 16 * m.nadd, hipMemcpyDeviceToDevice, st)) ||
                     (e = hipMemcpyAsync(k, m.akeep, m.nadd, hipMemcpyDeviceToDevice, st)) ||
                     (e = spin_sync(st)))) {
    (void)hipFree(a);
    (void)hipFree(k);
    set_error(std::string("slio map: grow adds: ") + hipGetErrorString(e));
    return SLIO_EDEVICE;
  }
  (void)hipFree(m.add4);
  (void)hipFree(m.akeep);
  m.add4 = a;
  m.akeep = k;
  m.add_cap = cap;
  return SLIO_OK;
}

static MapView map_view(const MapDev& m) {
  const CoarseView cv{m.cg, m.clo, m.chi};
  return MapView{m.g, m.n, m.pts, m.start, m.blk, m.bstart, m.nblk, m.ncells, cv};
}

// KD_TREE::Add_Points on the device map: n points at `in` (device float4,
// .w ignored); returns the downsample counter (tmp_counter).
// Add_Points(downsample) for exact boxes by hash grouping (k_ds_hash,
// k_ds_groups_hash); *fallback = a voxel key outside ds_key's range was seen
// and nothing was changed (the caller then sorts).
static int map_add_hashed(Ctx& c, const float4* in, int64_t n, float ds, int64_t* counter, bool* fallback) {
  MapDev& m = *c.map;
  hipStream_t st = c.stream;
  *fallback = false;
  int hb = 10;
  while (((int64_t)1 << hb) < 2 * n) ++hb;
  const int64_t H = (int64_t)1 << hb;
  auto& B = m.b_add;
  hipError_t e;
  // B[0]: hash keys, B[1]: member counts, B[2]: members, B[4]: survivor flags,
  // B[5]: their ranks, B[6]: counters (ops, -, out-of-range)
  if ((e = m.take(B[0], 8 * H)) || (e = m.take(B[1], 4 * H)) || (e = m.take(B[2], 4 * kDsInline * H)) ||
      (e = m.take(B[4], 4 * n)) || (e = m.take(B[5], 4 * n)) || (e = m.take(B[6], 64))) {
    set_error(std::string("slio map: hipMalloc: ") + hipGetErrorString(e));
    return SLIO_ENOMEM;
  }
  uint64_t* hkey = (uint64_t*)B[0].p;
  uint32_t* hcnt = (uint32_t*)B[1].p;
  uint32_t* hmem = (uint32_t*)B[2].p;
  uint32_t* surv = (uint32_t*)B[4].p;
  uint32_t* rank = (uint32_t*)B[5].p;
  unsigned long long* dcount = (unsigned long long*)B[6].p;
  // room for every point up front: the survivors are appended (past m.nadd)
  // before the readback that counts them
  if (int rc = add_reserve(m, n, st)) return rc;
  k_ds_init<<<grid_blocks(std::max<int64_t>(H, n)), 256, 0, st>>>(hkey, hcnt, H, surv, n, dcount);
  k_ds_hash<<<grid_blocks(n), 256, 0, st>>>(in, n, ds, hb, hkey, hcnt, hmem, dcount + 2);
  k_ds_groups_hash<<<grid_blocks(H), 256, 0, st>>>(in, n, ds, hb, hkey, hcnt, hmem, map_view(m), m.keep, surv,
                                                   dcount);
  // the survivors' ranks and their append, then their total and the
  // counters in one readback (a key out of range: nothing was appended past
  // m.nadd that counts, and no flag changed)
  if (int rc = scan_launch(surv, rank, n, st)) return rc;
  k_append<<<grid_blocks(n), 256, 0, st>>>(in, surv, rank, n, m.add4, m.akeep, m.nadd, m.next_id);
  uint32_t last[2] = {0, 0};
  unsigned long long ops[3] = {0, 0, 0};
  const Rb rb[3] = {{&last[0], rank + n - 1, 4}, {&last[1], surv + n - 1, 4}, {ops, dcount, 24}};
  if ((e = readback(st, rb, 3))) {
    set_error(std::string("slio map: groups: ") + hipGetErrorString(e));
    return SLIO_EDEVICE;
  }
  const uint32_t total = last[0] + last[1];
  if (ops[2]) {
    *fallback = true;
    return SLIO_OK;
  }
  *counter = (int64_t)ops[0];
  if ((e = hipGetLastError())) {
    set_error(std::string("slio map: append: ") + hipGetErrorString(e));
    return SLIO_EDEVICE;
  }
  m.nadd += total;
  m.next_id += total;
  m.dirty = true;  // deletions (keep flags) and / or additions
  return SLIO_OK;
}

static int map_add(Ctx& c, const float4* in, int64_t n, bool downsample, float ds, int64_t* counter) {
  MapDev& m = *c.map;
  hipStream_t st = c.stream;
  *counter = 0;
  if (n == 0) return SLIO_OK;
  if ((int64_t)m.next_id + n >= (int64_t)0x7FFFFFFF) {
    set_error("slio map: point ids exhausted (2^31)");
    return SLIO_ECAPACITY;
  }
  if (!downsample) {
    if (int rc = add_reserve(m, n, st)) return rc;
    k_append<<<grid_blocks(n), 256, 0, st>>>(in, nullptr, nullptr, n, m.add4, m.akeep, m.nadd, m.next_id);
    SLIO_HIP(hipGetLastError());
    m.nadd += n;
    m.next_id += (uint32_t)n;
    m.dirty = true;
    return SLIO_OK;
  }
  // the box searches need every stored point in the index
  if (int rc = map_refresh_locked(c, true)) return rc;
  {
    // exact boxes (a power-of-two size <= 1, see below): groups by hashing
    // the voxel keys -- no key-range readback, no sort (SLIO_NO_DS_HASH=1:
    // the sorting path)
    int ds_exp0 = 0;
    const char* nh = std::getenv("SLIO_NO_DS_HASH");
    const bool no_hash = nh && nh[0] && nh[0] != '0';
    if (!no_hash && std::frexp(ds, &ds_exp0) == 0.5f && ds <= 1.0f) {
      bool fallback = false;
      if (int rc = map_add_hashed(c, in, n, ds, counter, &fallback)) return rc;
      if (!fallback) return SLIO_OK;
    }
  }
  uint64_t *k0 = nullptr, *k1 = nullptr;
  uint32_t *v0 = nullptr, *v1 = nullptr, *surv = nullptr, *rank = nullptr;
  unsigned long long* dcount = nullptr;
  void* tmp = nullptr;
  int rc = SLIO_OK;
  do {
    // temporaries kept on the map across calls (a live map adds every scan;
    // hipFree would also synchronise the device)
    hipError_t e;
    auto& B = m.b_add;
    if ((e = m.take(B[0], 8 * n)) || (e = m.take(B[1], 8 * n)) || (e = m.take(B[2], 4 * n)) ||
        (e = m.take(B[3], 4 * n)) || (e = m.take(B[4], 4 * n)) || (e = m.take(B[5], 4 * n)) ||
        (e = m.take(B[6], 64))) {
      set_error(std::string("slio map: hipMalloc: ") + hipGetErrorString(e));
      rc = SLIO_ENOMEM;
      break;
    }
    k0 = (uint64_t*)B[0].p;
    k1 = (uint64_t*)B[1].p;
    v0 = (uint32_t*)B[2].p;
    v1 = (uint32_t*)B[3].p;
    surv = (uint32_t*)B[4].p;
    rank = (uint32_t*)B[5].p;
    dcount = (unsigned long long*)B[6].p;
    size_t tb = 0;
    if ((e = hipcub::DeviceRadixSort::SortPairs(nullptr, tb, k0, k1, v0, v1, (int)n, 0, 63, st)) ||
        (e = m.take(B[7], tb))) {
      set_error(std::string("slio map: sort: ") + hipGetErrorString(e));
      rc = SLIO_EDEVICE;
      break;
    }
    tmp = B[7].p;
    tb = B[7].cap;
    const int nb = grid_blocks(n);
    // Boxes interact only through float rounding: for a power-of-two size
    // <= 1 (0.5, the reference default) p / ds, floor * ds and + ds are all
    // exact while |key| + 1 < 2^24 (checked below on the call's key range),
    // every box is exactly [k ds, (k + 1) ds), and no point can lie outside
    // its own box or in two -- nothing to detect
    int ds_exp = 0;
    bool exact_boxes = std::frexp(ds, &ds_exp) == 0.5f && ds <= 1.0f;
    // Then only key equality matters (k_ds_groups; k_ds_conflicts and
    // k_ds_sequential, which look keys up by value, do not run): the keys are
    // packed relative to the call's voxel range, so the radix sort covers a
    // few dozen bits instead of 63 (8 onesweep passes: ~100 us for ~20k keys)
    int sort_bits = 63;
    if (exact_boxes) {
      int32_t* rg = (int32_t*)((char*)B[6].p + 16);  // after dcount (B[6]: 64 bytes)
      const int32_t init[6] = {INT32_MAX, INT32_MAX, INT32_MAX, INT32_MIN, INT32_MIN, INT32_MIN};
      int32_t got[6];
      if ((e = hipMemcpyAsync(rg, init, 24, hipMemcpyHostToDevice, st))) {
        set_error(std::string("slio map: range: ") + hipGetErrorString(e));
        rc = SLIO_EDEVICE;
        break;
      }
      k_ds_range<<<std::min(nb, 256), 256, 0, st>>>(in, n, ds, rg);
      const Rb rb{got, rg, 24};
      if ((e = readback(st, &rb, 1))) {
        set_error(std::string("slio map: range: ") + hipGetErrorString(e));
        rc = SLIO_EDEVICE;
        break;
      }
      for (int a = 0; a < 6; ++a)
        if (std::llabs((long long)got[a]) >= (1ll << 24) - 1) exact_boxes = false;  // (k + 1) ds inexact
      int bits[3];
      for (int a = 0; a < 3; ++a) {
        const int64_t span = (int64_t)got[3 + a] - (int64_t)got[a] + 1;
        bits[a] = 0;
        while (bits[a] < 40 && ((int64_t)1 << bits[a]) < span) ++bits[a];
      }
      if (exact_boxes && bits[0] + bits[1] + bits[2] <= 48) {
        sort_bits = std::max(1, bits[0] + bits[1] + bits[2]);
        const DsPack pk{got[0], got[1], got[2], bits[1] + bits[2], bits[2]};
        k_ds_keys_packed<<<nb, 256, 0, st>>>(in, n, ds, pk, k0, v0);
      }
    }
    if (sort_bits == 63) k_ds_keys<<<nb, 256, 0, st>>>(in, n, ds, k0, v0);
    if ((e = hipcub::DeviceRadixSort::SortPairs(tmp, tb, k0, k1, v0, v1, (int)n, 0, sort_bits, st)) ||
        (e = hipMemsetAsync(surv, 0, 4 * n, st)) || (e = hipMemsetAsync(dcount, 0, 16, st))) {
      set_error(std::string("slio map: sort: ") + hipGetErrorString(e));
      rc = SLIO_EDEVICE;
      break;
    }
    if (!exact_boxes)
      k_ds_conflicts<<<nb, 256, 0, st>>>(in, k1, v1, n, ds, map_view(m), m.keep, dcount + 1);
    k_ds_groups<<<nb, 256, 0, st>>>(in, k1, v1, n, ds, map_view(m), m.keep, surv, dcount);
    uint32_t total = 0;
    if ((rc = scan_flags(surv, rank, n, st, &total))) break;
    unsigned long long ops[2] = {0, 0};
    const Rb rbo{ops, dcount, 16};
    if ((e = readback(st, &rbo, 1))) {
      set_error(std::string("slio map: groups: ") + hipGetErrorString(e));
      rc = SLIO_EDEVICE;
      break;
    }
    if (ops[1]) {
      // interacting groups (k_ds_conflicts): the exact sequential order
      k_ds_sequential<<<1, 1, 0, st>>>(in, k1, v1, n, ds, map_view(m), m.keep, surv, dcount);
      if ((rc = scan_flags(surv, rank, n, st, &total))) break;
      const Rb rbs{ops, dcount, 8};
      if ((e = readback(st, &rbs, 1))) {
        set_error(std::string("slio map: sequential Add_Points: ") + hipGetErrorString(e));
        rc = SLIO_EDEVICE;
        break;
      }
      ++m.sequential_calls;
    }
    *counter = (int64_t)ops[0];
    if ((rc = add_reserve(m, total, st))) break;
    k_append<<<nb, 256, 0, st>>>(in, surv, rank, n, m.add4, m.akeep, m.nadd, m.next_id);
    if ((e = hipGetLastError())) {
      set_error(std::string("slio map: append: ") + hipGetErrorString(e));
      rc = SLIO_EDEVICE;
      break;
    }
    m.nadd += total;
    m.next_id += total;
    m.dirty = true;  // deletions (keep flags) and / or additions
  } while (0);
  return rc;
}

// ---------------------------------------------------------------- merge rebuild
// A rebuild that keeps the grid does not sort the map again: the survivors
// are already in (cell, id) order and every addition has a larger id than
// every stored point, so the new order is, cell by cell, the cell's survivors
// (old order) followed by its additions (id order).  With rank = the
// survivors' exclusive prefix count and lb(c) = the number of (live, sorted)
// additions in cells < c:
//   new_start[c]       = rank(old_start[c]) + lb(c)
//   survivor p, cell c -> new_start[c] + rank[p] - rank(old_start[c])
//   addition j, cell c -> new_start[c + 1] - (lb(c + 1) - j)
// (rank(n0) = the survivor count).  Bit-identical to the sort: same points,
// same order, same cell table.
constexpr int kMergeTile = 4096;
constexpr int64_t kCoarseRetighten = 16;  // cells per workgroup of k_merge_start (256 threads x 16)
__device__ __forceinline__ uint32_t lower_bound_u32(const uint32_t* __restrict__ a, uint32_t lo, uint32_t hi,
                                                    uint32_t v) {
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a[mid] < v)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}
__global__ __launch_bounds__(256) void k_merge_start(const uint32_t* __restrict__ old_start,
                                                     const uint32_t* __restrict__ rank, int64_t n0,
                                                     const uint32_t* __restrict__ n0p_p,
                                                     const uint32_t* __restrict__ sk, const uint32_t* __restrict__ jt,
                                                     int64_t ncells1, uint32_t* __restrict__ new_start) {
  __shared__ uint32_t lk[kMergeTile];
  const int64_t c0 = (int64_t)blockIdx.x * kMergeTile;
  const int64_t c1 = min(c0 + (int64_t)kMergeTile, ncells1);
  const int t = threadIdx.x;
  const uint32_t j0 = jt[blockIdx.x], m = jt[blockIdx.x + 1] - j0;
  const bool inl = m <= (uint32_t)kMergeTile;
  if (inl)
    for (uint32_t k = t; k < m; k += blockDim.x) lk[k] = sk[j0 + k];
  // every load of the thread's 16 cells in flight before any use (one round
  // trip for the cell table, one for the ranks: a load-use chain per cell
  // made this kernel latency-bound)
  constexpr int kPer = kMergeTile / 256;
  uint32_t os[kPer], r[kPer];
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int64_t c = c0 + t + 256 * u;
    os[u] = c < c1 ? old_start[c] : 0u;
  }
  const uint32_t n0p = *n0p_p;
#pragma unroll
  for (int u = 0; u < kPer; ++u) r[u] = (int64_t)os[u] < n0 ? rank[os[u]] : n0p;
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int64_t c = c0 + t + 256 * u;
    if (c >= c1) continue;
    uint32_t lo = 0, hi = m;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if ((inl ? lk[mid] : sk[j0 + mid]) < (uint32_t)c)
        lo = mid + 1;
      else
        hi = mid;
    }
    new_start[c] = r[u] + j0 + lo;
  }
}
__device__ __forceinline__ uint32_t map_cell(const float4& v, const GridGeom& g) {
  const int cx = min(max(cell_coord(v.x, g.ox, g.inv_h), 0), g.dx - 1);
  const int cy = min(max(cell_coord(v.y, g.oy, g.inv_h), 0), g.dy - 1);
  const int cz = min(max(cell_coord(v.z, g.oz, g.inv_h), 0), g.dz - 1);
  return ((uint32_t)cz * (uint32_t)g.dy + (uint32_t)cy) * (uint32_t)g.dx + (uint32_t)cx;
}
// jp[t] = lb(cell of point t * kRankTile), t < ntiles; jp[ntiles] = na.  The
// stored points are in cell order, so a point p of tile t in cell c has
// jp[t] <= lb(c) <= jp[t + 1]
// (and in the same launch jt[t] = lb(t * kMergeTile), t <= ctiles: every
// cell tile's first addition for k_merge_start, one thread per tile -- a
// per-workgroup search at the head of k_merge_start put ~15 dependent loads
// in front of every tile: 294 us for the 10M map's grid)
__global__ void k_merge_ptiles(const float4* __restrict__ pts, int64_t ntiles, GridGeom g,
                               const uint32_t* __restrict__ sk, uint32_t na, uint32_t* __restrict__ jp,
                               int64_t ctiles, int64_t ncells1, uint32_t* __restrict__ jt) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t <= ctiles) {
    jt[t] = lower_bound_u32(sk, 0, na, (uint32_t)min(t * (int64_t)kMergeTile, ncells1));
    return;
  }
  t -= ctiles + 1;
  if (t > ntiles) return;
  jp[t] = t == ntiles ? na : lower_bound_u32(sk, 0, na, map_cell(pts[t * kRankTile], g));
}
// survivor p of cell c goes to new_start[c] + rank[p] - rank(old_start[c])
// = rank[p] + lb(c): one tile of kRankTile points per workgroup, 16 per
// thread with every load in flight before any use, lb(c) from the tile's
// additions in LDS (no per-point cell-table gathers: the dependent
// pts -> old_start -> rank chain made the one-point-per-thread kernel
// latency-bound, ~104 us for the 10M map)
__global__ __launch_bounds__(256) void k_merge_pts(const float4* __restrict__ pts, const uint8_t* __restrict__ keep,
                                                   const uint32_t* __restrict__ rank, const uint32_t* __restrict__ sk,
                                                   const uint32_t* __restrict__ jp, int64_t n0, GridGeom g,
                                                   float4* __restrict__ out, uint8_t* __restrict__ okeep) {
  constexpr int kPer = kRankTile / 256, kLds = 1024;
  __shared__ uint32_t lk[kLds];
  const int64_t p0 = (int64_t)blockIdx.x * kRankTile + threadIdx.x;
  const uint32_t j0 = jp[blockIdx.x], m = jp[blockIdx.x + 1] - j0;
  const bool inl = m <= (uint32_t)kLds;
  if (inl)
    for (uint32_t k = threadIdx.x; k < m; k += 256) lk[k] = sk[j0 + k];
  float4 v[kPer];
  uint32_t r[kPer];
  uint8_t kp[kPer];
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int64_t p = p0 + 256 * u;
    kp[u] = p < n0 ? keep[p] : (uint8_t)0;
    v[u] = p < n0 ? pts[p] : make_float4(0.f, 0.f, 0.f, 0.f);
    r[u] = p < n0 ? rank[p] : 0u;
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    if (!kp[u]) continue;
    const uint32_t c = map_cell(v[u], g);
    uint32_t lo = 0, hi = m;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if ((inl ? lk[mid] : sk[j0 + mid]) < c)
        lo = mid + 1;
      else
        hi = mid;
    }
    out[r[u] + j0 + lo] = v[u];
    okeep[r[u] + j0 + lo] = 1;
  }
}
// the additions' fine cell keys, dead ones keyed kDeadKey (sorted after
// every live one, and above every cell a lower bound asks for); chk[0] += the
// live count, chk[1] = 1 when a live addition is not a cell inside the grid
// (or not finite): the merge is then void and the caller re-grids by sorting
constexpr uint32_t kDeadKey = 0xFFFFFFFFu;
struct MergeBox {
  float lo[3], hi[3];
};
__global__ __launch_bounds__(256) void k_merge_keys(const float4* __restrict__ adds, const uint8_t* __restrict__ akeep,
                                                    int64_t n1, GridGeom g, MergeBox bx, uint32_t* __restrict__ keys,
                                                    uint32_t* __restrict__ vals, uint32_t* __restrict__ chk) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool live = false, fits = true;
  if (i < n1) {
    live = akeep[i] != 0;
    const float4 v = adds[i];
    fits = v.x >= bx.lo[0] && v.x <= bx.hi[0] && v.y >= bx.lo[1] && v.y <= bx.hi[1] && v.z >= bx.lo[2] &&
           v.z <= bx.hi[2];
    keys[i] = live ? map_cell(v, g) : kDeadKey;
    vals[i] = (uint32_t)i;
  }
  const int cnt = __syncthreads_count(live);
  const int bad = __syncthreads_or(live && !fits);
  if (threadIdx.x == 0) {
    if (cnt) atomicAdd(chk, (uint32_t)cnt);
    if (bad) atomicOr(chk + 1, 1u);
  }
}
__global__ void k_merge_adds(const float4* __restrict__ adds, const uint32_t* __restrict__ sk,
                             const uint32_t* __restrict__ sv, uint32_t na, const uint32_t* __restrict__ new_start,
                             float4* __restrict__ out, uint8_t* __restrict__ okeep) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= na) return;
  const uint32_t c = sk[j];
  if (c == kDeadKey) return;
  const uint32_t e = lower_bound_u32(sk, j, na, c + 1);
  out[new_start[c + 1] - (e - j)] = adds[sv[j]];
  okeep[new_start[c + 1] - (e - j)] = 1;
}

// The merge rebuild (see k_merge_start) of m: *handled = false when the
// additions do not all lie at least one cell inside the grid (then the caller
// rebuilds by sorting, with a new grid).  Stream-ordered and speculative: the
// merge runs into temporaries while k_merge_keys checks the additions, and
// ONE readback (survivor count, live additions, the edge flag) decides
// whether the map takes the result (three synchronisations before: the
// counts, the additions' box, the end).
static int merge_rebuild(MapDev& m, hipStream_t st, bool* handled) {
  *handled = false;
  const int64_t n0 = m.n, n1 = m.nadd;
  const GridGeom g = m.g;
  hipError_t e;
  auto fail = [&](const char* what, hipError_t err) {
    set_error(std::string("slio map merge: ") + what + ": " + hipGetErrorString(err));
    return err == hipErrorOutOfMemory ? SLIO_ENOMEM : SLIO_EDEVICE;
  };
  const int64_t na_cap = std::max<int64_t>(n1, 1);
  const int64_t rtiles = (n0 + kRankTile - 1) / kRankTile;
  const int64_t nc1 = m.ncells + 1, ntiles = (nc1 + kMergeTile - 1) / kMergeTile;
  if ((e = m.take(m.b_ref[1], 4 * (rtiles + 3))) || (e = m.take(m.b_ref[2], 4 * n0)) ||
      (e = m.take(m.b_tmp[1], 4 * na_cap)) || (e = m.take(m.b_tmp[2], 4 * na_cap)) ||
      (e = m.take(m.b_tmp[3], 4 * na_cap)) || (e = m.take(m.b_tmp[4], 4 * na_cap)) ||
      (e = m.take(m.b_tmp[5], 4 * (ntiles + 1))) || (e = m.take(m.b_tmp[6], 4 * (rtiles + 1))) ||
      (e = m.take(m.b_ref[0], 16 * (n0 + n1))) || (e = m.take(m.b_start2, sizeof(uint32_t) * nc1)) ||
      (e = m.take(m.b_keep2, n0 + n1)))
    return fail("hipMalloc", e);
  uint32_t* tcnt = (uint32_t*)m.b_ref[1].p;  // [rtiles] tile bases, survivors, live additions, edge flag
  uint32_t* rank = (uint32_t*)m.b_ref[2].p;
  uint32_t* ak = (uint32_t*)m.b_tmp[1].p;
  uint32_t* sk = (uint32_t*)m.b_tmp[2].p;
  uint32_t* av = (uint32_t*)m.b_tmp[3].p;
  uint32_t* sv = (uint32_t*)m.b_tmp[4].p;
  uint32_t* jt = (uint32_t*)m.b_tmp[5].p;
  uint32_t* jp = (uint32_t*)m.b_tmp[6].p;
  float4* out = (float4*)m.b_ref[0].p;
  uint32_t* new_start = (uint32_t*)m.b_start2.p;
  k_keep_tiles<<<(unsigned)rtiles, 256, 0, st>>>(m.keep, n0, rtiles, tcnt);
  k_tile_scan<<<1, 256, 0, st>>>(tcnt, rtiles);
  k_keep_rank<<<(unsigned)rtiles, 256, 0, st>>>(m.keep, n0, tcnt, rank);
  if (n1) {
    // the live additions must lie a cell inside the kept grid
    MergeBox bx;
    const float o[3] = {g.ox, g.oy, g.oz};
    const int d[3] = {g.dx, g.dy, g.dz};
    for (int a = 0; a < 3; ++a) {
      bx.lo[a] = o[a] + g.h;
      bx.hi[a] = o[a] + (float)(d[a] - 1) * g.h;
    }
    k_merge_keys<<<grid_blocks(n1), 256, 0, st>>>(m.add4, m.akeep, n1, g, bx, ak, av, tcnt + rtiles + 1);
    // (stable: a cell's additions stay in id order; the dead ones sort last)
    size_t tb = 0;
    if ((e = hipcub::DeviceRadixSort::SortPairs(nullptr, tb, ak, sk, av, sv, (int)n1, 0, 32, st)) ||
        (e = m.take(m.b_tmp[7], tb)))
      return fail("sort size", e);
    tb = m.b_tmp[7].cap;
    if ((e = hipcub::DeviceRadixSort::SortPairs(m.b_tmp[7].p, tb, ak, sk, av, sv, (int)n1, 0, 32, st)))
      return fail("sort", e);
  }
  uint8_t* okeep = (uint8_t*)m.b_keep2.p;
  k_merge_ptiles<<<grid_blocks(ntiles + rtiles + 2), 256, 0, st>>>(m.pts, rtiles, g, sk, (uint32_t)n1, jp, ntiles,
                                                                    nc1, jt);
  k_merge_start<<<(unsigned)ntiles, 256, 0, st>>>(m.start, rank, n0, tcnt + rtiles, sk, jt, nc1, new_start);
  k_merge_pts<<<(unsigned)rtiles, 256, 0, st>>>(m.pts, m.keep, rank, sk, jp, n0, g, out, okeep);
  if (n1) k_merge_adds<<<grid_blocks(n1), 256, 0, st>>>(m.add4, sk, sv, (uint32_t)n1, new_start, out, okeep);
  // coarse level: the boxes widened by the additions (deleted points leave
  // them conservative); the points themselves are the fine runs.  In place
  // before the readback: a declined merge re-grids by sorting, which builds
  // the coarse level anew
  if (n1) k_coarse_extend<<<grid_blocks(n1), 256, 0, st>>>(m.add4, m.akeep, n1, g, m.clo, m.chi, m.cg);
  if ((e = hipGetLastError())) return fail("merge kernels", e);
  uint32_t cnt[3] = {0, 0, 0};
  {
    const Rb rb{cnt, tcnt + rtiles, 12};
    if ((e = readback(st, &rb, 1))) return fail("counts", e);
  }
  if (cnt[2]) return SLIO_OK;  // an addition near or past the grid's edge (or non-finite): re-grid by sorting
  const uint32_t n0p = cnt[0], na = cnt[1];
  *handled = true;
  const int64_t n = (int64_t)n0p + na;
  // new views: points and cell table swap buffers with their temporaries
  std::swap(m.b_pts, m.b_ref[0]);
  std::swap(m.b_start, m.b_start2);
  m.pts = (float4*)m.b_pts.p;
  m.start = (uint32_t*)m.b_start.p;
  m.n = n;
  std::swap(m.b_keep, m.b_keep2);  // (set by k_merge_pts / k_merge_adds)
  m.keep = (uint8_t*)m.b_keep.p;
  // the boxes only widen through merges: once the deletions since they were
  // tight pass n / kCoarseRetighten, the coarse level is rebuilt from the new
  // cell table -- the boxes a sorting rebuild gives
  m.del_loose += n0 - (int64_t)n0p;
  if (m.del_loose * kCoarseRetighten > n) {
    if ((e = m.take(m.b_tmp[6], 4 * (m.nccells + 1)))) return fail("hipMalloc", e);
    uint32_t* ccnt = (uint32_t*)m.b_tmp[6].p;
    k_coarse_count<<<grid_blocks(m.nccells), 256, 0, st>>>(m.start, g, m.cg, m.nccells, ccnt);
    k_coarse_boxes<<<grid_blocks(m.nccells), 256, 0, st>>>(m.pts, m.start, g, m.cg, ccnt, m.nccells, m.clo, m.chi);
    if ((e = hipGetLastError())) return fail("coarse boxes", e);
    m.del_loose = 0;
  }
  m.blk = nullptr;
  m.bstart = nullptr;
  m.nblk = 0;
  m.blk_deferred = block_rows_wanted(m);
  m.stable_passes = 0;
#ifdef SLIO_BOUNDS_CHECK
  {
    const int64_t nc = m.ncells;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(c_dbg_npts), &n, sizeof(n));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(c_dbg_ncells), &nc, sizeof(nc));
  }
#endif
  if (std::getenv("SLIO_DEBUG_REBUILD"))
    std::fprintf(stderr, "slio rebuild: merge n %lld (survivors %u of %lld, additions %u of %lld)\n", (long long)n,
                 n0p, (long long)n0, na, (long long)n1);
  return SLIO_OK;
}

// Rebuild the index from the surviving points and the pending additions
// (when the map changed since the last build).  adds_only: only when points
// were added (deletions alone are honoured through the keep flags).
static int map_refresh(Ctx& c, bool adds_only) {
  if (!c.map || !c.map->dirty) return SLIO_OK;
  std::unique_lock<std::shared_mutex> lk(c.map->mu);
  if (!c.map->dirty) return SLIO_OK;  // another user rebuilt it meanwhile
  if (int rc = map_read_sync(c)) return rc;
  if (int rc = map_write_begin(c)) return rc;
  const int rc = map_refresh_locked(c, adds_only);
  const int rc2 = map_write_end(c);
  return rc ? rc : rc2;
}

// the rebuild itself: MapDev::mu held exclusively, the stream ordered after
// the other users (map_write_begin)
static int map_refresh_locked(Ctx& c, bool adds_only) {
  if (!c.map || !c.map->dirty) return SLIO_OK;
  MapDev& m = *c.map;
  if (adds_only && m.nadd == 0) return SLIO_OK;
  if (int rc = nbr_settle(c)) return rc;  // the rebuild moves the points
  hipStream_t st = c.stream;
  const int64_t n0 = m.n, n1 = m.nadd, nt = n0 + n1;
  {
    // a grid that still holds every point: merge instead of sorting
    // (SLIO_NO_MERGE=1: always sort)
    const char* nm = std::getenv("SLIO_NO_MERGE");
    if (n0 > 0 && m.start && m.clo && !(nm && nm[0] && nm[0] != '0')) {
      bool handled = false;
      const int rc = merge_rebuild(m, st, &handled);
      if (handled || rc) {
        if (rc) {
          m.broken = true;
          m.free_index();
        }
        m.nadd = 0;
        m.version++;
        m.dirty = false;
        return rc;
      }
    }
  }
  hipError_t e;
  // survivors: stored points (cell order) and additions (id order) compacted
  // into in4; the sort in build_index orders them by (cell, id) anyway
  if ((e = m.take(m.b_ref[0], 16 * nt)) || (e = m.take(m.b_ref[1], 4 * nt)) || (e = m.take(m.b_ref[2], 4 * nt)) ||
      (e = m.take(m.b_ref[3], 32))) {
    set_error(std::string("slio map rebuild: hipMalloc: ") + hipGetErrorString(e));
    return SLIO_ENOMEM;
  }
  float4* in4 = (float4*)m.b_ref[0].p;
  uint32_t* flag = (uint32_t*)m.b_ref[1].p;
  uint32_t* rank = (uint32_t*)m.b_ref[2].p;
  int32_t* bb = (int32_t*)m.b_ref[3].p;
  if (n0) k_widen_flags<<<grid_blocks(n0), 256, 0, st>>>(m.keep, n0, flag);
  if (n1) k_widen_flags<<<grid_blocks(n1), 256, 0, st>>>(m.akeep, n1, flag + n0);
  uint32_t total = 0;
  if (int rc = scan_flags(flag, rank, nt, st, &total)) return rc;
  const int64_t n = total;
  if (n0) k_compact4<<<grid_blocks(n0), 256, 0, st>>>(m.pts, flag, rank, n0, in4);
  // (the ranks of the additions continue the stored points': one scan)
  if (n1) k_compact4<<<grid_blocks(n1), 256, 0, st>>>(m.add4, flag + n0, rank + n0, n1, in4);
  const int32_t init[8] = {INT32_MAX, INT32_MAX, INT32_MAX, INT32_MIN, INT32_MIN, INT32_MIN, 0, 0};
  int32_t got[8];
  if ((e = hipMemcpyAsync(bb, init, 32, hipMemcpyHostToDevice, st))) {
    set_error(std::string("slio map rebuild: ") + hipGetErrorString(e));
    return SLIO_EDEVICE;
  }
  if (n) k_bbox4<<<std::min(grid_blocks(n), 512), 256, 0, st>>>(in4, n, bb);
  const Rb rbb{got, bb, 32};
  if ((e = readback(st, &rbb, 1))) {
    set_error(std::string("slio map rebuild: bbox: ") + hipGetErrorString(e));
    return SLIO_EDEVICE;
  }
  if (got[6]) {
    set_error("slio map rebuild: non-finite map coordinate");
    return SLIO_EINVAL;
  }
  float mn[3] = {0, 0, 0}, mx[3] = {0, 0, 0};
  if (n)
    for (int a = 0; a < 3; ++a) {
      mn[a] = fkey_inv(got[a]);
      mx[a] = fkey_inv(got[3 + a]);
    }
  // in4 is b_ref[0]: build_index reads it while writing the b_* tables
  const bool had_points = n0 > 0;
  m.free_index();
  m.nadd = 0;
  const int rc = build_index(m, in4, n, mn, mx, st, "slio map rebuild", false, true, had_points);
  if (rc) {
    // part-way: the stored points are gone from the views; fail every later
    // use of the map instead of searching a partial index
    m.broken = true;
    m.free_index();
  }
  m.version++;
  m.dirty = false;
  return rc;
}

}  // namespace slio

extern "C" {

int slio_map_upload(slio_handle h, const float* x, const float* y, const float* z, int64_t n) {
  SLIO_CHECK_H(h);
  if (n < 0 || (n > 0 && (!x || !y || !z)) || n >= (int64_t)0xFFFFFFFFll) {
    set_error("slio_map_upload: bad arguments");
    return SLIO_EINVAL;
  }
  auto m = std::make_shared<MapDev>();
  m->device = h->c.prm.device;
  m->cell0 = h->c.prm.grid_cell;
  m->max_cells = h->c.prm.max_grid_cells;
  m->next_id = (uint32_t)n;
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
  float *dx_ = nullptr, *dy_ = nullptr, *dz_ = nullptr;
  float4* in4 = nullptr;
  int rc = SLIO_OK;
  if (n > 0) {
    hipError_t e;
    if ((e = hipMalloc(&dx_, 4 * n)) || (e = hipMalloc(&dy_, 4 * n)) || (e = hipMalloc(&dz_, 4 * n)) ||
        (e = hipMalloc(&in4, 16 * n))) {
      set_error(std::string("slio_map_upload: hipMalloc: ") + hipGetErrorString(e));
      rc = SLIO_ENOMEM;
    } else if ((e = hipMemcpyAsync(dx_, x, 4 * n, hipMemcpyHostToDevice, st)) ||
               (e = hipMemcpyAsync(dy_, y, 4 * n, hipMemcpyHostToDevice, st)) ||
               (e = hipMemcpyAsync(dz_, z, 4 * n, hipMemcpyHostToDevice, st))) {
      set_error(std::string("slio_map_upload: H2D: ") + hipGetErrorString(e));
      rc = SLIO_EDEVICE;
    } else {
      k_pack_ids<<<grid_blocks(n), 256, 0, st>>>(dx_, dy_, dz_, n, 0u, in4);
    }
  }
  if (!rc) rc = build_index(*m, in4, n, mn, mx, st, "slio_map_upload");
  for (void* q : {(void*)dx_, (void*)dy_, (void*)dz_, (void*)in4})
    if (q) (void)hipFree(q);
  if (rc) return rc;
  {
    // sharers of this map order their streams after its build
    SLIO_HIP(hipEventCreateWithFlags(&m->ready, hipEventDisableTiming));
    SLIO_HIP(hipEventRecord(m->ready, st));
    m->epoch = 1;
  }
  if ((rc = nbr_settle_shared(h->c))) return rc;
  map_attach(h->c, m);
  h->c.seen_epoch = 1;
  h->c.searched = false;
  return SLIO_OK;
}

int slio_map_share(slio_handle h, slio_handle src) {
  SLIO_CHECK_H(h);
  if (!src || !src->c.map || src->c.prm.device != h->c.prm.device) {
    set_error("slio_map_share: source has no map on this device");
    return SLIO_EINVAL;
  }
  if (h == src) return SLIO_OK;
  if (int rc = nbr_settle_shared(h->c)) return rc;
  map_attach(h->c, src->c.map);
  h->c.searched = false;
  return SLIO_OK;
}

int slio_map_info(slio_handle h, int32_t dims[3], float* cell, int64_t* n) {
  SLIO_CHECK_H(h);
  if (!h->c.map) {
    set_error("slio_map_info: no map");
    return SLIO_ESTATE;
  }
  if (int rc = map_refresh(h->c)) return rc;
  std::shared_lock<std::shared_mutex> lk(h->c.map->mu);
  if (dims) {
    dims[0] = h->c.map->g.dx;
    dims[1] = h->c.map->g.dy;
    dims[2] = h->c.map->g.dz;
  }
  if (cell) *cell = h->c.map->g.h;
  if (n) *n = h->c.map->n;
  return SLIO_OK;
}

int slio_map_add_points(slio_handle h, const float* x, const float* y, const float* z, int64_t n,
                        int downsample, float downsample_size, int64_t* counter) {
  SLIO_CHECK_H(h);
  Ctx& c = h->c;
  if (!c.map) {
    set_error("slio_map_add_points: no map");
    return SLIO_ESTATE;
  }
  if (n < 0 || (n > 0 && (!x || !y || !z)) || (downsample && !(downsample_size > 0.0f))) {
    set_error("slio_map_add_points: bad arguments");
    return SLIO_EINVAL;
  }
  for (int64_t i = 0; i < n; ++i)
    if (!std::isfinite(x[i]) || !std::isfinite(y[i]) || !std::isfinite(z[i])) {
      set_error("slio_map_add_points: non-finite coordinate");
      return SLIO_EINVAL;
    }
  int64_t cnt = 0;
  if (n > 0) {
    std::unique_lock<std::shared_mutex> lk(c.map->mu);
    if (int rc = map_read_sync(c)) return rc;
    if (int rc = map_write_begin(c)) return rc;
    float *dx_ = nullptr, *dy_ = nullptr, *dz_ = nullptr;
    float4* in4 = nullptr;
    int rc = SLIO_OK;
    hipError_t e;
    if ((e = hipMalloc(&dx_, 4 * n)) || (e = hipMalloc(&dy_, 4 * n)) || (e = hipMalloc(&dz_, 4 * n)) ||
        (e = hipMalloc(&in4, 16 * n))) {
      set_error(std::string("slio_map_add_points: hipMalloc: ") + hipGetErrorString(e));
      rc = SLIO_ENOMEM;
    } else if ((e = hipMemcpyAsync(dx_, x, 4 * n, hipMemcpyHostToDevice, c.stream)) ||
               (e = hipMemcpyAsync(dy_, y, 4 * n, hipMemcpyHostToDevice, c.stream)) ||
               (e = hipMemcpyAsync(dz_, z, 4 * n, hipMemcpyHostToDevice, c.stream))) {
      set_error(std::string("slio_map_add_points: H2D: ") + hipGetErrorString(e));
      rc = SLIO_EDEVICE;
    } else {
      k_pack_ids<<<grid_blocks(n), 256, 0, c.stream>>>(dx_, dy_, dz_, n, 0u, in4);
      rc = map_add(c, in4, n, downsample != 0, downsample_size, &cnt);
      if (!rc) (void)spin_sync(c.stream);
    }
    if (int rc2 = map_write_end(c); rc2 && !rc) rc = rc2;
    for (void* q : {(void*)dx_, (void*)dy_, (void*)dz_, (void*)in4})
      if (q) (void)hipFree(q);
    if (rc) return rc;
  }
  if (counter) *counter = cnt;
  return SLIO_OK;
}

int slio_map_delete_boxes(slio_handle h, const float* boxes, int64_t nboxes, int64_t* deleted) {
  SLIO_CHECK_H(h);
  Ctx& c = h->c;
  if (!c.map) {
    set_error("slio_map_delete_boxes: no map");
    return SLIO_ESTATE;
  }
  if (nboxes < 0 || (nboxes > 0 && !boxes)) {
    set_error("slio_map_delete_boxes: bad arguments");
    return SLIO_EINVAL;
  }
  MapDev& m = *c.map;
  std::unique_lock<std::shared_mutex> lk(m.mu);
  if (int rc = map_read_sync(c)) return rc;
  if (int rc = map_write_begin(c)) return rc;
  unsigned long long* dc = nullptr;
  SLIO_HIP(hipMalloc(&dc, 8));
  SLIO_HIP(hipMemsetAsync(dc, 0, 8, c.stream));
  for (int64_t b0 = 0; b0 < nboxes; b0 += 8) {
    Boxes8 bx{};
    bx.n = (int)std::min<int64_t>(8, nboxes - b0);
    for (int k = 0; k < bx.n; ++k)
      for (int j = 0; j < 6; ++j) bx.b[k][j] = boxes[6 * (b0 + k) + j];
    if (m.n) k_map_delete<<<grid_blocks(m.n), 256, 0, c.stream>>>(m.pts, m.keep, m.n, bx, dc);
    if (m.nadd) k_map_delete<<<grid_blocks(m.nadd), 256, 0, c.stream>>>(m.add4, m.akeep, m.nadd, bx, dc);
  }
  unsigned long long k = 0;
  hipError_t e = hipMemcpyAsync(&k, dc, 8, hipMemcpyDeviceToHost, c.stream);
  if (!e) e = hipStreamSynchronize(c.stream);
  (void)hipFree(dc);
  if (e) {
    set_error(std::string("slio_map_delete_boxes: ") + hipGetErrorString(e));
    return SLIO_EDEVICE;
  }
  if (k) m.dirty = true;
  if (deleted) *deleted = (int64_t)k;
  return map_write_end(c);
}

// map_incremental's two Add_Points in one stream of launches with ONE
// readback (exact hash boxes, nothing pending in the index): the lists'
// counts, the survivors and the counters stay on the device until the end,
// where the classify counts used to be read back first and the appends
// launched after.  *fallback: a voxel key outside ds_key's range (nothing
// added, no flag changed): the caller takes the per-call path.
static int map_incremental_hashed(Ctx& c, const float4* w4, uint32_t* fa, uint32_t* fn, uint32_t* ra,
                                  uint32_t* rn, float4* l1, float4* l2, int64_t n, float ds, int64_t out[3],
                                  bool* fallback) {
  MapDev& m = *c.map;
  hipStream_t st = c.stream;
  *fallback = false;
  const int nb = grid_blocks(n);
  if (int rc = scan_launch(fa, ra, n, st)) return rc;
  if (int rc = scan_launch(fn, rn, n, st)) return rc;
  k_compact4<<<nb, 256, 0, st>>>(w4, fa, ra, n, l1);
  k_compact4<<<nb, 256, 0, st>>>(w4, fn, rn, n, l2);
  int hb = 10;
  while (((int64_t)1 << hb) < 2 * n) ++hb;
  const int64_t H = (int64_t)1 << hb;
  auto& B = m.b_add;
  hipError_t e;
  if ((e = m.take(B[0], 8 * H)) || (e = m.take(B[1], 4 * H)) || (e = m.take(B[2], 4 * kDsInline * H)) ||
      (e = m.take(B[4], 4 * n)) || (e = m.take(B[5], 4 * n)) || (e = m.take(B[6], 64))) {
    set_error(std::string("slio map: hipMalloc: ") + hipGetErrorString(e));
    return SLIO_ENOMEM;
  }
  uint64_t* hkey = (uint64_t*)B[0].p;
  uint32_t* hcnt = (uint32_t*)B[1].p;
  uint32_t* hmem = (uint32_t*)B[2].p;
  uint32_t* surv = (uint32_t*)B[4].p;
  uint32_t* rank = (uint32_t*)B[5].p;
  unsigned long long* dcount = (unsigned long long*)B[6].p;  // [0, 24): ops, -, out of range; [24, 36): counts
  uint32_t* cnt = (uint32_t*)((char*)B[6].p + 24);
  if (int rc = add_reserve(m, 2 * n, st)) return rc;
  k_ds_init<<<grid_blocks(std::max<int64_t>(H, n)), 256, 0, st>>>(hkey, hcnt, H, surv, n, dcount);
  k_ds_hash<<<nb, 256, 0, st>>>(l1, n, ds, hb, hkey, hcnt, hmem, dcount + 2, ra + n - 1, fa + n - 1);
  k_ds_groups_hash<<<grid_blocks(H), 256, 0, st>>>(l1, n, ds, hb, hkey, hcnt, hmem, map_view(m), m.keep, surv,
                                                   dcount);
  if (int rc = scan_launch(surv, rank, n, st)) return rc;
  k_append<<<nb, 256, 0, st>>>(l1, surv, rank, n, m.add4, m.akeep, m.nadd, m.next_id);
  k_append_after<<<nb, 256, 0, st>>>(l2, n, rn + n - 1, fn + n - 1, rank + n - 1, surv + n - 1, m.add4, m.akeep,
                                     m.nadd, m.next_id);
  k_inc_counts<<<1, 64, 0, st>>>(ra + n - 1, fa + n - 1, rn + n - 1, fn + n - 1, rank + n - 1, surv + n - 1, cnt);
  unsigned long long got[5];  // ops, -, out of range, then the three counts as 32-bit words
  {
    const Rb rb{got, dcount, 36};
    if ((e = hipGetLastError()) || (e = readback(st, &rb, 1))) {
      set_error(std::string("slio_map_incremental: ") + hipGetErrorString(e));
      return SLIO_EDEVICE;
    }
  }
  if (got[2]) {
    *fallback = true;
    return SLIO_OK;
  }
  uint32_t k3[3];
  std::memcpy(k3, &got[3], 12);
  const uint32_t na = k3[0], nn = k3[1], total = k3[2];
  out[0] = na;
  out[1] = nn;
  out[2] = (int64_t)got[0];
  m.nadd += (int64_t)total + nn;
  m.next_id += total + nn;
  if (na || nn) m.dirty = true;  // deletions (keep flags) and / or additions (as the per-call path)
  return SLIO_OK;
}

int slio_map_incremental(slio_handle h, const slio_state* x, double filter_size_map_min, int ekf_inited,
                         int64_t counts[3]) {
  SLIO_CHECK_H(h);
  Ctx& c = h->c;
  if (!x || !(filter_size_map_min > 0.0)) {
    set_error("slio_map_incremental: bad arguments");
    return SLIO_EINVAL;
  }
  if (!c.map) {
    set_error("slio_map_incremental: no map");
    return SLIO_ESTATE;
  }
  std::unique_lock<std::shared_mutex> map_lock(c.map->mu);
  if (!c.searched || c.search_version != c.map->version) {
    set_error("slio_map_incremental: no search pass on the current map (Nearest_Points)");
    return SLIO_ESTATE;
  }
  if (int rc = map_read_sync(c)) return rc;
  if (int rc = map_write_begin(c)) return rc;
  if (c.prm.nranks != 1) {
    set_error("slio_map_incremental: needs the whole scan (nranks == 1)");
    return SLIO_EINVAL;
  }
  const int64_t n = c.n;
  WorldMat W;
  {
    // Eigen Quaternion::toRotationMatrix (Sophus SO3::matrix)
    auto mat = [](const double* q, double* R) {
      const double w = q[0], qx = q[1], qy = q[2], qz = q[3];
      const double tx = 2.0 * qx, ty = 2.0 * qy, tz = 2.0 * qz;
      const double twx = tx * w, twy = ty * w, twz = tz * w;
      const double txx = tx * qx, txy = ty * qx, txz = tz * qx;
      const double tyy = ty * qy, tyz = tz * qy, tzz = tz * qz;
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
    mat(x->rot, W.R);
    mat(x->rli, W.RL);
    for (int k = 0; k < 3; ++k) {
      W.pos[k] = x->pos[k];
      W.tli[k] = x->tli[k];
    }
  }
  int64_t out[3] = {0, 0, 0};
  if (n > 0) {
    float4 *w4 = nullptr, *l1 = nullptr, *l2 = nullptr;
    uint32_t *fa = nullptr, *fn = nullptr, *ra = nullptr, *rn = nullptr;
    int rc = SLIO_OK;
    do {
      hipError_t e;
      auto& B = c.inc;  // kept across scans (hipFree would synchronise the device)
      if ((e = MapDev::take(B[0], 16 * n)) || (e = MapDev::take(B[1], 16 * n)) ||
          (e = MapDev::take(B[2], 16 * n)) || (e = MapDev::take(B[3], 4 * n)) ||
          (e = MapDev::take(B[4], 4 * n)) || (e = MapDev::take(B[5], 4 * n)) || (e = MapDev::take(B[6], 4 * n))) {
        set_error(std::string("slio_map_incremental: hipMalloc: ") + hipGetErrorString(e));
        rc = SLIO_ENOMEM;
        break;
      }
      w4 = (float4*)B[0].p;
      l1 = (float4*)B[1].p;
      l2 = (float4*)B[2].p;
      fa = (uint32_t*)B[3].p;
      fn = (uint32_t*)B[4].p;
      ra = (uint32_t*)B[5].p;
      rn = (uint32_t*)B[6].p;
      const int nb = grid_blocks(n);
      k_map_classify<<<nb, 256, 0, c.stream>>>(c.bx, c.by, c.bz, n, W, c.nbr_pos, c.map->pts,
                                               filter_size_map_min, ekf_inited, w4, fa, fn);
      {
        MapDev& m = *c.map;
        const float ds = (float)filter_size_map_min;
        int ds_exp = 0;
        const char* nh = std::getenv("SLIO_NO_DS_HASH");
        if (!(nh && nh[0] && nh[0] != '0') && std::frexp(ds, &ds_exp) == 0.5f && ds <= 1.0f &&
            !(m.dirty && m.nadd > 0) && (int64_t)m.next_id + 2 * n < (int64_t)0x7FFFFFFF) {
          bool fallback = false;
          if ((rc = map_incremental_hashed(c, w4, fa, fn, ra, rn, l1, l2, n, ds, out, &fallback))) break;
          if (!fallback) break;
        }
      }
      uint32_t na = 0, nn = 0;
      if ((rc = scan_flags2(fa, ra, fn, rn, n, c.stream, &na, &nn))) break;
      k_compact4<<<nb, 256, 0, c.stream>>>(w4, fa, ra, n, l1);
      k_compact4<<<nb, 256, 0, c.stream>>>(w4, fn, rn, n, l2);
      out[0] = na;
      out[1] = nn;
      int64_t cnt = 0, cnt2 = 0;
      if ((rc = map_add(c, l1, na, true, (float)filter_size_map_min, &cnt))) break;
      if ((rc = map_add(c, l2, nn, false, (float)filter_size_map_min, &cnt2))) break;
      out[2] = cnt;
      SLIO_HIP(spin_sync(c.stream));
    } while (0);
    if (int rc2 = map_write_end(c); rc2 && !rc) rc = rc2;
    if (rc) return rc;
  }
  if (counts)
    for (int k = 0; k < 3; ++k) counts[k] = out[k];
  return SLIO_OK;
}

int slio_map_download(slio_handle h, float* x, float* y, float* z, uint32_t* ids, int64_t cap, int64_t* n) {
  SLIO_CHECK_H(h);
  Ctx& c = h->c;
  if (!c.map) {
    set_error("slio_map_download: no map");
    return SLIO_ESTATE;
  }
  if (int rc = map_refresh(c)) return rc;
  std::shared_lock<std::shared_mutex> lk(c.map->mu);
  if (int rc = map_read_sync(c)) return rc;
  const MapDev& m = *c.map;
  if (n) *n = m.n;
  if (cap < m.n || (m.n > 0 && (!x || !y || !z || !ids))) {
    set_error("slio_map_download: buffer too small");
    return SLIO_ECAPACITY;
  }
  std::vector<float4> buf((size_t)m.n);
  if (m.n) {
    SLIO_HIP(hipMemcpyAsync(buf.data(), m.pts, 16 * m.n, hipMemcpyDeviceToHost, c.stream));
    SLIO_HIP(hipStreamSynchronize(c.stream));
  }
  std::vector<std::pair<uint32_t, uint32_t>> order((size_t)m.n);
  for (int64_t i = 0; i < m.n; ++i) {
    uint32_t id;
    std::memcpy(&id, &buf[i].w, 4);
    order[i] = {id, (uint32_t)i};
  }
  std::sort(order.begin(), order.end());
  for (int64_t k = 0; k < m.n; ++k) {
    const float4& p = buf[order[k].second];
    x[k] = p.x;
    y[k] = p.y;
    z[k] = p.z;
    ids[k] = order[k].first;
  }
  return SLIO_OK;
}

// Test hook (not in the header): the last pass's per-chunk partials,
// num_chunks(n) x 91 doubles (global chunk index; other ranks' chunks are
// stale), so tests can rebuild the segment / super tree from them.
int slio_dbg_chunk_partials(slio_handle h, double* out, int64_t cap, int64_t* nchunks) {
  SLIO_CHECK_H(h);
  Ctx& c = h->c;
  if (!nchunks) return SLIO_EINVAL;
  const int64_t C = num_chunks(c.n);
  *nchunks = C;
  if (!c.chunk_part || C == 0) return SLIO_ESTATE;
  if (cap < C * SLIO_NPROD || !out) return SLIO_ECAPACITY;
  SLIO_HIP(hipMemcpyAsync(out, c.chunk_part, sizeof(double) * SLIO_NPROD * C, hipMemcpyDeviceToHost, c.stream));
  SLIO_HIP(hipStreamSynchronize(c.stream));
  return SLIO_OK;
}

// test support (not in include/slio.h): the index's points in their stored
// (cell, id) order, x, y, z, bits(id) per point, after the pending rebuild
int slio_dbg_map_raw(slio_handle h, float* xyzw, int64_t cap, int64_t* n) {
  SLIO_CHECK_H(h);
  Ctx& c = h->c;
  if (!c.map || !n) return SLIO_ESTATE;
  if (int rc = map_refresh(c)) return rc;
  std::shared_lock<std::shared_mutex> lk(c.map->mu);
  if (int rc = map_read_sync(c)) return rc;
  *n = c.map->n;
  if (cap < c.map->n || (c.map->n > 0 && !xyzw)) return SLIO_ECAPACITY;
  if (c.map->n) {
    SLIO_HIP(hipMemcpyAsync(xyzw, c.map->pts, 16 * c.map->n, hipMemcpyDeviceToHost, c.stream));
    SLIO_HIP(hipStreamSynchronize(c.stream));
  }
  return SLIO_OK;
}

// test support (not in include/slio.h): the coarse level's boxes, lo then hi
// (nccells float4 each: x, y, z and the count word), after the pending rebuild
int slio_dbg_map_coarse(slio_handle h, float* lohi, int64_t cap, int64_t* nccells) {
  SLIO_CHECK_H(h);
  Ctx& c = h->c;
  if (!c.map || !nccells) return SLIO_ESTATE;
  if (int rc = map_refresh(c)) return rc;
  std::shared_lock<std::shared_mutex> lk(c.map->mu);
  if (int rc = map_read_sync(c)) return rc;
  const int64_t nc = c.map->nccells;
  *nccells = nc;
  if (cap < 2 * nc || (nc > 0 && !lohi)) return SLIO_ECAPACITY;
  if (nc) {
    SLIO_HIP(hipMemcpyAsync(lohi, c.map->clo, 16 * nc, hipMemcpyDeviceToHost, c.stream));
    SLIO_HIP(hipMemcpyAsync(lohi + 4 * nc, c.map->chi, 16 * nc, hipMemcpyDeviceToHost, c.stream));
    SLIO_HIP(hipStreamSynchronize(c.stream));
  }
  return SLIO_OK;
}

int slio_fov_segment(const double pos_lid[3], float box_min[3], float box_max[3], int* initialized,
                     double cube_len, float det_range, float boxes_out[18], int* nboxes) {
  if (!pos_lid || !box_min || !box_max || !initialized || !boxes_out || !nboxes) {
    set_error("slio_fov_segment: bad arguments");
    return SLIO_EINVAL;
  }
  // lasermap_fov_segment (laserMapping.cpp:309-365), MOV_THRESHOLD 1.5 (:40)
  const float kMov = 1.5f;
  *nboxes = 0;
  if (!*initialized) {
    for (int i = 0; i < 3; ++i) {
      box_min[i] = (float)(pos_lid[i] - cube_len / 2.0);
      box_max[i] = (float)(pos_lid[i] + cube_len / 2.0);
    }
    *initialized = 1;
    return SLIO_OK;
  }
  float dist[3][2];
  bool need_move = false;
  for (int i = 0; i < 3; ++i) {
    dist[i][0] = (float)std::fabs(pos_lid[i] - box_min[i]);
    dist[i][1] = (float)std::fabs(pos_lid[i] - box_max[i]);
    if (dist[i][0] <= kMov * det_range || dist[i][1] <= kMov * det_range) need_move = true;
  }
  if (!need_move) return SLIO_OK;
  float nmin[3], nmax[3];
  for (int i = 0; i < 3; ++i) {
    nmin[i] = box_min[i];
    nmax[i] = box_max[i];
  }
  const float mov = (float)std::max((cube_len - 2.0 * kMov * det_range) * 0.5 * 0.9,
                                    double(det_range * (kMov - 1)));
  int k = 0;
  for (int i = 0; i < 3; ++i) {
    float tmin[3] = {box_min[0], box_min[1], box_min[2]}, tmax[3] = {box_max[0], box_max[1], box_max[2]};
    if (dist[i][0] <= kMov * det_range) {
      nmax[i] -= mov;
      nmin[i] -= mov;
      tmin[i] = box_max[i] - mov;
    } else if (dist[i][1] <= kMov * det_range) {
      nmax[i] += mov;
      nmin[i] += mov;
      tmax[i] = box_min[i] + mov;
    } else {
      continue;
    }
    for (int j = 0; j < 3; ++j) {
      boxes_out[6 * k + j] = tmin[j];
      boxes_out[6 * k + 3 + j] = tmax[j];
    }
    ++k;
  }
  for (int i = 0; i < 3; ++i) {
    box_min[i] = nmin[i];
    box_max[i] = nmax[i];
  }
  *nboxes = k;
  return SLIO_OK;
}

}  // extern "C"

// downSizeFilterSurf of n device points (dx_, dy_, dz_) into the handle's scan
static int voxel_device(Ctx& c, const float* dx_, const float* dy_, const float* dz_, int64_t n, float leaf,
                        int64_t* n_down) {
  hipStream_t st = c.stream;
  uint32_t *k0 = nullptr, *k1 = nullptr, *v0 = nullptr, *v1 = nullptr, *hd = nullptr, *rk = nullptr;
  int32_t* bb = nullptr;
  int rc = nbr_settle_shared(c);  // the scan it was searched with is replaced
  if (rc) return rc;
  int64_t m = 0;
  bool passthrough = false;
  do {
    if (n == 0) break;
    hipError_t e;
    // (pre[0..3] may hold the undistorted input: slio_scan_upload_undistort_voxel)
    MapDev::Buf* B = c.pre + 8;
    if ((e = MapDev::take(B[0], 4 * n)) || (e = MapDev::take(B[1], 4 * n)) || (e = MapDev::take(B[2], 4 * n)) ||
        (e = MapDev::take(B[3], 4 * n)) || (e = MapDev::take(B[4], 4 * n)) || (e = MapDev::take(B[5], 4 * n)) ||
        (e = MapDev::take(B[6], 32 + sizeof(VgGeom) + 8))) {
      set_error(std::string("slio_scan_upload_voxel: hipMalloc: ") + hipGetErrorString(e));
      rc = SLIO_ENOMEM;
      break;
    }
    k0 = (uint32_t*)B[0].p;
    k1 = (uint32_t*)B[1].p;
    v0 = (uint32_t*)B[2].p;
    v1 = (uint32_t*)B[3].p;
    hd = (uint32_t*)B[4].p;
    rk = (uint32_t*)B[5].p;
    bb = (int32_t*)B[6].p;
    const int32_t init[8] = {INT32_MAX, INT32_MAX, INT32_MAX, INT32_MIN, INT32_MIN, INT32_MIN, 0, 0};
    if ((e = hipMemcpyAsync(bb, init, 32, hipMemcpyHostToDevice, st))) {
      set_error(std::string("slio_scan_upload_voxel: H2D: ") + hipGetErrorString(e));
      rc = SLIO_EDEVICE;
      break;
    }
    // the box, the geometry and the voxel keys stay on the device: ONE
    // readback below (voxel count and the geometry's flags) where the box used
    // to come back first
    VgGeom* gdev = reinterpret_cast<VgGeom*>((char*)B[6].p + 32);
    uint32_t* vflags = reinterpret_cast<uint32_t*>((char*)B[6].p + 32 + sizeof(VgGeom));
    k_vg_bbox<<<std::min(grid_blocks(n), 64), 256, 0, st>>>(dx_, dy_, dz_, n, bb);
    k_vg_geom<<<1, 64, 0, st>>>(bb, leaf, gdev, vflags);
    const int nb = grid_blocks(n);
    k_vg_keys<<<nb, 256, 0, st>>>(dx_, dy_, dz_, n, gdev, k0, v0);
    size_t tb = 0;
    if ((e = hipcub::DeviceRadixSort::SortPairs(nullptr, tb, k0, k1, v0, v1, (int)n, 0, 32, st)) ||
        (e = MapDev::take(B[7], tb)) ||
        (e = hipcub::DeviceRadixSort::SortPairs(B[7].p, tb, k0, k1, v0, v1, (int)n, 0, 32, st))) {
      set_error(std::string("slio_scan_upload_voxel: sort: ") + hipGetErrorString(e));
      rc = SLIO_EDEVICE;
      break;
    }
    k_vg_heads<<<nb, 256, 0, st>>>(k1, n, hd);
    if ((rc = scan_launch(hd, rk, n, st))) break;
    uint32_t got[4] = {0, 0, 0, 0};
    {
      const Rb rb[3] = {{&got[0], rk + n - 1, 4}, {&got[1], hd + n - 1, 4}, {&got[2], vflags, 8}};
      if ((e = readback(st, rb, 3))) {
        set_error(std::string("slio_scan_upload_voxel: counts: ") + hipGetErrorString(e));
        rc = SLIO_EDEVICE;
        break;
      }
    }
    if (got[2]) break;  // no finite point: empty scan
    if (got[3]) {
      passthrough = true;  // PCL: leaf too small for the cloud, output = input
      break;
    }
    m = (int64_t)got[0] + got[1];
    if (m > c.prm.max_points) {
      set_error("slio_scan_upload_voxel: downsampled scan exceeds max_points");
      rc = SLIO_ECAPACITY;
      break;
    }
    if ((rc = ensure_scan_buffers(c))) break;
    k_vg_centroids<<<nb, 256, 0, st>>>(dx_, dy_, dz_, k1, v1, hd, rk, n, c.bx, c.by, c.bz);
    if ((e = hipGetLastError())) {
      set_error(std::string("slio_scan_upload_voxel: ") + hipGetErrorString(e));
      rc = SLIO_EDEVICE;
      break;
    }
  } while (0);
  if (!rc && passthrough) {
    if (n > c.prm.max_points) {
      set_error("slio_scan_upload_voxel: scan exceeds max_points");
      rc = SLIO_ECAPACITY;
    } else if (!(rc = ensure_scan_buffers(c))) {
      // non-finite points stay (PCL copies the input as is)
      (void)hipMemcpyAsync(c.bx, dx_, 4 * n, hipMemcpyDeviceToDevice, st);
      (void)hipMemcpyAsync(c.by, dy_, 4 * n, hipMemcpyDeviceToDevice, st);
      (void)hipMemcpyAsync(c.bz, dz_, 4 * n, hipMemcpyDeviceToDevice, st);
      m = n;
    }
  }
  if (!rc) {
    // (no synchronisation: every user of the scan buffers runs on this
    // stream, after the centroids)
    if (m > 0 && c.bx) (void)hipMemsetAsync(c.sel, 0, m, st);
    if (const hipError_t e = hipGetLastError()) {
      set_error(std::string("slio_scan_upload_voxel: ") + hipGetErrorString(e));
      return SLIO_EDEVICE;
    }
    c.n = m;
    c.searched = false;
    if (n_down) *n_down = m;
  }
  return rc;
}

// ---------------------------------------------------------------- LIO-SAM scan-to-map
// mapOptmization.cpp cornerOptimization (:1303-1432), surfOptimization
// (:1438-1515) and the rows / normal equations of LMOptimization
// (:1552-1626) on the device; the 6x6 solve stays on the host
// (slio_s2m_lm_step).  One handle per feature class: its map is
// laserCloud{Corner,Surf}FromMapDS, its scan laserCloud{Corner,Surf}LastDS.

// pointAssociateToMap (:359-373) with the float affine of
// pcl::getTransformation(transformTobeMapped)
struct Aff12 {
  float m[12];
};
__global__ void k_s2m_transform(const float* __restrict__ bx, const float* __restrict__ by,
                                const float* __restrict__ bz, int64_t n, Aff12 T, float* __restrict__ wx,
                                float* __restrict__ wy, float* __restrict__ wz) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float x = bx[i], y = by[i], z = bz[i];
  wx[i] = ((T.m[0] * x + T.m[1] * y) + T.m[2] * z) + T.m[3];
  wy[i] = ((T.m[4] * x + T.m[5] * y) + T.m[6] * z) + T.m[7];
  wz[i] = ((T.m[8] * x + T.m[9] * y) + T.m[10] * z) + T.m[11];
}

// OpenCV's hypot (lapack.cpp): scaled, in the element type
__device__ __forceinline__ float cv_hypot(float a, float b) {
  a = fabsf(a);
  b = fabsf(b);
  if (a > b) {
    b /= a;
    return a * sqrtf(1 + b * b);
  }
  if (b > 0) {
    a /= b;
    return b * sqrtf(1 + a * a);
  }
  return 0;
}

// cv::eigen of a symmetric 3x3 float matrix: OpenCV hal::Jacobi
// (JacobiImpl_, lapack.cpp) -- eigenvalues W descending, eigenvectors the
// rows of V.  Fully unrolled over compile-time indices (n = 3).
__device__ __forceinline__ void cv_jacobi3(float A[9], float W[3], float V[9]) {
  const float eps = 1.1920928955078125e-07f;
#pragma unroll
  for (int k = 0; k < 9; ++k) V[k] = (k % 4 == 0) ? 1.0f : 0.0f;
  int indR[3], indC[3];
  W[0] = A[0];
  W[1] = A[4];
  W[2] = A[8];
  // k = 0: row max over cols 1..2; k = 1: col 2 and column max over rows 0
  indR[0] = (fabsf(A[1]) < fabsf(A[2])) ? 2 : 1;
  indR[1] = 2;
  indC[1] = 0;
  indC[2] = (fabsf(A[2]) < fabsf(A[5])) ? 1 : 0;
  for (int iters = 0; iters < 3 * 3 * 30; ++iters) {
    int k = 0;
    float mv = fabsf(A[indR[0]]);
    {
      const float val = fabsf(A[3 + indR[1]]);
      if (mv < val) mv = val, k = 1;
    }
    int l = indR[k];
    for (int i = 1; i < 3; ++i) {
      const float val = fabsf(A[3 * indC[i] + i]);
      if (mv < val) mv = val, k = indC[i], l = i;
    }
    const float p = A[3 * k + l];
    if (fabsf(p) <= eps) break;
    float y = (float)((W[l] - W[k]) * 0.5);
    float t = fabsf(y) + cv_hypot(p, y);
    float sn = cv_hypot(p, t);
    const float c = t / sn;
    sn = p / sn;
    t = (p / t) * p;
    if (y < 0) sn = -sn, t = -t;
    A[3 * k + l] = 0;
    W[k] -= t;
    W[l] += t;
    float a0, b0;
#define SLIO_ROT(v0, v1) a0 = v0, b0 = v1, v0 = a0 * c - b0 * sn, v1 = a0 * sn + b0 * c
    for (int i = 0; i < k; ++i) SLIO_ROT(A[3 * i + k], A[3 * i + l]);
    for (int i = k + 1; i < l; ++i) SLIO_ROT(A[3 * k + i], A[3 * i + l]);
    for (int i = l + 1; i < 3; ++i) SLIO_ROT(A[3 * k + i], A[3 * l + i]);
    for (int i = 0; i < 3; ++i) SLIO_ROT(V[3 * k + i], V[3 * l + i]);
#undef SLIO_ROT
    for (int j = 0; j < 2; ++j) {
      const int idx = j == 0 ? k : l;
      if (idx < 2) {
        int m = idx + 1;
        float mvv = fabsf(A[3 * idx + m]);
        for (int i = idx + 2; i < 3; ++i) {
          const float val = fabsf(A[3 * idx + i]);
          if (mvv < val) mvv = val, m = i;
        }
        indR[idx] = m;
      }
      if (idx > 0) {
        int m = 0;
        float mvv = fabsf(A[idx]);
        for (int i = 1; i < idx; ++i) {
          const float val = fabsf(A[3 * i + idx]);
          if (mvv < val) mvv = val, m = i;
        }
        indC[idx] = m;
      }
    }
  }
  for (int k = 0; k < 2; ++k) {
    int m = k;
    for (int i = k + 1; i < 3; ++i)
      if (W[m] < W[i]) m = i;
    if (k != m) {
      const float tw = W[m];
      W[m] = W[k];
      W[k] = tw;
      for (int i = 0; i < 3; ++i) {
        const float tv = V[3 * m + i];
        V[3 * m + i] = V[3 * k + i];
        V[3 * k + i] = tv;
      }
    }
  }
}

// coefficients (coeff.x, y, z, intensity) and selection of every scan point
template <int KIND>  // 0: corner (point-to-line), 1: surf (point-to-plane)
__global__ void k_s2m_coeff(const float* __restrict__ wx, const float* __restrict__ wy,
                            const float* __restrict__ wz, int64_t n, const uint32_t* __restrict__ nbr_pos,
                            const float* __restrict__ nbr_sqd, const float4* __restrict__ pts,
                            float4* __restrict__ coeff, uint8_t* __restrict__ sel) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t ok = 0;
  float4 cf = make_float4(0, 0, 0, 0);
  const float x0 = wx[i], y0 = wy[i], z0 = wz[i];
  if (nbr_sqd[i * 5 + 4] < 1.0f) {  // (< 1.0 is false for +inf: fewer than 5 map points)
    float nb[5][3];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const float4 p = pts[nbr_pos[i * 5 + j]];
      nb[j][0] = p.x;
      nb[j][1] = p.y;
      nb[j][2] = p.z;
    }
    if (KIND == 0) {
      float cx = 0, cy = 0, cz = 0;
#pragma unroll
      for (int j = 0; j < 5; ++j) {
        cx += nb[j][0];
        cy += nb[j][1];
        cz += nb[j][2];
      }
      cx /= 5;
      cy /= 5;
      cz /= 5;
      float a11 = 0, a12 = 0, a13 = 0, a22 = 0, a23 = 0, a33 = 0;
#pragma unroll
      for (int j = 0; j < 5; ++j) {
        const float ax = nb[j][0] - cx, ay = nb[j][1] - cy, az = nb[j][2] - cz;
        a11 += ax * ax;
        a12 += ax * ay;
        a13 += ax * az;
        a22 += ay * ay;
        a23 += ay * az;
        a33 += az * az;
      }
      a11 /= 5;
      a12 /= 5;
      a13 /= 5;
      a22 /= 5;
      a23 /= 5;
      a33 /= 5;
      float A[9] = {a11, a12, a13, a12, a22, a23, a13, a23, a33}, W[3], V[9];
      cv_jacobi3(A, W, V);
      if (W[0] > 3 * W[1]) {
        const float x1 = cx + 0.1 * V[0], y1 = cy + 0.1 * V[1], z1 = cz + 0.1 * V[2];
        const float x2 = cx - 0.1 * V[0], y2 = cy - 0.1 * V[1], z2 = cz - 0.1 * V[2];
        const float u = (x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1);
        const float v = (x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1);
        const float w = (y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1);
        const float a012 = sqrtf(u * u + v * v + w * w);
        const float l12 = sqrtf((x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2) + (z1 - z2) * (z1 - z2));
        const float la = ((y1 - y2) * u + (z1 - z2) * v) / a012 / l12;
        const float lb = -((x1 - x2) * u - (z1 - z2) * w) / a012 / l12;
        const float lc = -((x1 - x2) * v + (y1 - y2) * w) / a012 / l12;
        const float ld2 = a012 / l12;
        const float s = 1 - 0.9 * fabsf(ld2);
        cf = make_float4(s * la, s * lb, s * lc, s * ld2);
        ok = s > 0.1;
      }
    } else {
      float sol[3];
      qr_solve_m1_dev(nb, sol);
      float pa = sol[0], pb = sol[1], pc = sol[2], pd = 1;
      const float ps = sqrtf(pa * pa + pb * pb + pc * pc);
      pa /= ps;
      pb /= ps;
      pc /= ps;
      pd /= ps;
      bool valid = true;
#pragma unroll
      for (int j = 0; j < 5; ++j)
        if (fabsf(pa * nb[j][0] + pb * nb[j][1] + pc * nb[j][2] + pd) > 0.2) valid = false;
      if (valid) {
        const float pd2 = pa * x0 + pb * y0 + pc * z0 + pd;
        const float s = 1 - 0.9 * fabsf(pd2) / sqrtf(sqrtf(x0 * x0 + y0 * y0 + z0 * z0));
        cf = make_float4(s * pa, s * pb, s * pc, s * pd2);
        ok = s > 0.1;
      }
    }
  }
  coeff[i] = cf;
  sel[i] = ok;
}

// LMOptimization rows (:1583-1626, lidar <-> camera axis swap included) of the
// selected points and their A^T A (21) / A^T B (6) / count, summed in double:
// each workgroup its 256 points in a fixed tree (a butterfly over each
// wavefront's lanes, then the four wavefronts in order), one partial per
// workgroup.  (The 28 sequential block-wide LDS trees this replaces -- 252
// barriers -- took 27.8 us per launch for 20k points,
// profiles/r05_final_s2m_kernel_stats.csv.)
struct S2mTrig {
  float srx, crx, sry, cry, srz, crz;
};
constexpr int kS2mSums = 28;
__global__ __launch_bounds__(256) void k_s2m_rows(const float* __restrict__ bx, const float* __restrict__ by,
                                                  const float* __restrict__ bz, const float4* __restrict__ coeff,
                                                  const uint8_t* __restrict__ sel, int64_t n, S2mTrig T,
                                                  double* __restrict__ partial) {
  __shared__ double red[4 * kS2mSums];
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  double v[kS2mSums];
#pragma unroll
  for (int k = 0; k < kS2mSums; ++k) v[k] = 0.0;
  if (i < n && sel[i]) {
    const float4 cs = coeff[i];
    const float px = by[i], py = bz[i], pz = bx[i];   // lidar -> camera
    const float cx = cs.y, cy = cs.z, cz = cs.x, ci = cs.w;
    const float srx = T.srx, crx = T.crx, sry = T.sry, cry = T.cry, srz = T.srz, crz = T.crz;
    const float arx = (crx * sry * srz * px + crx * crz * sry * py - srx * sry * pz) * cx +
                      (-srx * srz * px - crz * srx * py - crx * pz) * cy +
                      (crx * cry * srz * px + crx * cry * crz * py - cry * srx * pz) * cz;
    const float ary = ((cry * srx * srz - crz * sry) * px + (sry * srz + cry * crz * srx) * py + crx * cry * pz) * cx +
                      ((-cry * crz - srx * sry * srz) * px + (cry * srz - crz * srx * sry) * py - crx * sry * pz) * cz;
    const float arz = ((crz * srx * sry - cry * srz) * px + (-cry * crz - srx * sry * srz) * py) * cx +
                      (crx * crz * px - crx * srz * py) * cy +
                      ((sry * srz + cry * crz * srx) * px + (crz * sry - cry * srx * srz) * py) * cz;
    const float a[6] = {arz, arx, ary, cz, cx, cy};
    const float b = -ci;
    int q = 0;
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
      for (int c = r; c < 6; ++c) v[q++] = (double)a[r] * (double)a[c];
#pragma unroll
    for (int r = 0; r < 6; ++r) v[21 + r] = (double)a[r] * (double)b;
    v[27] = 1.0;
  }
  // (a + b == b + a: both lanes of a butterfly pair hold the same sum)
#pragma unroll
  for (int off = 32; off > 0; off >>= 1)
#pragma unroll
    for (int k = 0; k < kS2mSums; ++k) v[k] = v[k] + __shfl_xor(v[k], off);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int k = 0; k < kS2mSums; ++k) red[w * kS2mSums + k] = v[k];
  __syncthreads();
  if (threadIdx.x < kS2mSums) {
    const int k = threadIdx.x;
    partial[(int64_t)blockIdx.x * kS2mSums + k] =
        ((red[k] + red[kS2mSums + k]) + red[2 * kS2mSums + k]) + red[3 * kS2mSums + k];
  }
}

// pcl::getTransformation (pcl/common/impl/eigen.hpp) in float, the trig
// correctly rounded (evaluated in double)
static Aff12 s2m_affine(const float tf[6]) {
  const float x = tf[3], y = tf[4], z = tf[5], roll = tf[0], pitch = tf[1], yaw = tf[2];
  auto fc = [](float a) { return (float)std::cos((double)a); };
  auto fs = [](float a) { return (float)std::sin((double)a); };
  const float A = fc(yaw), B = fs(yaw), C = fc(pitch), D = fs(pitch), E = fc(roll), F = fs(roll), DE = D * E,
              DF = D * F;
  Aff12 t;
  t.m[0] = A * C, t.m[1] = A * DF - B * E, t.m[2] = B * F + A * DE, t.m[3] = x;
  t.m[4] = B * C, t.m[5] = A * E + B * DF, t.m[6] = B * DE - A * F, t.m[7] = y;
  t.m[8] = -D, t.m[9] = C * F, t.m[10] = C * E, t.m[11] = z;
  return t;
}

extern "C" {

int slio_s2m_coeffs(slio_handle h, int kind, const float transform[6], int64_t* nsel) {
  SLIO_CHECK_H(h);
  Ctx& c = h->c;
  if ((kind != 0 && kind != 1) || !transform) {
    set_error("slio_s2m_coeffs: bad arguments");
    return SLIO_EINVAL;
  }
  if (!c.map || !c.bx) {
    set_error("slio_s2m_coeffs: map and scan needed");
    return SLIO_ESTATE;
  }
  if (c.prm.nranks != 1) {
    set_error("slio_s2m_coeffs: single-rank handles only");
    return SLIO_EINVAL;
  }
  const int64_t n = c.n;
  if (!c.wbx) {
    const int64_t cap = c.prm.max_points;
    hipError_t e;
    if ((e = hipMalloc(&c.wbx, 4 * cap)) || (e = hipMalloc(&c.wby, 4 * cap)) || (e = hipMalloc(&c.wbz, 4 * cap))) {
      set_error(std::string("slio_s2m_coeffs: hipMalloc: ") + hipGetErrorString(e));
      return SLIO_ENOMEM;
    }
  }
  if (n > 0) {
    k_s2m_transform<<<grid_blocks(n), 256, 0, c.stream>>>(c.bx, c.by, c.bz, n, s2m_affine(transform), c.wbx,
                                                           c.wby, c.wbz);
    // the 5-NN of the world points: the search pass in kNN-only mode with the
    // identity pose (body -> world of an identity pose is exact in float)
    slio_pose idp{};
    idp.rot[0] = 1.0;
    idp.rli[0] = 1.0;
    const PoseDev P = make_pose(&idp);
    const ScanDev sd{c.wbx, c.wby, c.wbz, n};
    if (int rc = enqueue_pass(c, &P, nullptr, 1, 0, nullptr, false, true, &sd)) return rc;
    std::shared_lock<std::shared_mutex> lk(c.map->mu);
    if (int rc = map_read_sync(c)) return rc;
    if (kind == 0)
      k_s2m_coeff<0><<<grid_blocks(n), 256, 0, c.stream>>>(c.wbx, c.wby, c.wbz, n, c.nbr_pos, c.nbr_sqd,
                                                            c.map->pts, c.plane, c.sel);
    else
      k_s2m_coeff<1><<<grid_blocks(n), 256, 0, c.stream>>>(c.wbx, c.wby, c.wbz, n, c.nbr_pos, c.nbr_sqd,
                                                            c.map->pts, c.plane, c.sel);
    SLIO_HIP(hipGetLastError());
  }
  c.s2m_kind = kind;
  if (nsel) {
    std::vector<uint8_t> sl((size_t)n);
    if (n) {
      SLIO_HIP(hipStreamSynchronize(c.stream));
      SLIO_HIP(hipMemcpy(sl.data(), c.sel, n, hipMemcpyDeviceToHost));
    }
    int64_t k = 0;
    for (uint8_t v : sl) k += v;
    *nsel = k;
  }
  return SLIO_OK;
}

int slio_s2m_get_coeffs(slio_handle h, float* coeff, uint8_t* sel) {
  SLIO_CHECK_H(h);
  Ctx& c = h->c;
  if (c.n > 0) {
    SLIO_HIP(hipStreamSynchronize(c.stream));
    if (coeff) SLIO_HIP(hipMemcpy(coeff, c.plane, 16 * c.n, hipMemcpyDeviceToHost));
    if (sel) SLIO_HIP(hipMemcpy(sel, c.sel, c.n, hipMemcpyDeviceToHost));
  }
  return SLIO_OK;
}

int slio_s2m_normal_equations(slio_handle h_corner, slio_handle h_surf, const float transform[6], float AtA[36],
                              float AtB[6], int64_t* nsel) {
  if (!transform || !AtA || !AtB) {
    set_error("slio_s2m_normal_equations: bad arguments");
    return SLIO_EINVAL;
  }
  // the camera-frame trig of LMOptimization (:1564-1569), float sin / cos
  S2mTrig T;
  auto fc = [](float a) { return (float)std::cos((double)a); };
  auto fs = [](float a) { return (float)std::sin((double)a); };
  T.srx = fs(transform[1]), T.crx = fc(transform[1]);
  T.sry = fs(transform[2]), T.cry = fc(transform[2]);
  T.srz = fs(transform[0]), T.crz = fc(transform[0]);
  double acc[kS2mSums] = {0};
  // corners first, then surfs (combineOptimizationCoeffs :1517-1543); both
  // clouds' rows launched before either is read back (their own streams)
  slio_handle hs2[2] = {h_corner, h_surf};
  for (slio_handle h : hs2) {
    if (!h || h->c.n == 0) continue;
    Ctx& c = h->c;
    const int nb = (int)((c.n + 255) / 256);
    k_s2m_rows<<<nb, 256, 0, c.stream>>>(c.bx, c.by, c.bz, c.plane, c.sel, c.n, T, c.chunk_part);
    SLIO_HIP(hipGetLastError());
  }
  for (slio_handle h : hs2) {
    if (!h || h->c.n == 0) continue;
    Ctx& c = h->c;
    const int nb = (int)((c.n + 255) / 256);
    std::vector<double> part((size_t)nb * kS2mSums);
    const Rb rb{part.data(), c.chunk_part, 8 * part.size()};
    SLIO_HIP(readback(c.stream, &rb, 1));
    for (int b = 0; b < nb; ++b)
      for (int k = 0; k < kS2mSums; ++k) acc[k] = acc[k] + part[(size_t)b * kS2mSums + k];
  }
  int q = 0;
  for (int r = 0; r < 6; ++r)
    for (int cc = r; cc < 6; ++cc, ++q) AtA[6 * r + cc] = AtA[6 * cc + r] = (float)acc[q];
  for (int r = 0; r < 6; ++r) AtB[r] = (float)acc[21 + r];
  if (nsel) *nsel = (int64_t)llround(acc[27]);
  return SLIO_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- scan undistortion
struct UndistEnd {
  double R[9], RL[9], TL[3], pos[3];
};

__global__ void k_time_keys(const float* __restrict__ t, int64_t n, uint32_t* __restrict__ keys,
                            uint32_t* __restrict__ vals) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  keys[i] = (uint32_t)fkey(t[i]) ^ 0x80000000u;  // float order as unsigned
  vals[i] = (uint32_t)i;
}

// UndistortPcl step 5 (IMU_Processing.hpp:351-401): point i of the time
// order takes the IMU segment (head k, tail k + 1) with the largest k <=
// npose - 2 whose offset is below its time -- the segment the reference's
// backward double loop assigns it -- and is moved to the scan end:
//   R_i = R_head Exp(gyr_tail dt),  T_ei = pos + vel dt + 0.5 acc dt dt - pos_end,
//   P' = R_LI^T (R_end^T (R_i (R_LI P + T_LI) + T_ei) - T_LI)
__global__ void k_undistort(const float* __restrict__ x, const float* __restrict__ y, const float* __restrict__ z,
                            const float* __restrict__ t, const uint32_t* __restrict__ order, int64_t n,
                            const slio_imu_pose* __restrict__ poses, int np, UndistEnd E, float* __restrict__ ox,
                            float* __restrict__ oy, float* __restrict__ oz, float* __restrict__ ot) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t o = order[i];
  const float px = x[o], py = y[o], pz = z[o], pt = t[o];
  ot[i] = pt;
  const double tt = (double)pt / double(1000);
  int lo = -1;
  if (np >= 2) {
    int a = 0, b = np - 2;  // largest k in [0, np-2] with offset[k] < tt
    while (a <= b) {
      const int m = (a + b) >> 1;
      if (poses[m].offset_time < tt) {
        lo = m;
        a = m + 1;
      } else {
        b = m - 1;
      }
    }
  }
  if (lo < 0) {
    ox[i] = px;
    oy[i] = py;
    oz[i] = pz;
    return;
  }
  // The reference's backward loop leaves its point iterator on the first
  // point once that point is done ("if (it_pcl == begin) break"), so every
  // earlier segment whose offset is below that point's time compensates it
  // again (IMU_Processing.hpp:365-399): mirrored for i == 0.
  float cx = px, cy = py, cz = pz;
  const int k_end = (i == 0) ? 0 : lo;
  for (int k = lo; k >= k_end; --k) {
    const slio_imu_pose& hd = poses[k];
    const slio_imu_pose& tl = poses[k + 1];
    if (!(tt > hd.offset_time)) break;
    const double dt = tt - hd.offset_time;
    const double w[3] = {tl.gyr[0] * dt, tl.gyr[1] * dt, tl.gyr[2] * dt};
    double Ex[9];
    qmatrix(so3_exp(w), Ex);
    double Ri[9];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int cc = 0; cc < 3; ++cc)
        Ri[3 * r + cc] = (hd.rot[3 * r] * Ex[cc] + hd.rot[3 * r + 1] * Ex[3 + cc]) + hd.rot[3 * r + 2] * Ex[6 + cc];
    const double P[3] = {(double)cx, (double)cy, (double)cz};
    double Tei[3], a[3], b[3], cv[3], d[3];
#pragma unroll
    for (int q = 0; q < 3; ++q)
      Tei[q] = ((hd.pos[q] + hd.vel[q] * dt) + ((0.5 * tl.acc[q]) * dt) * dt) - E.pos[q];
#pragma unroll
    for (int r = 0; r < 3; ++r)
      a[r] = ((E.RL[3 * r] * P[0] + E.RL[3 * r + 1] * P[1]) + E.RL[3 * r + 2] * P[2]) + E.TL[r];
#pragma unroll
    for (int r = 0; r < 3; ++r) b[r] = ((Ri[3 * r] * a[0] + Ri[3 * r + 1] * a[1]) + Ri[3 * r + 2] * a[2]) + Tei[r];
#pragma unroll
    for (int r = 0; r < 3; ++r) cv[r] = ((E.R[r] * b[0] + E.R[3 + r] * b[1]) + E.R[6 + r] * b[2]) - E.TL[r];
#pragma unroll
    for (int r = 0; r < 3; ++r) d[r] = (E.RL[r] * cv[0] + E.RL[3 + r] * cv[1]) + E.RL[6 + r] * cv[2];
    cx = (float)d[0];
    cy = (float)d[1];
    cz = (float)d[2];
  }
  ox[i] = cx;
  oy[i] = cy;
  oz[i] = cz;
}

// whether the host's point times are already in k_time_keys' order (the
// same unsigned keys, non-decreasing): then the stable sort is the identity
// and is skipped (a driver's scan usually arrives in firing order)
static bool time_keys_sorted(const float* t, int64_t n) {
  uint32_t prev = 0, bad = 0;
  for (int64_t i = 0; i < n; ++i) {
    int32_t b;
    std::memcpy(&b, t + i, 4);
    const uint32_t k = (uint32_t)(b >= 0 ? b : b ^ 0x7FFFFFFF) ^ 0x80000000u;
    bad |= (uint32_t)(k < prev);
    prev = k;
  }
  return bad == 0;
}

// undistorted scan in time order into device arrays ux, uy, uz, ut (n each)
static int undistort_device(Ctx& c, const float* x, const float* y, const float* z, const float* t, int64_t n,
                            const slio_imu_pose* poses, int np, const slio_state* xe, float* ux, float* uy, float* uz,
                            float* ut, bool sync_end = true) {
  hipStream_t st = c.stream;
  UndistEnd E;
  qmatrix(Quat{xe->rot[0], xe->rot[1], xe->rot[2], xe->rot[3]}, E.R);
  qmatrix(Quat{xe->rli[0], xe->rli[1], xe->rli[2], xe->rli[3]}, E.RL);
  for (int k = 0; k < 3; ++k) {
    E.TL[k] = xe->tli[k];
    E.pos[k] = xe->pos[k];
  }
  float *dx_ = nullptr, *dy_ = nullptr, *dz_ = nullptr, *dt_ = nullptr;
  uint32_t *k0 = nullptr, *k1 = nullptr, *v0 = nullptr, *v1 = nullptr;
  slio_imu_pose* dp = nullptr;
  int rc = SLIO_OK;
  do {
    hipError_t e;
    MapDev::Buf* B = c.pre + 4;  // pre[0..3]: the caller's output; pre[8..15]: voxel_device
    if ((e = MapDev::take(B[0], 16 * n)) || (e = MapDev::take(B[1], 16 * n)) ||
        (e = MapDev::take(B[2], sizeof(slio_imu_pose) * std::max(np, 1)))) {
      set_error(std::string("slio undistort: hipMalloc: ") + hipGetErrorString(e));
      rc = SLIO_ENOMEM;
      break;
    }
    dx_ = (float*)B[0].p;
    dy_ = dx_ + n;
    dz_ = dx_ + 2 * n;
    dt_ = dx_ + 3 * n;
    k0 = (uint32_t*)B[1].p;
    k1 = k0 + n;
    v0 = k0 + 2 * n;
    v1 = k0 + 3 * n;
    dp = (slio_imu_pose*)B[2].p;
    if ((e = hipMemcpyAsync(dx_, x, 4 * n, hipMemcpyHostToDevice, st)) ||
        (e = hipMemcpyAsync(dy_, y, 4 * n, hipMemcpyHostToDevice, st)) ||
        (e = hipMemcpyAsync(dz_, z, 4 * n, hipMemcpyHostToDevice, st)) ||
        (e = hipMemcpyAsync(dt_, t, 4 * n, hipMemcpyHostToDevice, st)) ||
        (np > 0 && (e = hipMemcpyAsync(dp, poses, sizeof(slio_imu_pose) * np, hipMemcpyHostToDevice, st)))) {
      set_error(std::string("slio undistort: H2D: ") + hipGetErrorString(e));
      rc = SLIO_EDEVICE;
      break;
    }
    const int nb = grid_blocks(n);
    k_time_keys<<<nb, 256, 0, st>>>(dt_, n, k0, v0);
    const bool in_order = time_keys_sorted(t, n);  // (while the copies and keys run)
    size_t tb = 0;
    if (!in_order &&
        ((e = hipcub::DeviceRadixSort::SortPairs(nullptr, tb, k0, k1, v0, v1, (int)n, 0, 32, st)) ||
         (e = MapDev::take(B[3], tb)) ||
         (e = hipcub::DeviceRadixSort::SortPairs(B[3].p, tb, k0, k1, v0, v1, (int)n, 0, 32, st)))) {
      set_error(std::string("slio undistort: sort: ") + hipGetErrorString(e));
      rc = SLIO_EDEVICE;
      break;
    }
    k_undistort<<<nb, 256, 0, st>>>(dx_, dy_, dz_, dt_, in_order ? v0 : v1, n, dp, np, E, ux, uy, uz, ut);
    // (the combined entry's VoxelGrid step follows on the stream and reads back
    // itself: no synchronisation here)
    if ((e = hipGetLastError()) || (sync_end && (e = spin_sync(st)))) {
      set_error(std::string("slio undistort: ") + hipGetErrorString(e));
      rc = SLIO_EDEVICE;
      break;
    }
  } while (0);
  return rc;
}

extern "C" {

int slio_undistort(slio_handle h, const float* x, const float* y, const float* z, const float* t_ms, int64_t n,
                   const slio_imu_pose* poses, int npose, const slio_state* x_end, float* ox, float* oy, float* oz,
                   float* ot_ms) {
  SLIO_CHECK_H(h);
  if (n < 0 || (n > 0 && (!x || !y || !z || !t_ms || !ox || !oy || !oz || !ot_ms)) || npose < 0 ||
      (npose > 0 && !poses) || !x_end || n >= (int64_t)0xFFFFFFFFll) {
    set_error("slio_undistort: bad arguments");
    return SLIO_EINVAL;
  }
  if (n == 0) return SLIO_OK;
  Ctx& c = h->c;
  SLIO_HIP(MapDev::take(c.pre[0], 16 * n));
  float* u = (float*)c.pre[0].p;
  int rc = undistort_device(c, x, y, z, t_ms, n, poses, npose, x_end, u, u + n, u + 2 * n, u + 3 * n);
  if (!rc) {
    hipError_t e;
    if ((e = hipMemcpy(ox, u, 4 * n, hipMemcpyDeviceToHost)) || (e = hipMemcpy(oy, u + n, 4 * n, hipMemcpyDeviceToHost)) ||
        (e = hipMemcpy(oz, u + 2 * n, 4 * n, hipMemcpyDeviceToHost)) ||
        (e = hipMemcpy(ot_ms, u + 3 * n, 4 * n, hipMemcpyDeviceToHost))) {
      set_error(std::string("slio_undistort: D2H: ") + hipGetErrorString(e));
      rc = SLIO_EDEVICE;
    }
  }
  return rc;
}

int slio_scan_upload_undistort_voxel(slio_handle h, const float* x, const float* y, const float* z,
                                     const float* t_ms, int64_t n, const slio_imu_pose* poses, int npose,
                                     const slio_state* x_end, float leaf, int64_t* n_down) {
  SLIO_CHECK_H(h);
  if (n < 0 || (n > 0 && (!x || !y || !z || !t_ms)) || npose < 0 || (npose > 0 && !poses) || !x_end ||
      !(leaf > 0.0f) || n >= (int64_t)0xFFFFFFFFll) {
    set_error("slio_scan_upload_undistort_voxel: bad arguments");
    return SLIO_EINVAL;
  }
  Ctx& c = h->c;
  float* u = nullptr;
  if (n > 0) {
    SLIO_HIP(MapDev::take(c.pre[0], 16 * n));
    u = (float*)c.pre[0].p;
  }
  int rc = n > 0 ? undistort_device(c, x, y, z, t_ms, n, poses, npose, x_end, u, u + n, u + 2 * n, u + 3 * n,
                                    false)
                 : SLIO_OK;
  if (!rc) rc = voxel_device(c, u, u ? u + n : nullptr, u ? u + 2 * n : nullptr, n, leaf, n_down);
  return rc;
}

int slio_scan_upload_voxel(slio_handle h, const float* x, const float* y, const float* z, int64_t n,
                           float leaf, int64_t* n_down) {
  SLIO_CHECK_H(h);
  Ctx& c = h->c;
  if (n < 0 || (n > 0 && (!x || !y || !z)) || !(leaf > 0.0f) || n >= (int64_t)0xFFFFFFFFll) {
    set_error("slio_scan_upload_voxel: bad arguments");
    return SLIO_EINVAL;
  }
  float *dx_ = nullptr, *dy_ = nullptr, *dz_ = nullptr;
  int rc = SLIO_OK;
  if (n > 0) {
    hipError_t e;
    if ((e = MapDev::take(c.pre[0], 12 * n))) {
      set_error(std::string("slio_scan_upload_voxel: hipMalloc: ") + hipGetErrorString(e));
      return SLIO_ENOMEM;
    }
    dx_ = (float*)c.pre[0].p;
    dy_ = dx_ + n;
    dz_ = dx_ + 2 * n;
    if ((e = hipMemcpyAsync(dx_, x, 4 * n, hipMemcpyHostToDevice, c.stream)) ||
        (e = hipMemcpyAsync(dy_, y, 4 * n, hipMemcpyHostToDevice, c.stream)) ||
        (e = hipMemcpyAsync(dz_, z, 4 * n, hipMemcpyHostToDevice, c.stream))) {
      set_error(std::string("slio_scan_upload_voxel: H2D: ") + hipGetErrorString(e));
      rc = SLIO_EDEVICE;
    }
  }
  if (!rc) rc = voxel_device(c, dx_, dy_, dz_, n, leaf, n_down);
  return rc;
}

int slio_scan_download(slio_handle h, float* x, float* y, float* z) {
  SLIO_CHECK_H(h);
  Ctx& c = h->c;
  if (c.n > 0 && (!x || !y || !z)) {
    set_error("slio_scan_download: bad arguments");
    return SLIO_EINVAL;
  }
  if (c.n > 0) {
    SLIO_HIP(hipStreamSynchronize(c.stream));
    SLIO_HIP(hipMemcpy(x, c.bx, 4 * c.n, hipMemcpyDeviceToHost));
    SLIO_HIP(hipMemcpy(y, c.by, 4 * c.n, hipMemcpyDeviceToHost));
    SLIO_HIP(hipMemcpy(z, c.bz, 4 * c.n, hipMemcpyDeviceToHost));
  }
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
  if (int rc = nbr_settle_shared(c)) return rc;  // the scan it was searched with is replaced
  if (int rc = ensure_scan_buffers(c)) return rc;
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
  const PoseDev P = make_pose(x);
  const int rc = enqueue_pass(c, &P, nullptr, do_search ? 1 : 0, extrinsic_est);
  if (rc) return rc;
  if (d_super) *d_super = c.d_super;
  return SLIO_OK;
}

}  // extern "C"

namespace slio {

// One device-resident update on one handle (slio_ikf_update_device), in
// steps, so that the rank handles of a group can interleave their passes
// with one collective per pass (slio_group_ikf_update).
struct UpdateRun {
  Ctx& c;
  slio_state* x;
  double* P;
  double R;
  int maxit, ext, mode;
  bool multi;   // the super rows are all-reduced between a pass and its filter step
  int first = 0, dim = 6;
  PoseDev pose0{};

  UpdateRun(Ctx& c_, slio_state* x_, double* P_, double R_, int maxit_, int ext_, int mode_, bool multi_)
      : c(c_), x(x_), P(P_), R(R_), maxit(maxit_), ext(ext_), mode(mode_), multi(multi_) {}

  int begin() {
    if (!c.ctl) {
      SLIO_HIP(hipMalloc(&c.ctl, sizeof(IkfCtl)));
      SLIO_HIP(hipHostMalloc(&c.h_ctl, sizeof(IkfCtl), hipHostMallocMapped | hipHostMallocCoherent));
      SLIO_HIP(hipHostGetDevicePointer((void**)&c.d_hctl, c.h_ctl, 0));
    }
    first = (mode == SLIO_MODE_REFERENCE) ? -1 : 0;
    // a fresh epoch: no certificate of an earlier update is ever used
    if (++c.kc_next == 0) {
      if (c.kepoch) SLIO_HIP(hipMemsetAsync(c.kepoch, 0, 4 * (num_chunks(c.prm.max_points) + 1), c.stream));
      c.kc_next = 1;
    }
    c.kc_epoch = c.sw.no_kc ? 0 : c.kc_next;
    // H's columns 6..11 are zero without extrinsic estimation (esekfom.hpp:218-220):
    // the filter step works on the first 6 error-state components
    dim = ext ? 12 : 6;
    slio_pose p;
    std::memcpy(p.rot, x->rot, sizeof(p.rot));
    std::memcpy(p.pos, x->pos, sizeof(p.pos));
    std::memcpy(p.rli, x->rli, sizeof(p.rli));
    std::memcpy(p.tli, x->tli, sizeof(p.tli));
    pose0 = make_pose(&p);
    return SLIO_OK;
  }

  // The control block comes in and goes out through the mapped host block:
  // pass 0 takes its pose by value and its filter step reads the block over
  // the bus (then keeps it in HBM); the step that ends the update writes x,
  // P and the flags back.  No copy-engine work on the path.  When the block
  // is written: before pass 0's launch on the fused path (that launch copies
  // it at its start), after pass 0's launch on the two-launch path (its
  // filter step, in the next launch, is the first reader).  Either way the
  // previous update has published, and its kernels still queued exit at
  // once (done in the HBM copy), so nothing else reads or writes the block.
  void fill_block() {
    IkfCtl& hc = *c.h_ctl;
    hc.x = *x;
    hc.xprop = *x;
    std::memcpy(hc.P, P, sizeof(double) * 576);
    hc.converge = 1;
    hc.t = 0;
    hc.done = 0;
    hc.search_now = 1;
    hc.passes = hc.searches = hc.valid_passes = 0;
    hc.mode = mode;
    hc.last_m = 0;
    hc.singular = 0;
    hc.published = 0;
    hc.timeout = 0;
    for (int k = 0; k < 24; ++k) hc.dxn[k] = 0.0;  // x == x_propagated on pass 0
  }

  SolveArgs args(int i) const {
    const bool p0 = i == first;
    const IkfCtl* src = p0 ? (const IkfCtl*)c.d_hctl : c.ctl;
    return SolveArgs{multi ? 0 : 1, dim, i - first, i, maxit, R, src, c.d_hctl};
  }

  // pass i: search / reuse kernels and k_super_sums (with the filter step on
  // a single rank; super rows only when multi)
  int pass(int i) {
    const bool p0 = i == first;
    const SolveArgs sa = args(i);
    // pass 0 always searches (converge starts true, esekfom.hpp:282)
    const int which = p0 ? 1 : (mode == SLIO_MODE_FIXED ? 1 : 2);
    if (fusable() && !(p0 && c.sw.no_fuse0)) {
      // one launch: search (or reuse) pass + sums + filter step.  The first
      // pass's launch copies the mapped host block into HBM, so the host
      // fills the block BEFORE that launch (measured: launching first and
      // handing the block over by a polled sequence word cost more than it
      // hid)
      if (p0) {
        // the previous update has published: nothing on the device still
        // reads or writes the block
        fill_block();
        if (!info_constants(P, dim, c.h_ctl->P11i, c.h_ctl->G)) {
          set_error("slio_ikf_update_device: singular covariance block P[:D, :D]");
          return SLIO_EINVAL;
        }
        SLIO_HSTAMP(c, 2);
      }
      const FuseArgs fa{c.ctl,   p0 ? (const IkfCtl*)c.d_hctl : nullptr,
                        c.d_seg, c.d_super,
                        c.ctl,   c.d_hctl,
                        c.count, R,
                        i,       maxit,
                        num_chunks(c.n), kNSeg,
                        0,       1,
                        nullptr, nullptr,
                        0};
      int rc = enqueue_pass(c, p0 ? &pose0 : nullptr, c.ctl, which, ext, &sa, true, false, nullptr, &fa);
      if (rc) return rc;
      if (p0) SLIO_HSTAMP(c, 3);
      SLIO_HIP(hipGetLastError());
      return SLIO_OK;
    }
    if (fused_rows() && !(p0 && c.sw.no_fuse0)) {
      const int nr = c.prm.nranks;
      const FuseArgs fa{c.ctl,   nullptr,
                        c.d_seg, c.d_super,
                        c.ctl,   c.d_hctl,
                        c.count, R,
                        i,       maxit,
                        num_chunks(c.n), kNSeg / nr,
                        c.prm.rank * (SLIO_NSUPER / nr), nr,
                        c.d_super, nullptr,
                        0};
      if (p0) fill_block();
      if (p0 && !info_constants(P, dim, c.h_ctl->P11i, c.h_ctl->G)) {
        set_error("slio_ikf_update_device: singular covariance block P[:D, :D]");
        return SLIO_EINVAL;
      }
      int rc = enqueue_pass(c, p0 ? &pose0 : nullptr, c.ctl, which, ext, &sa, true, false, nullptr, &fa);
      if (rc) return rc;
      SLIO_HIP(hipGetLastError());
      return SLIO_OK;
    }
    int rc = enqueue_pass(c, p0 ? &pose0 : nullptr, c.ctl, which, ext, &sa, !p0 || multi);
    if (rc) return rc;
    if (p0) {
      fill_block();
      // information-form constants of the update (P is fixed until its end),
      // formed on the host while pass 0's search runs; pass 0's filter step
      // reads them from the mapped block
      if (!info_constants(P, dim, c.h_ctl->P11i, c.h_ctl->G)) {
        (void)hipStreamSynchronize(c.stream);
        set_error("slio_ikf_update_device: singular covariance block P[:D, :D]");
        return SLIO_EINVAL;
      }
      if (!multi) enqueue_super(c, c.ctl, &sa);
    }
    SLIO_HIP(hipGetLastError());
    return SLIO_OK;
  }

  // Every pass runs as one fused launch (search or reuse pass + sums +
  // filter step, fused_tail) on a single rank with 2 lanes per query and no
  // sphere-first search, in either control flow (FIXED, or REFERENCE with
  // its reuse passes) and with or without extrinsic estimation (D = 12 / 6),
  // given at least 8 chunks per super-chunk (every segment row has a chunk).
  // SLIO_NO_FUSE=1 keeps two launches per pass.
  // the fused pass's configuration (2 lanes per query, no sphere-first
  // search, every segment row holds a chunk), whatever the rank count
  bool fused_ok() const {
    const int lpq = c.prm.lanes_per_query;
    return !c.sw.no_fuse && (lpq != 1 && lpq != 4 && lpq != 8) && !(c.prm.search_radius > 0.0f) &&
           num_chunks(c.n) >= (int64_t)kNSeg;
  }
  bool fusable() const {
    const bool off = c.sw.no_fuse;
    const int lpq = c.prm.lanes_per_query;
    return !off && !multi && c.prm.nranks == 1 &&
           (lpq != 1 && lpq != 4 && lpq != 8) && !(c.prm.search_radius > 0.0f) &&
           num_chunks(c.n) >= (int64_t)kNSeg;
  }
  // a rank of an all-reduce group: its pass, segment rows and super rows in
  // one launch (the rows-only fused tail), then the all-reduce and
  // k_ikf_solve -- no k_super_sums launch between the pass and the collective
  bool fused_rows() const { return multi && fused_ok() && (SLIO_NSUPER % c.prm.nranks) == 0; }

  // The whole update as one persistent launch (k_update_persist): the fused
  // configuration, and every chunk's workgroup resident at once (the
  // occupancy the device reports for the kernel, times its CUs).  That
  // count assumes the launch has the device to itself: with another live
  // handle on the device (its kernels, or another persistent launch, may
  // hold CUs while this launch's spinning workgroups wait for chunks that
  // cannot start) or a map shared with other handles, it takes a launch
  // per pass instead.
  bool persist_ok() {
    if (!c.sw.persist || c.sw.no_fuse0 || !fusable() || !c.goflag || c.ncu <= 0) return false;
    if (dev_users(c.prm.device, 0) > 1 || (c.map && c.map->users.size() > 1)) return false;
    if (c.persist_cap < 0) {
      int b6 = 0, b12 = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b6, k_update_persist<SLIO_SEARCH_U, 6>,
                                                       kSolveThreads, 0) != hipSuccess ||
          hipOccupancyMaxActiveBlocksPerMultiprocessor(&b12, k_update_persist<SLIO_SEARCH_U, 12>,
                                                       kSolveThreads, 0) != hipSuccess) {
        (void)hipGetLastError();
        b6 = b12 = 0;
      }
      c.persist_cap = (int64_t)std::min(b6, b12) * c.ncu;
    }
    return num_chunks(c.n) <= c.persist_cap;
  }
  int persist() {
    fill_block();
    if (!info_constants(P, dim, c.h_ctl->P11i, c.h_ctl->G)) {
      set_error("slio_ikf_update_device: singular covariance block P[:D, :D]");
      return SLIO_EINVAL;
    }
    if (++c.upd_seq <= 0) c.upd_seq = 1;
    c.h_ctl->seq = c.upd_seq;
    SLIO_HSTAMP(c, 2);
    const SolveArgs sa = args(first);
    FuseArgs fa{c.ctl,   (const IkfCtl*)c.d_hctl,
                c.d_seg, c.d_super,
                c.ctl,   c.d_hctl,
                c.count, R,
                first,   maxit,
                num_chunks(c.n), kNSeg,
                0,       1,
                nullptr, nullptr,
                c.upd_seq};
    fa.goflag = c.goflag;
    fa.wait_ticks = c.wait_ticks;
    if (int rc = enqueue_pass(c, &pose0, c.ctl, 1, ext, &sa, true, false, nullptr, &fa, maxit - first)) return rc;
    SLIO_HSTAMP(c, 3);
    SLIO_HIP(hipGetLastError());
    return SLIO_OK;
  }

  // multi-rank: the filter step of pass i after the all-reduce, on every rank
  int solve(int i) {
    const SolveArgs sa = args(i);
    if (dim == 12)
      k_ikf_solve<12><<<1, kSolveThreads, 0, c.stream>>>(c.ctl, sa.src, c.d_hctl, c.d_super, R, i, maxit);
    else
      k_ikf_solve<6><<<1, kSolveThreads, 0, c.stream>>>(c.ctl, sa.src, c.d_hctl, c.d_super, R, i, maxit);
    SLIO_HIP(hipGetLastError());
    return SLIO_OK;
  }

  int finish(slio_ikf_stats* stats) {
    SLIO_HSTAMP(c, 4);
    SLIO_HIP(wait_published(c));
    SLIO_HSTAMP(c, 5);
    const IkfCtl& hc = *c.h_ctl;
    // a wait that gave up let a pass run before its predecessor's filter step
    // (or skipped passes): the result is void even if the update ended
    if (!hc.done || hc.timeout) {
      const bool to = hc.timeout != 0;
      const std::string st = "(passes " + std::to_string(hc.passes) + ", searches " + std::to_string(hc.searches) +
                             ", converge " + std::to_string(hc.converge) + ", published " +
                             std::to_string(hc.published) + ")";
      // some workgroups (or ranks) may have arrived on the handle's counters
      // and others never will: back to zero before the next update
      reset_update_counters(c);
      if (to) {
        set_error("slio_ikf_update_device: a device-side wait gave up (persistent pass flag or group gate, "
                  "> 1 s) " + st + "; the handle's arrival counters were reset");
        return SLIO_ETIMEOUT;
      }
      set_error("slio_ikf_update_device: the update did not complete " + st);
      return SLIO_EDEVICE;
    }
    if (hc.singular) {
      set_error("slio_ikf_update_device: singular covariance");
      return SLIO_EINVAL;
    }
    *x = hc.x;
    std::memcpy(P, hc.P, sizeof(double) * 576);
    if (stats) {
      stats->passes = hc.passes;
      stats->searches = hc.searches;
      stats->valid_passes = hc.valid_passes;
      stats->converged = hc.converge;
      stats->last_m = hc.last_m;
      stats->device_ms = 0.0;
    }
    return SLIO_OK;
  }
};

// The group's in-device all-reduce (slio_create_group's reduce backend when
// ranks share a device, or on request across peer-accessible devices): one
// workgroup on rank 0's stream sums the ranks' 8 x 91 super rows in rank
// order and writes the total back into every rank's buffer.  Each super row
// has exactly one non-zero contributor (the rank owning that super-chunk), so
// the sum is an exact gather: the same bits as RCCL's SUM or one rank alone.
struct GroupSupers {
  double* sup[SLIO_NSUPER];
  int n;
};
__global__ __launch_bounds__(256) void k_group_reduce(GroupSupers g) {
  for (int e = threadIdx.x; e < SLIO_NSUPER * SLIO_NPROD; e += blockDim.x) {
    double v = g.sup[0][e];
    for (int r = 1; r < g.n; ++r) v = v + g.sup[r][e];
    for (int r = 0; r < g.n; ++r) g.sup[r][e] = v;
  }
}

// Fused group pass: between a rank's pass i and i + 1 on its stream, one
// thread waits until the group's filter step of pass i has run (the group's
// control block counts the pass, or ends the update, or a newer update owns
// it: seq).  The last rank to arrive runs that step inside its pass launch
// (fused_tail), so the wait is for a workgroup that is already running: no
// workgroup of the next pass occupies the device meanwhile, and the ranks'
// pass workgroups (<= the scan's chunks) always fit beside the N gates.  A
// wait past ~1 s gives up (the next pass then exits and the update reports
// that it did not complete) instead of hanging.
__global__ __launch_bounds__(64) void k_group_gate(const uint32_t* __restrict__ garrive, int pass_idx, int32_t seq,
                                                   IkfCtl* __restrict__ hblk, uint64_t wait_ticks) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = wall_clock64();
  const unsigned long long lim = wait_ticks ? wait_ticks : 100000000ull;
  if (lim == 1) {  // give up at once (the test hook of slio_debug_wait_limit)
    __hip_atomic_store(&hblk->timeout, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  while (true) {
    const uint64_t fl = __hip_atomic_load((const guint64*)(const uint64_t*)(garrive + 2), __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
    const int32_t fseq = (int32_t)(fl >> 32);
    const bool done = (fl & 0x80000000ull) != 0;
    const int32_t passes = (int32_t)(fl & 0x7fffffffull);
    // this update's step has counted the pass or ended the update, or a newer
    // update owns the group (a stale gate)
    if ((fseq == seq && (done || passes >= pass_idx)) || (int32_t)(fseq - seq) > 0) return;
    if (wall_clock64() - t0 > lim) {  // 100 MHz: 1 s
      // the group's mapped host block reports the timeout (SLIO_ETIMEOUT)
      __hip_atomic_store(&hblk->timeout, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// the in-library all-reduce of a handle's super rows (RCCL), on its stream
static int comm_allreduce(Ctx& c) {
  const ncclResult_t r = ncclAllReduce(c.d_super, c.d_super, (size_t)SLIO_NSUPER * SLIO_NPROD, ncclDouble,
                                       ncclSum, (ncclComm_t)c.comm, c.stream);
  if (r != ncclSuccess) {
    set_error(std::string("slio: ncclAllReduce: ") + ncclGetErrorString(r));
    return SLIO_EDEVICE;
  }
  return SLIO_OK;
}

}  // namespace slio

extern "C" {

int slio_ikf_update_device(slio_handle h, slio_state* x, double P[576], double R,
                           int maximum_iter, int extrinsic_est, int mode,
                           slio_allreduce_fn reduce, void* reduce_ctx, slio_ikf_stats* stats) {
  SLIO_CHECK_H(h);
  if (!x || !P || !(R > 0.0) || maximum_iter < 1 ||
      (mode != SLIO_MODE_REFERENCE && mode != SLIO_MODE_FIXED)) {
    set_error("slio_ikf_update_device: bad arguments");
    return SLIO_EINVAL;
  }
  Ctx& c = h->c;
  SLIO_HSTAMP(c, 0);
  // the caller's reduce hook, else the handle's communicator (any number of
  // ranks, one included: the same path as several)
  const bool comm = !reduce && c.comm;
  if (!reduce && !comm && c.prm.nranks > 1) {
    set_error("slio_ikf_update_device: nranks > 1 needs a reduce hook or slio_comm_init");
    return SLIO_ESTATE;
  }
  UpdateRun u(c, x, P, R, maximum_iter, extrinsic_est, mode, reduce || comm);
  if (int rc = u.begin()) return rc;
  SLIO_HSTAMP(c, 1);
  c.last_path = (!u.multi && u.persist_ok()) ? 1 : 0;
  if (c.last_path) {
    if (int rc = u.persist()) return rc;
  } else
  for (int i = u.first; i < maximum_iter; ++i) {
    // single rank: the filter step runs in the super-sum kernel's last block
    // (or the search pass's tail); multi-rank: pass -> all-reduce of the
    // super sums -> k_ikf_solve
    if (int rc = u.pass(i)) return rc;
    if (reduce) {
      if (reduce(reduce_ctx, c.d_super, (int64_t)SLIO_NSUPER * SLIO_NPROD, (void*)c.stream)) {
        set_error("slio_ikf_update_device: reduce callback failed");
        return SLIO_EDEVICE;
      }
    } else if (comm) {
      if (int rc = comm_allreduce(c)) return rc;
    }
    if (u.multi)
      if (int rc = u.solve(i)) return rc;
  }
  const int rc = u.finish(stats);
  SLIO_HSTAMP(c, 6);
  return rc;
}

int slio_comm_unique_id(uint8_t id[SLIO_COMM_ID_BYTES]) {
  static_assert(sizeof(ncclUniqueId) <= SLIO_COMM_ID_BYTES, "ncclUniqueId size");
  if (!id) return SLIO_EINVAL;
  ncclUniqueId u;
  const ncclResult_t r = ncclGetUniqueId(&u);
  if (r != ncclSuccess) {
    set_error(std::string("slio_comm_unique_id: ") + ncclGetErrorString(r));
    return SLIO_EDEVICE;
  }
  std::memset(id, 0, SLIO_COMM_ID_BYTES);
  std::memcpy(id, &u, sizeof(u));
  return SLIO_OK;
}

int slio_comm_init(slio_handle h, const uint8_t id[SLIO_COMM_ID_BYTES]) {
  SLIO_CHECK_H(h);
  Ctx& c = h->c;
  if (!id || c.comm) {
    set_error("slio_comm_init: null id or communicator already set");
    return SLIO_EINVAL;
  }
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  ncclComm_t comm = nullptr;
  const ncclResult_t r = ncclCommInitRank(&comm, c.prm.nranks, u, c.prm.rank);
  if (r != ncclSuccess) {
    set_error(std::string("slio_comm_init: ncclCommInitRank: ") + ncclGetErrorString(r));
    return SLIO_EDEVICE;
  }
  c.comm = comm;
  return SLIO_OK;
}

int slio_create_group(slio_handle* out, int ndev, const int* devices, const slio_params* p) {
  if (!out || !devices || !p || ndev < 1 || (SLIO_NSUPER % ndev) != 0) {
    set_error("slio_create_group: bad arguments (ndev must divide 8)");
    return SLIO_EINVAL;
  }
  int caller_dev = 0;
  SLIO_HIP(hipGetDevice(&caller_dev));
  for (int r = 0; r < ndev; ++r) out[r] = nullptr;
  // reduce backend: RCCL (ncclCommInitAll) when every rank has its own GPU;
  // the in-device reduce when ranks share a device (RCCL refuses that), or
  // when SLIO_GROUP_REDUCE=device asks for it across peer-accessible GPUs
  bool shared = false;
  for (int r = 0; r < ndev; ++r)
    for (int q = 0; q < r; ++q) shared = shared || devices[q] == devices[r];
  const char* env = std::getenv("SLIO_GROUP_REDUCE");
  int kind = shared ? 2 : 1;
  if (env && std::strcmp(env, "device") == 0) kind = 2;
  if (env && std::strcmp(env, "rccl") == 0) {
    if (shared) {
      set_error("slio_create_group: SLIO_GROUP_REDUCE=rccl needs one device per rank");
      return SLIO_EINVAL;
    }
    kind = 1;
  }
  int rc = SLIO_OK;
  for (int r = 0; r < ndev && !rc; ++r) {
    slio_params q = *p;
    q.device = devices[r];
    q.rank = r;
    q.nranks = ndev;
    rc = slio_create(&out[r], &q);
  }
  if (!rc && kind == 1) {
    std::vector<ncclComm_t> comms((size_t)ndev, nullptr);
    const ncclResult_t r = ncclCommInitAll(comms.data(), ndev, devices);
    if (r != ncclSuccess) {
      set_error(std::string("slio_create_group: ncclCommInitAll: ") + ncclGetErrorString(r));
      rc = SLIO_EDEVICE;
    } else {
      for (int q = 0; q < ndev; ++q) out[q]->c.comm = comms[q];
    }
  }
  if (!rc && kind == 2) {
    // rank 0's device reads and writes every rank's super rows
    for (int r = 1; r < ndev && !rc; ++r) {
      if (devices[r] == devices[0]) continue;
      int ok = 0;
      if (hipDeviceCanAccessPeer(&ok, devices[0], devices[r]) != hipSuccess || !ok) {
        set_error("slio_create_group: in-device reduce needs peer access from rank 0's GPU");
        rc = SLIO_EDEVICE;
        break;
      }
      (void)hipSetDevice(devices[0]);
      const hipError_t e = hipDeviceEnablePeerAccess(devices[r], 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
        set_error(std::string("slio_create_group: hipDeviceEnablePeerAccess: ") + hipGetErrorString(e));
        rc = SLIO_EDEVICE;
      }
      (void)hipGetLastError();
    }
    for (int r = 0; r < ndev && !rc; ++r) {
      (void)hipSetDevice(devices[r]);
      if (hipEventCreateWithFlags(&out[r]->c.grp_ev, hipEventDisableTiming) != hipSuccess) {
        set_error("slio_create_group: hipEventCreate failed");
        rc = SLIO_EDEVICE;
      }
    }
    if (!rc) {
      // the fused group pass's buffers, on rank 0's device
      (void)hipSetDevice(devices[0]);
      Ctx& c0 = out[0]->c;
      if (hipMalloc(&c0.gsup, sizeof(double) * SLIO_NSUPER * SLIO_NPROD) != hipSuccess ||
          hipMalloc(&c0.garrive, 4 * sizeof(uint32_t)) != hipSuccess ||
          hipMemset(c0.garrive, 0, 4 * sizeof(uint32_t)) != hipSuccess) {
        set_error("slio_create_group: allocation failed");
        rc = SLIO_ENOMEM;
      }
    }
  }
  if (rc) {
    for (int r = 0; r < ndev; ++r) {
      slio_destroy(out[r]);
      out[r] = nullptr;
    }
  } else {
    for (int r = 0; r < ndev; ++r) out[r]->c.group_reduce = kind;
  }
  (void)hipSetDevice(caller_dev);
  return rc;
}

int slio_group_reduce_kind(slio_handle h) {
  if (!h) return SLIO_EINVAL;
  return h->c.group_reduce;
}

namespace slio {

// slio_group_ikf_update's body; the caller restores the device and, after an
// error, drains every rank's stream
static int group_update(slio_handle* hs, int n, slio_state* x, double P[576], double R, int maximum_iter,
                        int extrinsic_est, int mode, slio_ikf_stats* stats) {
  const int kind = hs[0]->c.group_reduce;
  // every rank starts from the caller's x and P and ends with the same bits
  std::vector<slio_state> xs((size_t)n, *x);
  std::vector<std::vector<double>> Ps((size_t)n, std::vector<double>(P, P + 576));
  std::vector<UpdateRun> runs;
  runs.reserve((size_t)n);
  for (int r = 0; r < n; ++r)
    runs.emplace_back(hs[r]->c, &xs[r], Ps[r].data(), R, maximum_iter, extrinsic_est, mode, true);
  for (int r = 0; r < n; ++r) {
    SLIO_HIP(hipSetDevice(hs[r]->c.prm.device));
    if (int rc = runs[r].begin()) return rc;
  }
  GroupSupers gs{};
  gs.n = n;
  for (int r = 0; r < n; ++r) gs.sup[r] = hs[r]->c.d_super;
  Ctx& c0 = hs[0]->c;
  // Fused group pass (ranks sharing one device): per pass ONE launch per rank
  // (search or reuse pass + segment and super rows into the group's buffer +,
  // in the rank that arrives last, the filter step on the group's control
  // block, fused_tail) and, before every pass but the first, one gate launch
  // that waits for the previous pass's filter step; no events, no reduce or
  // filter-step launches, no host round trip until the end
  bool gfused = kind == 2 && c0.gsup && n > 1 && runs[0].fused_ok();
  for (int r = 1; r < n && gfused; ++r) gfused = hs[r]->c.prm.device == c0.prm.device;
  if (gfused) {
    const int64_t C = num_chunks(c0.n);
    const bool hs_on = c0.hstamp;
    if (hs_on) {
      c0.hst[0] = mono_ns();
      c0.hst[4] = c0.hst[5] = c0.hst[6] = 0;
    }
    if (++c0.upd_seq <= 0) c0.upd_seq = 1;
    const int32_t seq = c0.upd_seq;
    for (int r = 0; r < n; ++r) hs[r]->c.group_seq = seq;
    int rc = SLIO_OK;
    for (int i = runs[0].first; i < maximum_iter && !rc; ++i) {
      const bool p0 = i == runs[0].first;
      if (p0) {
        // the group's control block is rank 0's: its mapped host block in,
        // its pass-0 launch copies it to HBM
        runs[0].fill_block();
        c0.h_ctl->seq = seq;
        if (!info_constants(P, runs[0].dim, c0.h_ctl->P11i, c0.h_ctl->G)) {
          set_error("slio_group_ikf_update: singular covariance block P[:D, :D]");
          rc = SLIO_EINVAL;
          break;
        }
      }
      const int which = p0 ? 1 : (mode == SLIO_MODE_FIXED ? 1 : 2);
      for (int r = 0; r < n && !rc; ++r) {
        Ctx& cr = hs[r]->c;
        if (!p0) k_group_gate<<<1, 64, 0, cr.stream>>>(c0.garrive, i - runs[0].first, seq, c0.d_hctl, c0.wait_ticks);
        const SolveArgs sa = runs[r].args(i);
        const FuseArgs fa{c0.ctl,  (p0 && r == 0) ? (const IkfCtl*)c0.d_hctl : nullptr,
                          cr.d_seg, c0.gsup,
                          c0.ctl,  c0.d_hctl,
                          cr.count, R,
                          i,       maximum_iter,
                          C,       kNSeg / n,
                          r * (SLIO_NSUPER / n), n,
                          c0.gsup, c0.garrive,
                          seq,     nullptr,
                          c0.wait_ticks};
        rc = enqueue_pass(cr, p0 ? &runs[r].pose0 : nullptr, c0.ctl, which, extrinsic_est, &sa, true, false,
                          nullptr, &fa);
        if (!rc && hipGetLastError() != hipSuccess) {
          set_error("slio_group_ikf_update: launch failed");
          rc = SLIO_EDEVICE;
        }
      }
    }
    for (int r = 0; r < n; ++r) hs[r]->c.group_seq = 0;
    if (rc) return rc;
    if (hs_on) {
      c0.hst[1] = mono_ns();
      c0.hst[4] = c0.hst[1] - c0.hst[0];  // every launch (passes and gates)
    }
    // the step that ends the update runs in whichever rank arrives last:
    // wait for rank 0's published word while any rank's stream still has work
    {
      volatile int32_t* pub = &c0.h_ctl->published;
      for (uint32_t it = 1; !*pub; ++it) {
        if ((it & 255) == 0) {
          bool idle = true;
          for (int r = 0; r < n && idle; ++r) {
            const hipError_t e = hipStreamQuery(hs[r]->c.stream);
            if (e != hipSuccess && e != hipErrorNotReady) return SLIO_EDEVICE;
            idle = e == hipSuccess;
          }
          if (idle) break;  // every launch has ended: the flags tell whether it published
        }
        __builtin_ia32_pause();
      }
      std::atomic_thread_fence(std::memory_order_acquire);
    }
    if (hs_on) c0.hst[2] = mono_ns();
    slio_ikf_stats st0{};
    c0.hstamp = false;  // (finish's own stamps would overwrite the group's)
    const int rc2 = runs[0].finish(&st0);
    c0.hstamp = hs_on;
    if (rc2) return rc2;
    *x = xs[0];
    std::memcpy(P, Ps[0].data(), sizeof(double) * 576);
    if (stats) *stats = st0;
    if (hs_on) c0.hst[3] = mono_ns();
    return SLIO_OK;
  }
  // host stamps of the group update on rank 0's handle (slio_debug_host_stamps):
  // [0] entry, [1] every pass enqueued, [2] every rank's result seen, [3] exit;
  // [4] / [5] / [6] host ns spent enqueueing the ranks' pass launches / the
  // reduce (events + k_group_reduce or the RCCL group) / the filter steps
  const bool hs_on = c0.hstamp;
  int64_t t_a = 0;
  if (hs_on) {
    c0.hst[0] = mono_ns();
    c0.hst[4] = c0.hst[5] = c0.hst[6] = 0;
  }
  for (int i = runs[0].first; i < maximum_iter; ++i) {
    if (hs_on) t_a = mono_ns();
    for (int r = 0; r < n; ++r) {
      SLIO_HIP(hipSetDevice(hs[r]->c.prm.device));
      if (int rc = runs[r].pass(i)) return rc;
      if (kind == 2 && r > 0) SLIO_HIP(hipEventRecord(hs[r]->c.grp_ev, hs[r]->c.stream));
    }
    if (hs_on) {
      const int64_t t = mono_ns();
      c0.hst[4] += t - t_a;
      t_a = t;
    }
    if (kind == 1) {
      // one RCCL all-reduce of the 8 x 91 super rows per pass, all ranks
      // enqueued by this thread as one group (each on its own stream)
      if (ncclGroupStart() != ncclSuccess) {
        set_error("slio_group_ikf_update: ncclGroupStart");
        return SLIO_EDEVICE;
      }
      int rc = SLIO_OK;
      for (int r = 0; r < n && !rc; ++r) rc = comm_allreduce(hs[r]->c);
      if (ncclGroupEnd() != ncclSuccess && !rc) {
        set_error("slio_group_ikf_update: ncclGroupEnd");
        rc = SLIO_EDEVICE;
      }
      if (rc) return rc;
    } else {
      // in-device reduce on rank 0's stream after every rank's pass; every
      // rank's filter step after the reduce
      SLIO_HIP(hipSetDevice(c0.prm.device));
      for (int r = 1; r < n; ++r) SLIO_HIP(hipStreamWaitEvent(c0.stream, hs[r]->c.grp_ev, 0));
      k_group_reduce<<<1, 256, 0, c0.stream>>>(gs);
      SLIO_HIP(hipGetLastError());
      SLIO_HIP(hipEventRecord(c0.grp_ev, c0.stream));
      for (int r = 1; r < n; ++r) {
        SLIO_HIP(hipSetDevice(hs[r]->c.prm.device));
        SLIO_HIP(hipStreamWaitEvent(hs[r]->c.stream, c0.grp_ev, 0));
      }
    }
    if (hs_on) {
      const int64_t t = mono_ns();
      c0.hst[5] += t - t_a;
      t_a = t;
    }
    for (int r = 0; r < n; ++r) {
      SLIO_HIP(hipSetDevice(hs[r]->c.prm.device));
      if (int rc2 = runs[r].solve(i)) return rc2;
    }
    if (hs_on) c0.hst[6] += mono_ns() - t_a;
  }
  if (hs_on) c0.hst[1] = mono_ns();
  slio_ikf_stats st0{};
  for (int r = 0; r < n; ++r) {
    SLIO_HIP(hipSetDevice(hs[r]->c.prm.device));
    slio_ikf_stats st{};
    const bool keep = hs[r]->c.hstamp;
    hs[r]->c.hstamp = false;  // (finish's own stamps would overwrite the group's)
    const int rc = runs[r].finish(&st);
    hs[r]->c.hstamp = keep;
    if (rc) return rc;
    if (r == 0) st0 = st;
  }
  if (hs_on) c0.hst[2] = mono_ns();
  for (int r = 1; r < n; ++r)
    if (std::memcmp(&xs[r], &xs[0], sizeof(slio_state)) != 0 ||
        std::memcmp(Ps[r].data(), Ps[0].data(), sizeof(double) * 576) != 0) {
      set_error("slio_group_ikf_update: ranks disagree (x or P differ bitwise)");
      return SLIO_EDEVICE;
    }
  *x = xs[0];
  std::memcpy(P, Ps[0].data(), sizeof(double) * 576);
  if (stats) *stats = st0;
  if (hs_on) c0.hst[3] = mono_ns();
  return SLIO_OK;
}

}  // namespace slio

int slio_group_ikf_update(slio_handle* hs, int n, slio_state* x, double P[576], double R, int maximum_iter,
                          int extrinsic_est, int mode, slio_ikf_stats* stats) {
  if (!hs || n < 1 || !x || !P || !(R > 0.0) || maximum_iter < 1 ||
      (mode != SLIO_MODE_REFERENCE && mode != SLIO_MODE_FIXED)) {
    set_error("slio_group_ikf_update: bad arguments");
    return SLIO_EINVAL;
  }
  for (int r = 0; r < n; ++r)
    if (!hs[r] || hs[r]->c.prm.nranks != n || hs[r]->c.prm.rank != r || !hs[r]->c.group_reduce ||
        hs[r]->c.group_reduce != hs[0]->c.group_reduce) {
      set_error("slio_group_ikf_update: handles must be ranks 0..n-1 of one group (slio_create_group)");
      return SLIO_EINVAL;
    }
  int caller_dev = 0;
  SLIO_HIP(hipGetDevice(&caller_dev));
  const int rc = group_update(hs, n, x, P, R, maximum_iter, extrinsic_est, mode, stats);
  if (rc) {
    // work already queued on the other ranks must not outlive the call (the
    // next update refills their control blocks)
    for (int r = 0; r < n; ++r) {
      (void)hipSetDevice(hs[r]->c.prm.device);
      (void)hipStreamSynchronize(hs[r]->c.stream);
    }
    for (int r = 0; r < n; ++r) {
      (void)hipSetDevice(hs[r]->c.prm.device);
      reset_update_counters(hs[r]->c);
    }
  }
  (void)hipSetDevice(caller_dev);
  return rc;
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
  const bool keep = (enable & SLIO_PROFILE_KEEP) != 0;
  const int sel = enable & ~SLIO_PROFILE_KEEP;
  c.prof_mask = (sel == 1) ? 7 : ((sel >> 1) & 7);
  c.prof = c.prof_mask != 0;
  if (!keep)
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
  SLIO_HIP(wait_stream(c));
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
  if (int rc = nbr_settle_shared(c)) return rc;
  if (c.nbr_stale) {
    set_error("slio_get_neighbors: another handle sharing the map rebuilt it after this handle's last "
              "search pass; run a search pass again");
    return SLIO_ESTATE;
  }
  SLIO_HIP(hipStreamSynchronize(c.stream));
  if (n <= 0) return SLIO_OK;
  if (idx) SLIO_HIP(hipMemcpy(idx, c.nbr_idx + b * 5, 4 * 5 * n, hipMemcpyDeviceToHost));
  if (sqd) SLIO_HIP(hipMemcpy(sqd, c.nbr_sqd + b * 5, 4 * 5 * n, hipMemcpyDeviceToHost));
  if (sel) SLIO_HIP(hipMemcpy(sel, c.sel + b, n, hipMemcpyDeviceToHost));
  return SLIO_OK;
}

int slio_far_queries(slio_handle h, int64_t* n) {
  SLIO_CHECK_H(h);
  uint32_t v[16] = {};
  SLIO_HIP(hipStreamSynchronize(h->c.stream));
  SLIO_HIP(hipMemcpy(v, h->c.count, sizeof(v), hipMemcpyDeviceToHost));
  if (n) *n = v[6];
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


#ifdef SLIO_SOLVE_STAMP
extern "C" int slio_dbg_solve_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sstamp), sizeof(g_sstamp)) == hipSuccess ? 0 : -1;
}
#endif
