// frontend_oracle.cpp -- CPU restatement of the LIO-SAM / LeGO-LOAM front-end
// hot path.  TEST INFRASTRUCTURE ONLY: linked
// by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline, never by
// the product path (agi_lidar_slam_amd/).
//
// Parity unpinned: the reference nodes need PCL / OpenCV / Eigen / ROS, none
// of which exist here, so this is restated from the reference text
// (file:line below) and the published algorithms of the third-party pieces
// (pcl::getTransformation, Eigen Transform::inverse / 3x3 inverse, PCL
// VoxelGrid::applyFilter).  Deterministic choices where the reference is
// implementation-defined (documented in DESIGN.md §front-end):
//   * float sin/cos/atan2 are evaluated in double and rounded to float (the
//     correctly rounded float value);
//   * std::sort ties (featureExtraction.cpp:201-202, VoxelGrid's index sort)
//     are broken by point index (orc_lio_features_ex / voxel_grid_pcl_order
//     also run the reference's own std::sort calls, to count ties and show
//     whether the order changes anything);
//   * smoothness entries the reference never initialises (index < 5 or
//     >= cloudSize - 5; read for ring 0 sector 0, featureExtraction.cpp:196)
//     are {value 0, ind = own index} with neighbourPicked = 1.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace {

// float trig as correctly rounded values
inline float fcos(float a) { return (float)std::cos((double)a); }
inline float fsin(float a) { return (float)std::sin((double)a); }
inline float fatan2(float y, float x) { return (float)std::atan2((double)y, (double)x); }

struct Aff {  // Eigen::Affine3f, row-major 3x4
  float m[3][4];
};

// pcl::getTransformation(x, y, z, roll, pitch, yaw) (pcl/common/impl/eigen.hpp)
Aff get_transformation(float x, float y, float z, float roll, float pitch, float yaw) {
  const float A = fcos(yaw), B = fsin(yaw), C = fcos(pitch), D = fsin(pitch), E = fcos(roll),
              F = fsin(roll), DE = D * E, DF = D * F;
  Aff t;
  t.m[0][0] = A * C;
  t.m[0][1] = A * DF - B * E;
  t.m[0][2] = B * F + A * DE;
  t.m[0][3] = x;
  t.m[1][0] = B * C;
  t.m[1][1] = A * E + B * DF;
  t.m[1][2] = B * DE - A * F;
  t.m[1][3] = y;
  t.m[2][0] = -D;
  t.m[2][1] = C * F;
  t.m[2][2] = C * E;
  t.m[2][3] = z;
  return t;
}

// Eigen cofactor_3x3<i, j>
inline float cof(const Aff& a, int i, int j) {
  const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
  return a.m[i1][j1] * a.m[i2][j2] - a.m[i1][j2] * a.m[i2][j1];
}

// Eigen Transform<float,3,Affine>::inverse(): linear().inverse() (3x3
// cofactor inverse, InverseImpl.h) and t' = -(R^-1 t)
Aff inverse(const Aff& a) {
  const float c0 = cof(a, 0, 0), c1 = cof(a, 1, 0), c2 = cof(a, 2, 0);
  const float det = (c0 * a.m[0][0] + c1 * a.m[1][0]) + c2 * a.m[2][0];
  const float invdet = 1.0f / det;
  Aff r;
  r.m[0][0] = c0 * invdet;
  r.m[0][1] = c1 * invdet;
  r.m[0][2] = c2 * invdet;
  r.m[1][0] = cof(a, 0, 1) * invdet;
  r.m[1][1] = cof(a, 1, 1) * invdet;
  r.m[1][2] = cof(a, 2, 1) * invdet;
  r.m[2][0] = cof(a, 0, 2) * invdet;
  r.m[2][1] = cof(a, 1, 2) * invdet;
  r.m[2][2] = cof(a, 2, 2) * invdet;
  for (int i = 0; i < 3; ++i)
    r.m[i][3] = -((r.m[i][0] * a.m[0][3] + r.m[i][1] * a.m[1][3]) + r.m[i][2] * a.m[2][3]);
  return r;
}

// Affine * Affine: linear = L.linear * R.linear, t = L.linear * R.t + L.t
Aff compose(const Aff& l, const Aff& r) {
  Aff o;
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j)
      o.m[i][j] = (l.m[i][0] * r.m[0][j] + l.m[i][1] * r.m[1][j]) + l.m[i][2] * r.m[2][j];
    o.m[i][3] = ((l.m[i][0] * r.m[0][3] + l.m[i][1] * r.m[1][3]) + l.m[i][2] * r.m[2][3]) + l.m[i][3];
  }
  return o;
}

// imageProjection.cpp:492-529 findRotation
void find_rotation(double pointTime, const double* imuTime, const double* rx, const double* ry,
                   const double* rz, int imuPointerCur, float* ox, float* oy, float* oz) {
  int f = 0;
  while (f < imuPointerCur) {
    if (pointTime < imuTime[f]) break;
    ++f;
  }
  if (pointTime > imuTime[f] || f == 0) {
    *ox = (float)rx[f];
    *oy = (float)ry[f];
    *oz = (float)rz[f];
  } else {
    const int b = f - 1;
    const double rf = (pointTime - imuTime[b]) / (imuTime[f] - imuTime[b]);
    const double rb = (imuTime[f] - pointTime) / (imuTime[f] - imuTime[b]);
    *ox = (float)(rx[f] * rf + rx[b] * rb);
    *oy = (float)(ry[f] * rf + ry[b] * rb);
    *oz = (float)(rz[f] * rf + rz[b] * rb);
  }
}


// pcl::VoxelGrid<PointXYZI>::applyFilter with downsample_all_data_ (PCL 1.10
// VoxelGrid::applyFilter + CentroidPoint) on the points xyzi[pos[q]]; writes
// the centroids to out, returns their number.  Index ties by position.
int64_t voxel_grid(const float* xyzi, const std::vector<int64_t>& pos, float leaf, float* out) {
  if (pos.empty()) return 0;
  const float inv = 1.0f / leaf;
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (int64_t p : pos)
    for (int a = 0; a < 3; ++a) {
      mn[a] = std::min(mn[a], xyzi[p * 4 + a]);
      mx[a] = std::max(mx[a], xyzi[p * 4 + a]);
    }
  const int64_t dx = (int64_t)((mx[0] - mn[0]) * inv) + 1;
  const int64_t dy = (int64_t)((mx[1] - mn[1]) * inv) + 1;
  const int64_t dz = (int64_t)((mx[2] - mn[2]) * inv) + 1;
  int64_t ns = 0;
  if (dx * dy * dz > (int64_t)INT32_MAX) {  // PCL: output = input
    for (int64_t p : pos) std::memcpy(out + (ns++) * 4, xyzi + p * 4, 16);
    return ns;
  }
  int minb[3], divb[3];
  for (int a = 0; a < 3; ++a) {
    minb[a] = (int)std::floor(mn[a] * inv);
    divb[a] = (int)std::floor(mx[a] * inv) - minb[a] + 1;
  }
  const int mul[3] = {1, divb[0], divb[0] * divb[1]};
  std::vector<std::pair<uint32_t, int64_t>> iv;
  iv.reserve(pos.size());
  for (size_t q = 0; q < pos.size(); ++q) {
    const float* pp = xyzi + pos[q] * 4;
    int ijk[3];
    for (int a = 0; a < 3; ++a) ijk[a] = (int)(std::floor(pp[a] * inv) - (float)minb[a]);
    iv.emplace_back((uint32_t)(ijk[0] * mul[0] + ijk[1] * mul[1] + ijk[2] * mul[2]), (int64_t)q);
  }
  std::sort(iv.begin(), iv.end());
  size_t a0 = 0;
  while (a0 < iv.size()) {
    size_t a1 = a0 + 1;
    while (a1 < iv.size() && iv[a1].first == iv[a0].first) ++a1;
    float sm[4] = {0, 0, 0, 0};
    for (size_t q = a0; q < a1; ++q)
      for (int c = 0; c < 4; ++c) sm[c] += xyzi[pos[iv[q].second] * 4 + c];
    const float cnt = (float)(a1 - a0);
    for (int c = 0; c < 4; ++c) out[ns * 4 + c] = sm[c] / cnt;
    ++ns;
    a0 = a1;
  }
  return ns;
}

// The same VoxelGrid with PCL 1.10's own index sort: std::sort of
// {idx, cloud_point_index} with operator< on idx only (voxel_grid.hpp,
// cloud_point_index_idx), i.e. libstdc++ introsort's order inside a voxel.
int64_t voxel_grid_pcl_order(const float* xyzi, const std::vector<int64_t>& pos, float leaf, float* out) {
  struct Idx {
    uint32_t idx, cpi;
    bool operator<(const Idx& o) const { return idx < o.idx; }
  };
  if (pos.empty()) return 0;
  const float inv = 1.0f / leaf;
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (int64_t p : pos)
    for (int a = 0; a < 3; ++a) {
      mn[a] = std::min(mn[a], xyzi[p * 4 + a]);
      mx[a] = std::max(mx[a], xyzi[p * 4 + a]);
    }
  const int64_t dx = (int64_t)((mx[0] - mn[0]) * inv) + 1;
  const int64_t dy = (int64_t)((mx[1] - mn[1]) * inv) + 1;
  const int64_t dz = (int64_t)((mx[2] - mn[2]) * inv) + 1;
  int64_t ns = 0;
  if (dx * dy * dz > (int64_t)INT32_MAX) {
    for (int64_t p : pos) std::memcpy(out + (ns++) * 4, xyzi + p * 4, 16);
    return ns;
  }
  int minb[3], divb[3];
  for (int a = 0; a < 3; ++a) {
    minb[a] = (int)std::floor(mn[a] * inv);
    divb[a] = (int)std::floor(mx[a] * inv) - minb[a] + 1;
  }
  const int mul[3] = {1, divb[0], divb[0] * divb[1]};
  std::vector<Idx> iv;
  iv.reserve(pos.size());
  for (size_t q = 0; q < pos.size(); ++q) {
    const float* pp = xyzi + pos[q] * 4;
    int ijk[3];
    for (int a = 0; a < 3; ++a) ijk[a] = (int)(std::floor(pp[a] * inv) - (float)minb[a]);
    iv.push_back(Idx{(uint32_t)(ijk[0] * mul[0] + ijk[1] * mul[1] + ijk[2] * mul[2]), (uint32_t)q});
  }
  std::sort(iv.begin(), iv.end());
  size_t a0 = 0;
  while (a0 < iv.size()) {
    size_t a1 = a0 + 1;
    while (a1 < iv.size() && iv[a1].idx == iv[a0].idx) ++a1;
    float sm[4] = {0, 0, 0, 0};
    for (size_t q = a0; q < a1; ++q)
      for (int c = 0; c < 4; ++c) sm[c] += xyzi[pos[iv[q].cpi] * 4 + c];
    const float cnt = (float)(a1 - a0);
    for (int c = 0; c < 4; ++c) out[ns * 4 + c] = sm[c] / cnt;
    ++ns;
    a0 = a1;
  }
  return ns;
}

// featureExtraction.cpp:108-177 / featureAssociation.cpp:807-876:
// calculateSmoothness + markOccludedPoints over (range, column) lists.
// picked = 1 for entries the reference never initialises (< 5, >= n - 5).
void smooth_occlude(const float* prange, const int32_t* col_ind, int64_t n, float* curvature,
                    std::vector<int>& picked, std::vector<float>& sval) {
  picked.assign(n, 1);
  sval.assign(n, 0.0f);
  for (int64_t i = 0; i < n; ++i) curvature[i] = 0.0f;
  for (int64_t i = 5; i < n - 5; ++i) {
    const float* r = prange;
    const float diffRange = r[i - 5] + r[i - 4] + r[i - 3] + r[i - 2] + r[i - 1] - r[i] * 10 +
                            r[i + 1] + r[i + 2] + r[i + 3] + r[i + 4] + r[i + 5];
    curvature[i] = diffRange * diffRange;
    picked[i] = 0;
    sval[i] = curvature[i];
  }
  for (int64_t i = 5; i < n - 6; ++i) {
    const float depth1 = prange[i], depth2 = prange[i + 1];
    const int columnDiff = std::abs(int(col_ind[i + 1] - col_ind[i]));
    if (columnDiff < 10) {
      if (depth1 - depth2 > 0.3) {
        for (int k = 0; k <= 5; ++k) picked[i - k] = 1;
      } else if (depth2 - depth1 > 0.3) {
        for (int k = 1; k <= 6; ++k) picked[i + k] = 1;
      }
    }
    const float diff1 = std::abs(float(prange[i - 1] - prange[i]));
    const float diff2 = std::abs(float(prange[i + 1] - prange[i]));
    if (diff1 > 0.02 * prange[i] && diff2 > 0.02 * prange[i]) picked[i] = 1;
  }
}

}  // namespace

extern "C" {

// ---------------------------------------------------------------- LIO-SAM
// projectPointCloud (imageProjection.cpp:610-650) + deskewPoint (:565-604)
// + cloudExtraction (:656-678).
// in: n points SoA (x, y, z, intensity f32, ring u16, time f32 s relative to
//     timeScanCur); deskew table imu_time/rot_xyz[n_imu] (n_imu =
//     imuPointerCur + 1, imageProjection.cpp:345-392), deskew != 0 iff
//     deskewFlag == 1 && imuAvailable.
// out: range_mat[N_SCAN*H] (FLT_MAX = empty), cell_owner[N_SCAN*H] (input
//     index or -1), start/end ring index[N_SCAN], col_ind/prange[n_ext],
//     ext_xyzi[n_ext*4]; returns n_ext.
int64_t orc_lio_project(int n_scan, int horizon, int downsample_rate, float min_range,
                        float max_range, const float* x, const float* y, const float* z,
                        const float* intensity, const uint16_t* ring, const float* time, int64_t n,
                        const double* imu_time, const double* rot_x, const double* rot_y,
                        const double* rot_z, int n_imu, double time_scan_cur, int deskew,
                        float* range_mat, int32_t* cell_owner, int32_t* start_ring,
                        int32_t* end_ring, int32_t* col_ind, float* prange, float* ext_xyzi) {
  const int64_t cells = (int64_t)n_scan * horizon;
  std::vector<float> full((size_t)cells * 4, 0.0f);
  for (int64_t c = 0; c < cells; ++c) {
    range_mat[c] = FLT_MAX;
    cell_owner[c] = -1;
  }
  const float ang_res_x = 360.0 / float(horizon);
  const int imuPointerCur = n_imu - 1;
  bool first = true;
  Aff startInv{};
  for (int64_t i = 0; i < n; ++i) {
    const float px = x[i], py = y[i], pz = z[i];
    const float range = std::sqrt(px * px + py * py + pz * pz);  // utility.h:382-384
    if (range < min_range || range > max_range) continue;
    const int row = ring[i];
    if (row < 0 || row >= n_scan) continue;
    if (row % downsample_rate != 0) continue;
    const float horizonAngle = fatan2(px, py) * 180 / M_PI;
    int col = -std::round((horizonAngle - 90.0) / ang_res_x) + horizon / 2;
    if (col >= horizon) col -= horizon;
    if (col < 0 || col >= horizon) continue;
    const int64_t c = col + (int64_t)row * horizon;
    if (range_mat[c] != FLT_MAX) continue;
    float ox = px, oy = py, oz = pz;
    if (deskew && imuPointerCur > 0) {
      const double pointTime = time_scan_cur + time[i];
      float rx, ry, rz;
      find_rotation(pointTime, imu_time, rot_x, rot_y, rot_z, imuPointerCur, &rx, &ry, &rz);
      if (first) {
        startInv = inverse(get_transformation(0, 0, 0, rx, ry, rz));
        first = false;
      }
      const Aff bt = compose(startInv, get_transformation(0, 0, 0, rx, ry, rz));
      ox = bt.m[0][0] * px + bt.m[0][1] * py + bt.m[0][2] * pz + bt.m[0][3];
      oy = bt.m[1][0] * px + bt.m[1][1] * py + bt.m[1][2] * pz + bt.m[1][3];
      oz = bt.m[2][0] * px + bt.m[2][1] * py + bt.m[2][2] * pz + bt.m[2][3];
    }
    range_mat[c] = range;
    cell_owner[c] = (int32_t)i;
    full[c * 4 + 0] = ox;
    full[c * 4 + 1] = oy;
    full[c * 4 + 2] = oz;
    full[c * 4 + 3] = intensity[i];
  }
  int64_t count = 0;
  for (int r = 0; r < n_scan; ++r) {
    start_ring[r] = (int32_t)(count - 1 + 5);
    for (int j = 0; j < horizon; ++j) {
      const int64_t c = j + (int64_t)r * horizon;
      if (range_mat[c] != FLT_MAX) {
        col_ind[count] = j;
        prange[count] = range_mat[c];
        std::memcpy(ext_xyzi + count * 4, &full[c * 4], 16);
        ++count;
      }
    }
    end_ring[r] = (int32_t)(count - 1 - 5);
  }
  return count;
}

// featureExtraction.cpp:108-131 calculateSmoothness, :137-177
// markOccludedPoints, :183-296 extractFeatures (+ per-ring pcl::VoxelGrid,
// PCL VoxelGrid::applyFilter with downsample_all_data_ / CentroidPoint).
// out: curvature[n], picked0[n] (after markOccludedPoints), label[n] (final),
//      corner_xyzi / surface_xyzi (capacity n); counts via n_corner/n_surface.
// std_ties = 0: ties of the sector sort by point index (the device's order);
// 1: the reference's own call, std::sort over {float value; size_t ind}
// elements with by_value (value only, featureExtraction.cpp:16-20, 201-202),
// i.e. libstdc++ introsort's order for equal values.  n_tied (optional):
// keys that share their value with another key of the same sector sort.
int orc_lio_features_ex(int n_scan, float edge_threshold, float surf_threshold, float leaf,
                        const int32_t* start_ring, const int32_t* end_ring, const int32_t* col_ind,
                        const float* prange, const float* ext_xyzi, int64_t n, float* curvature,
                        uint8_t* picked0, int32_t* label, float* corner_xyzi, int64_t* n_corner,
                        float* surface_xyzi, int64_t* n_surface, int std_ties, int64_t* n_tied) {
  std::vector<float> sval;
  std::vector<int> picked;
  smooth_occlude(prange, col_ind, n, curvature, picked, sval);
  std::vector<int64_t> sind(n);
  for (int64_t i = 0; i < n; ++i) sind[i] = i;
  std::vector<int> lab(n, 0);
  for (int64_t i = 0; i < n; ++i) picked0[i] = (uint8_t)picked[i];

  auto suppress = [&](int64_t ind) {
    picked[ind] = 1;
    for (int l = 1; l <= 5; l++) {
      const int columnDiff = std::abs(int(col_ind[ind + l] - col_ind[ind + l - 1]));
      if (columnDiff > 10) break;
      picked[ind + l] = 1;
    }
    for (int l = -1; l >= -5; l--) {
      const int columnDiff = std::abs(int(col_ind[ind + l] - col_ind[ind + l + 1]));
      if (columnDiff > 10) break;
      picked[ind + l] = 1;
    }
  };
  int64_t nc = 0, ns = 0;
  std::vector<int64_t> scan;  // surfaceCloudScan (positions)
  std::vector<int64_t> order;
  for (int i = 0; i < n_scan; i++) {
    scan.clear();
    for (int j = 0; j < 6; j++) {
      const int sp = (start_ring[i] * (6 - j) + end_ring[i] * j) / 6;
      const int ep = (start_ring[i] * (5 - j) + end_ring[i] * (j + 1)) / 6 - 1;
      if (sp >= ep) continue;
      if (std_ties) {
        // the reference's element type and comparator, sorted in place
        struct smoothness_t {
          float value;
          size_t ind;
        };
        std::vector<smoothness_t> cs(ep - sp);
        for (int k = sp; k < ep; ++k) cs[k - sp] = smoothness_t{sval[k], (size_t)sind[k]};
        std::sort(cs.begin(), cs.end(),
                  [](const smoothness_t& a, const smoothness_t& b) { return a.value < b.value; });
        for (int k = sp; k < ep; ++k) {
          sval[k] = cs[k - sp].value;
          sind[k] = (int64_t)cs[k - sp].ind;
        }
      } else {
        // std::sort(begin + sp, begin + ep, by_value), ties by index
        order.resize(ep - sp);
        for (int k = sp; k < ep; ++k) order[k - sp] = k;
        std::sort(order.begin(), order.end(), [&](int64_t a, int64_t b) {
          if (sval[a] != sval[b]) return sval[a] < sval[b];
          return sind[a] < sind[b];
        });
        std::vector<float> v2(ep - sp);
        std::vector<int64_t> i2(ep - sp);
        for (int k = sp; k < ep; ++k) {
          v2[k - sp] = sval[order[k - sp]];
          i2[k - sp] = sind[order[k - sp]];
        }
        for (int k = sp; k < ep; ++k) {
          sval[k] = v2[k - sp];
          sind[k] = i2[k - sp];
        }
      }
      if (n_tied)
        for (int k = sp; k < ep; ++k)
          *n_tied += (k > sp && sval[k] == sval[k - 1]) || (k + 1 < ep && sval[k] == sval[k + 1]);
      int largestPickedNum = 0;
      for (int k = ep; k >= sp; k--) {
        const int64_t ind = sind[k];
        if (picked[ind] == 0 && curvature[ind] > edge_threshold) {
          largestPickedNum++;
          if (largestPickedNum <= 20) {
            lab[ind] = 1;
            std::memcpy(corner_xyzi + nc * 4, ext_xyzi + ind * 4, 16);
            ++nc;
          } else {
            break;
          }
          suppress(ind);
        }
      }
      for (int k = sp; k <= ep; k++) {
        const int64_t ind = sind[k];
        if (picked[ind] == 0 && curvature[ind] < surf_threshold) {
          lab[ind] = -1;
          suppress(ind);
        }
      }
      for (int k = sp; k <= ep; k++)
        if (lab[k] <= 0) scan.push_back(k);
    }
    ns += voxel_grid(ext_xyzi, scan, leaf, surface_xyzi + ns * 4);
  }
  for (int64_t i = 0; i < n; ++i) label[i] = lab[i];
  *n_corner = nc;
  *n_surface = ns;
  return 0;
}

int orc_lio_features(int n_scan, float edge_threshold, float surf_threshold, float leaf,
                     const int32_t* start_ring, const int32_t* end_ring, const int32_t* col_ind,
                     const float* prange, const float* ext_xyzi, int64_t n, float* curvature,
                     uint8_t* picked0, int32_t* label, float* corner_xyzi, int64_t* n_corner,
                     float* surface_xyzi, int64_t* n_surface) {
  return orc_lio_features_ex(n_scan, edge_threshold, surf_threshold, leaf, start_ring, end_ring, col_ind,
                             prange, ext_xyzi, n, curvature, picked0, label, corner_xyzi, n_corner,
                             surface_xyzi, n_surface, 0, nullptr);
}

}  // extern "C"

// ---------------------------------------------------------------- LeGO-LOAM
// Parameters of LeGO-LOAM/include/utility.h:20-49 (VLP-16 defaults) and
// featureAssociation.cpp:222 (less-flat VoxelGrid leaf 0.2).
struct orc_lego_params {
  int32_t n_scan, horizon, ground_scan_ind, seg_valid_point, seg_valid_line;
  float ang_res_x, ang_res_y, ang_bottom, sensor_mount_angle, segment_theta;
  float edge_thr, surf_thr, leaf, scan_period;
};

namespace {
inline bool row_of(const orc_lego_params* P, float x, float y, float z, int64_t& row) {
  // verticalAngle = atan2(z, sqrt(x^2 + y^2)) * 180 / M_PI; rowIdn is a
  // size_t: the float quotient truncates toward zero, so (-1, 0) -> 0 and
  // anything <= -1 (or NaN) wraps out of range (imageProjection.cpp:177-182)
  const float va = (float)((double)(fatan2(z, std::sqrt(x * x + y * y)) * 180.0f) / M_PI);
  const float q = (va + P->ang_bottom) / P->ang_res_y;
  if (!(q > -1.0f) || !(q < (float)P->n_scan)) return false;
  row = (int64_t)q;
  return row < P->n_scan;
}
inline bool col_of(const orc_lego_params* P, float x, float y, int64_t& col) {
  const float ha = (float)((double)(fatan2(x, y) * 180.0f) / M_PI);
  int64_t c = (int64_t)(-std::round(((double)ha - 90.0) / (double)P->ang_res_x) + P->horizon / 2);
  if (c >= P->horizon) c -= P->horizon;
  if (c < 0 || c >= P->horizon) return false;
  col = c;
  return true;
}
}  // namespace

extern "C" {

// findStartEndAngle + projectPointCloud + groundRemoval + cloudSegmentation
// (LeGO-LOAM/src/imageProjection.cpp:160-330, labelComponents :332-393):
// the last point wins a cell; ground by the inter-ring pitch (sequential per
// column); BFS components in row-major seed order, feasible if >= 30 points or
// >= seg_valid_point points on >= seg_valid_line rings (labelCount order),
// else 999999; the segmented cloud keeps every 5th ground column away from the
// seam.  Returns the segmented cloud size.
int64_t orc_lego_project(const orc_lego_params* P, const float* x, const float* y, const float* z,
                         int64_t n, float* orient /* start, end, diff */, float* range_mat,
                         int32_t* cell_point, int8_t* ground, int32_t* label, int32_t* start_ring,
                         int32_t* end_ring, uint8_t* ground_flag, int32_t* col_ind, float* seg_range,
                         float* seg_xyzi, float* outlier_xyzi, int64_t* n_outlier) {
  const int N = P->n_scan, H = P->horizon;
  const int64_t cells = (int64_t)N * H;
  // findStartEndAngle (:160-175)
  if (n >= 2) {
    const float so = -fatan2(y[0], x[0]);
    float eo = (float)(-(double)fatan2(y[n - 1], x[n - 2]) + 2 * M_PI);
    if (eo - so > 3 * M_PI)
      eo = (float)((double)eo - 2 * M_PI);
    else if (eo - so < M_PI)
      eo = (float)((double)eo + 2 * M_PI);
    orient[0] = so;
    orient[1] = eo;
    orient[2] = eo - so;
  } else {
    orient[0] = orient[1] = orient[2] = 0.0f;
  }
  std::vector<float> full((size_t)cells * 4, 0.0f);
  for (int64_t c = 0; c < cells; ++c) {
    range_mat[c] = FLT_MAX;
    cell_point[c] = -1;
    ground[c] = 0;
    label[c] = 0;
  }
  for (int64_t i = 0; i < n; ++i) {
    const float px = x[i], py = y[i], pz = z[i];
    int64_t row, col;
    if (!row_of(P, px, py, pz, row)) continue;
    if (!col_of(P, px, py, col)) continue;
    const float range = std::sqrt(px * px + py * py + pz * pz);
    const int64_t c = col + row * H;
    range_mat[c] = range;
    cell_point[c] = (int32_t)i;
    full[c * 4 + 0] = px;
    full[c * 4 + 1] = py;
    full[c * 4 + 2] = pz;
    full[c * 4 + 3] = (float)((double)(float)row + (double)(float)col / 10000.0);
  }
  // groundRemoval (:216-262)
  for (int j = 0; j < H; ++j)
    for (int i = 0; i < P->ground_scan_ind; ++i) {
      const int64_t lo = j + (int64_t)i * H, up = j + (int64_t)(i + 1) * H;
      if (cell_point[lo] < 0 || cell_point[up] < 0) {
        ground[lo] = -1;
        continue;
      }
      const float dx = full[up * 4] - full[lo * 4];
      const float dy = full[up * 4 + 1] - full[lo * 4 + 1];
      const float dz = full[up * 4 + 2] - full[lo * 4 + 2];
      const float angle = (float)((double)(fatan2(dz, std::sqrt(dx * dx + dy * dy)) * 180.0f) / M_PI);
      if (std::abs(angle - P->sensor_mount_angle) <= 10) {
        ground[lo] = 1;
        ground[up] = 1;
      }
    }
  for (int64_t c = 0; c < cells; ++c)
    if (ground[c] == 1 || range_mat[c] == FLT_MAX) label[c] = -1;
  // cloudSegmentation / labelComponents (:268-393)
  const float alphaX = (float)((double)P->ang_res_x / 180.0 * M_PI);
  const float alphaY = (float)((double)P->ang_res_y / 180.0 * M_PI);
  const float sX = fsin(alphaX), cX = fcos(alphaX), sY = fsin(alphaY), cY = fcos(alphaY);
  const int nb[4][2] = {{-1, 0}, {0, 1}, {0, -1}, {1, 0}};
  int labelCount = 1;
  std::vector<int> qx(cells), qy(cells), px_(cells), py_(cells);
  std::vector<char> line(N);
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < H; ++j) {
      if (label[j + (int64_t)i * H] != 0) continue;
      std::fill(line.begin(), line.end(), 0);
      int qs = 0, qe = 1, ap = 1;
      qx[0] = i;
      qy[0] = j;
      px_[0] = i;
      py_[0] = j;
      while (qs < qe) {
        const int fx = qx[qs], fy = qy[qs];
        ++qs;
        label[fy + (int64_t)fx * H] = labelCount;
        for (int k = 0; k < 4; ++k) {
          const int tx = fx + nb[k][0];
          int ty = fy + nb[k][1];
          if (tx < 0 || tx >= N) continue;
          if (ty < 0) ty = H - 1;
          if (ty >= H) ty = 0;
          if (label[ty + (int64_t)tx * H] != 0) continue;
          const float ra = range_mat[fy + (int64_t)fx * H], rb = range_mat[ty + (int64_t)tx * H];
          const float d1 = std::max(ra, rb), d2 = std::min(ra, rb);
          const bool horiz = nb[k][0] == 0;
          const float angle = fatan2(d2 * (horiz ? sX : sY), (d1 - d2 * (horiz ? cX : cY)));
          if (angle > P->segment_theta) {
            qx[qe] = tx;
            qy[qe] = ty;
            ++qe;
            label[ty + (int64_t)tx * H] = labelCount;
            line[tx] = 1;
            px_[ap] = tx;
            py_[ap] = ty;
            ++ap;
          }
        }
      }
      bool feasible = false;
      if (ap >= 30)
        feasible = true;
      else if (ap >= P->seg_valid_point) {
        int lc = 0;
        for (int r = 0; r < N; ++r) lc += line[r] ? 1 : 0;
        if (lc >= P->seg_valid_line) feasible = true;
      }
      if (feasible)
        ++labelCount;
      else
        for (int q = 0; q < ap; ++q) label[py_[q] + (int64_t)px_[q] * H] = 999999;
    }
  int64_t sz = 0, no = 0;
  for (int i = 0; i < N; ++i) {
    start_ring[i] = (int32_t)(sz - 1 + 5);
    for (int j = 0; j < H; ++j) {
      const int64_t c = j + (int64_t)i * H;
      if (label[c] > 0 || ground[c] == 1) {
        if (label[c] == 999999) {
          if (i > P->ground_scan_ind && j % 5 == 0) {
            std::memcpy(outlier_xyzi + no * 4, &full[c * 4], 16);
            ++no;
          }
          continue;
        }
        if (ground[c] == 1)
          if (j % 5 != 0 && j > 5 && j < H - 5) continue;
        ground_flag[sz] = ground[c] == 1;
        col_ind[sz] = j;
        seg_range[sz] = range_mat[c];
        std::memcpy(seg_xyzi + sz * 4, &full[c * 4], 16);
        ++sz;
      }
    }
    end_ring[i] = (int32_t)(sz - 1 - 5);
  }
  *n_outlier = no;
  return sz;
}

// IMU state of FeatureAssociation (featureAssociation.cpp:86-132) consumed by
// adjustDistortion: the 200-entry ring buffer filled by imuHandler /
// AccumulateIMUShiftAndRotation (:430-588, host side), pointers and the
// angular rotation of the previous scan.
struct orc_lego_imu {
  const double* time;
  const float *roll, *pitch, *yaw, *velo_x, *velo_y, *velo_z, *shift_x, *shift_y, *shift_z;
  const float *ang_x, *ang_y, *ang_z;
  int32_t pointer_last, pointer_last_iteration, que_len;
  double time_scan_cur;
  float ang_last[3];
};
struct orc_lego_imu_out {
  float rpy_start[3], rpy_cur[3], velo_from_start[3], angular_from_start[3], ang_last[3];
  int32_t pointer_last_iteration;
};

// adjustDistortion (:617-805) + calculateSmoothness + markOccludedPoints +
// extractFeatures (:807-1007).  seg_xyzi is the segmented cloud of
// orc_lego_project; deskewed (n x 4) receives the adjusted points (LOAM frame
// x = y, y = z, z = x; intensity = ring + scanPeriod * relTime).  Outputs:
// cornerPointsSharp, cornerPointsLessSharp, surfPointsFlat,
// surfPointsLessFlat (per-ring VoxelGrid leaf).
int orc_lego_features(const orc_lego_params* P, const float* orient, const int32_t* start_ring,
                      const int32_t* end_ring, const uint8_t* ground_flag, const int32_t* col_ind,
                      const float* seg_range, const float* seg_xyzi, int64_t n,
                      const orc_lego_imu* imu, orc_lego_imu_out* io, float* deskewed,
                      float* curvature, uint8_t* picked0, int32_t* label, float* sharp,
                      int64_t* n_sharp, float* less_sharp, int64_t* n_less_sharp, float* flat,
                      int64_t* n_flat, float* less_flat, int64_t* n_less_flat) {
  const float so = orient[0], eo = orient[1], od = orient[2];
  const float scanPeriod = P->scan_period;
  bool halfPassed = false;
  float rs = 0, ps = 0, ys = 0, cRs = 0, cPs = 0, cYs = 0, sRs = 0, sPs = 0, sYs = 0;
  float vxs = 0, vys = 0, vzs = 0;
  if (imu) {
    for (int a = 0; a < 3; ++a) io->ang_last[a] = imu->ang_last[a];
    io->pointer_last_iteration = imu->pointer_last_iteration;
  }
  for (int64_t i = 0; i < n; i++) {
    float px = seg_xyzi[i * 4 + 1], py = seg_xyzi[i * 4 + 2], pz = seg_xyzi[i * 4 + 0];
    float ori = -fatan2(px, pz);
    if (!halfPassed) {
      if (ori < so - M_PI / 2)
        ori = (float)((double)ori + 2 * M_PI);
      else if (ori > so + M_PI * 3 / 2)
        ori = (float)((double)ori - 2 * M_PI);
      if (ori - so > M_PI) halfPassed = true;
    } else {
      ori = (float)((double)ori + 2 * M_PI);
      if (ori < eo - M_PI * 3 / 2)
        ori = (float)((double)ori + 2 * M_PI);
      else if (ori > eo + M_PI / 2)
        ori = (float)((double)ori - 2 * M_PI);
    }
    const float relTime = (ori - so) / od;
    const float inten = int(seg_xyzi[i * 4 + 3]) + scanPeriod * relTime;
    if (imu && imu->pointer_last >= 0) {
      const int Q = imu->que_len;
      const float pointTime = relTime * scanPeriod;
      const double tq = imu->time_scan_cur + pointTime;
      int f = imu->pointer_last_iteration;
      while (f != imu->pointer_last) {
        if (tq < imu->time[f]) break;
        f = (f + 1) % Q;
      }
      float rc, pc, yc, vxc, vyc, vzc;
      const bool after = tq > imu->time[f];
      const int b = (f + Q - 1) % Q;
      float rf = 0, rb = 0;
      if (after) {
        rc = imu->roll[f];
        pc = imu->pitch[f];
        yc = imu->yaw[f];
        vxc = imu->velo_x[f];
        vyc = imu->velo_y[f];
        vzc = imu->velo_z[f];
      } else {
        rf = (float)((tq - imu->time[b]) / (imu->time[f] - imu->time[b]));
        rb = (float)((imu->time[f] - tq) / (imu->time[f] - imu->time[b]));
        rc = imu->roll[f] * rf + imu->roll[b] * rb;
        pc = imu->pitch[f] * rf + imu->pitch[b] * rb;
        if (imu->yaw[f] - imu->yaw[b] > M_PI)
          yc = (float)(imu->yaw[f] * rf + ((double)imu->yaw[b] + 2 * M_PI) * rb);
        else if (imu->yaw[f] - imu->yaw[b] < -M_PI)
          yc = (float)(imu->yaw[f] * rf + ((double)imu->yaw[b] - 2 * M_PI) * rb);
        else
          yc = imu->yaw[f] * rf + imu->yaw[b] * rb;
        vxc = imu->velo_x[f] * rf + imu->velo_x[b] * rb;
        vyc = imu->velo_y[f] * rf + imu->velo_y[b] * rb;
        vzc = imu->velo_z[f] * rf + imu->velo_z[b] * rb;
      }
      io->rpy_cur[0] = rc;
      io->rpy_cur[1] = pc;
      io->rpy_cur[2] = yc;
      if (i == 0) {
        rs = rc;
        ps = pc;
        ys = yc;
        vxs = vxc;
        vys = vyc;
        vzs = vzc;
        float ax, ay, az;
        if (after) {
          ax = imu->ang_x[f];
          ay = imu->ang_y[f];
          az = imu->ang_z[f];
        } else {
          ax = imu->ang_x[f] * rf + imu->ang_x[b] * rb;
          ay = imu->ang_y[f] * rf + imu->ang_y[b] * rb;
          az = imu->ang_z[f] * rf + imu->ang_z[b] * rb;
        }
        io->angular_from_start[0] = ax - io->ang_last[0];
        io->angular_from_start[1] = ay - io->ang_last[1];
        io->angular_from_start[2] = az - io->ang_last[2];
        io->ang_last[0] = ax;
        io->ang_last[1] = ay;
        io->ang_last[2] = az;
        cRs = fcos(rs);
        cPs = fcos(ps);
        cYs = fcos(ys);
        sRs = fsin(rs);
        sPs = fsin(ps);
        sYs = fsin(ys);
      } else {
        // VeloToStartIMU (:392-427)
        {
          const float vx = vxc - vxs, vy = vyc - vys, vz = vzc - vzs;
          const float x1 = cYs * vx - sYs * vz, y1 = vy, z1 = sYs * vx + cYs * vz;
          const float x2 = x1, y2 = cPs * y1 + sPs * z1, z2 = -sPs * y1 + cPs * z1;
          io->velo_from_start[0] = cRs * x2 + sRs * y2;
          io->velo_from_start[1] = -sRs * x2 + cRs * y2;
          io->velo_from_start[2] = z2;
        }
        // TransformToStartIMU (:429-458); imuShiftFromStartCur stays 0
        // (ShiftToStartIMU is never called in this fork)
        const float x1 = fcos(rc) * px - fsin(rc) * py;
        const float y1 = fsin(rc) * px + fcos(rc) * py;
        const float z1 = pz;
        const float x2 = x1;
        const float y2 = fcos(pc) * y1 - fsin(pc) * z1;
        const float z2 = fsin(pc) * y1 + fcos(pc) * z1;
        const float x3 = fcos(yc) * x2 + fsin(yc) * z2;
        const float y3 = y2;
        const float z3 = -fsin(yc) * x2 + fcos(yc) * z2;
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
    deskewed[i * 4 + 0] = px;
    deskewed[i * 4 + 1] = py;
    deskewed[i * 4 + 2] = pz;
    deskewed[i * 4 + 3] = inten;
  }
  if (imu && imu->pointer_last >= 0 && n > 0) {
    io->rpy_start[0] = rs;
    io->rpy_start[1] = ps;
    io->rpy_start[2] = ys;
  }
  if (imu) io->pointer_last_iteration = imu->pointer_last;  // :804, unconditional
  // calculateSmoothness + markOccludedPoints
  std::vector<float> sval;
  std::vector<int> picked;
  smooth_occlude(seg_range, col_ind, n, curvature, picked, sval);
  for (int64_t i = 0; i < n; ++i) picked0[i] = (uint8_t)picked[i];
  std::vector<int64_t> sind(n);
  for (int64_t i = 0; i < n; ++i) sind[i] = i;
  std::vector<int> lab(n, 0);
  auto suppress = [&](int64_t ind) {
    picked[ind] = 1;
    for (int l = 1; l <= 5; l++) {
      if (std::abs(int(col_ind[ind + l] - col_ind[ind + l - 1])) > 10) break;
      picked[ind + l] = 1;
    }
    for (int l = -1; l >= -5; l--) {
      if (std::abs(int(col_ind[ind + l] - col_ind[ind + l + 1])) > 10) break;
      picked[ind + l] = 1;
    }
  };
  int64_t ns = 0, nls = 0, nf = 0, nlf = 0;
  std::vector<int64_t> scan, order;
  for (int i = 0; i < P->n_scan; i++) {
    scan.clear();
    for (int j = 0; j < 6; j++) {
      const int sp = (start_ring[i] * (6 - j) + end_ring[i] * j) / 6;
      const int ep = (start_ring[i] * (5 - j) + end_ring[i] * (j + 1)) / 6 - 1;
      if (sp >= ep) continue;
      order.resize(ep - sp);
      for (int k = sp; k < ep; ++k) order[k - sp] = k;
      std::sort(order.begin(), order.end(), [&](int64_t a, int64_t b) {
        if (sval[a] != sval[b]) return sval[a] < sval[b];
        return sind[a] < sind[b];
      });
      std::vector<float> v2(ep - sp);
      std::vector<int64_t> i2(ep - sp);
      for (int k = sp; k < ep; ++k) {
        v2[k - sp] = sval[order[k - sp]];
        i2[k - sp] = sind[order[k - sp]];
      }
      for (int k = sp; k < ep; ++k) {
        sval[k] = v2[k - sp];
        sind[k] = i2[k - sp];
      }
      int largestPickedNum = 0;
      for (int k = ep; k >= sp; k--) {
        const int64_t ind = sind[k];
        if (picked[ind] == 0 && curvature[ind] > P->edge_thr && !ground_flag[ind]) {
          largestPickedNum++;
          if (largestPickedNum <= 2) {
            lab[ind] = 2;
            std::memcpy(sharp + (ns++) * 4, deskewed + ind * 4, 16);
            std::memcpy(less_sharp + (nls++) * 4, deskewed + ind * 4, 16);
          } else if (largestPickedNum <= 20) {
            lab[ind] = 1;
            std::memcpy(less_sharp + (nls++) * 4, deskewed + ind * 4, 16);
          } else {
            break;
          }
          suppress(ind);
        }
      }
      int smallestPickedNum = 0;
      for (int k = sp; k <= ep; k++) {
        const int64_t ind = sind[k];
        if (picked[ind] == 0 && curvature[ind] < P->surf_thr && ground_flag[ind]) {
          lab[ind] = -1;
          std::memcpy(flat + (nf++) * 4, deskewed + ind * 4, 16);
          smallestPickedNum++;
          if (smallestPickedNum >= 4) break;
          suppress(ind);
        }
      }
      for (int k = sp; k <= ep; k++)
        if (lab[k] <= 0) scan.push_back(k);
    }
    nlf += voxel_grid(deskewed, scan, P->leaf, less_flat + nlf * 4);
  }
  for (int64_t i = 0; i < n; ++i) label[i] = lab[i];
  *n_sharp = ns;
  *n_less_sharp = nls;
  *n_flat = nf;
  *n_less_flat = nlf;
  return 0;
}

}  // extern "C"

// downSizeFilterSurf (laserMapping.cpp:683-686, 737-739): pcl::VoxelGrid
// over a cloud's xyz; non-finite points are skipped (PCL with is_dense
// false).  pcl_order = 0: ties of the voxel index sort by point index (the
// device's order); 1: PCL 1.10's std::sort order.  Returns the number of
// centroids written to ox / oy / oz (capacity n).
extern "C" int64_t orc_voxel_grid_xyz(const float* x, const float* y, const float* z, int64_t n, float leaf,
                                      int pcl_order, float* ox, float* oy, float* oz) {
  std::vector<float> xyzi((size_t)n * 4);
  std::vector<int64_t> pos;
  for (int64_t i = 0; i < n; ++i) {
    xyzi[4 * i] = x[i];
    xyzi[4 * i + 1] = y[i];
    xyzi[4 * i + 2] = z[i];
    xyzi[4 * i + 3] = 0.0f;
    if (std::isfinite(x[i]) && std::isfinite(y[i]) && std::isfinite(z[i])) pos.push_back(i);
  }
  std::vector<float> out(pos.size() * 4 + 4);
  const int64_t m = pcl_order ? voxel_grid_pcl_order(xyzi.data(), pos, leaf, out.data())
                              : voxel_grid(xyzi.data(), pos, leaf, out.data());
  for (int64_t k = 0; k < m; ++k) {
    ox[k] = out[4 * k];
    oy[k] = out[4 * k + 1];
    oz[k] = out[4 * k + 2];
  }
  return m;
}
