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
//     are broken by point index;
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
int orc_lio_features(int n_scan, float edge_threshold, float surf_threshold, float leaf,
                     const int32_t* start_ring, const int32_t* end_ring, const int32_t* col_ind,
                     const float* prange, const float* ext_xyzi, int64_t n, float* curvature,
                     uint8_t* picked0, int32_t* label, float* corner_xyzi, int64_t* n_corner,
                     float* surface_xyzi, int64_t* n_surface) {
  std::vector<float> sval(n, 0.0f);
  std::vector<int64_t> sind(n);
  std::vector<int> picked(n, 1);
  std::vector<int> lab(n, 0);
  for (int64_t i = 0; i < n; ++i) {
    curvature[i] = 0.0f;
    sind[i] = i;
  }
  for (int64_t i = 5; i < n - 5; ++i) {
    const float* r = prange;
    const float diffRange = r[i - 5] + r[i - 4] + r[i - 3] + r[i - 2] + r[i - 1] - r[i] * 10 +
                            r[i + 1] + r[i + 2] + r[i + 3] + r[i + 4] + r[i + 5];
    curvature[i] = diffRange * diffRange;
    picked[i] = 0;
    lab[i] = 0;
    sval[i] = curvature[i];
    sind[i] = i;
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
    // pcl::VoxelGrid (leaf) on surfaceCloudScan
    if (scan.empty()) continue;
    const float inv = 1.0f / leaf;
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int64_t p : scan)
      for (int a = 0; a < 3; ++a) {
        mn[a] = std::min(mn[a], ext_xyzi[p * 4 + a]);
        mx[a] = std::max(mx[a], ext_xyzi[p * 4 + a]);
      }
    const int64_t dx = (int64_t)((mx[0] - mn[0]) * inv) + 1;
    const int64_t dy = (int64_t)((mx[1] - mn[1]) * inv) + 1;
    const int64_t dz = (int64_t)((mx[2] - mn[2]) * inv) + 1;
    if (dx * dy * dz > (int64_t)INT32_MAX) {  // PCL: output = input
      for (int64_t p : scan) {
        std::memcpy(surface_xyzi + ns * 4, ext_xyzi + p * 4, 16);
        ++ns;
      }
      continue;
    }
    int minb[3], maxb[3], divb[3];
    for (int a = 0; a < 3; ++a) {
      minb[a] = (int)std::floor(mn[a] * inv);
      maxb[a] = (int)std::floor(mx[a] * inv);
      divb[a] = maxb[a] - minb[a] + 1;
    }
    const int mul[3] = {1, divb[0], divb[0] * divb[1]};
    std::vector<std::pair<uint32_t, int64_t>> iv;  // (voxel idx, position in scan)
    iv.reserve(scan.size());
    for (size_t q = 0; q < scan.size(); ++q) {
      const float* pp = ext_xyzi + scan[q] * 4;
      int ijk[3];
      for (int a = 0; a < 3; ++a) ijk[a] = (int)(std::floor(pp[a] * inv) - (float)minb[a]);
      const int idx = ijk[0] * mul[0] + ijk[1] * mul[1] + ijk[2] * mul[2];
      iv.emplace_back((uint32_t)idx, (int64_t)q);
    }
    std::sort(iv.begin(), iv.end());
    size_t a0 = 0;
    while (a0 < iv.size()) {
      size_t a1 = a0 + 1;
      while (a1 < iv.size() && iv[a1].first == iv[a0].first) ++a1;
      float s[4] = {0, 0, 0, 0};
      for (size_t q = a0; q < a1; ++q) {
        const float* pp = ext_xyzi + scan[iv[q].second] * 4;
        for (int c = 0; c < 4; ++c) s[c] += pp[c];
      }
      const float cnt = (float)(a1 - a0);
      for (int c = 0; c < 4; ++c) surface_xyzi[ns * 4 + c] = s[c] / cnt;
      ++ns;
      a0 = a1;
    }
  }
  for (int64_t i = 0; i < n; ++i) label[i] = lab[i];
  *n_corner = nc;
  *n_surface = ns;
  return 0;
}

}  // extern "C"
