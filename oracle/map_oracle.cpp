// CPU oracle of S-FAST_LIO's map maintenance (TEST INFRASTRUCTURE ONLY: the
// product never links, loads or calls this; tests/ use it as the checker).
//
// Restates, as operations on the SET of valid map points:
//   pointBodyToWorld         src/S-FAST_LIO/src/laserMapping.cpp:276-287
//   lasermap_fov_segment     laserMapping.cpp:309-365
//   map_incremental          laserMapping.cpp:382-433
//   KD_TREE::Add_Points      include/ikd-Tree/ikd_Tree.cpp:419-512
//     (downsample: box = voxel of downsample_size around the point, the
//      point nearest the box centre survives; same_point :1533-1536 with
//      EPSS 1e-6 ikd_Tree.h:13; calc_dist :1539-1544)
//   KD_TREE::Delete_Point_Boxes ikd_Tree.cpp:559-579 with the half-open box
//     predicate of Search_by_range / Delete_by_range (vmin <= p < vmax)
// ikd-Tree keeps no point ids.  This framework's Nearest_Points indices are
// ids: uploaded points get 0..n-1, and every Add_Points call gives the new
// points that survive it the next ids in list order.  Where ikd-Tree's
// traversal order would decide (two stored points exactly as near the box
// centre), the lower id wins.  Sequential, one point at a time, exactly as
// the reference loops.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <unordered_map>
#include <vector>

namespace {

struct Pt {
  float x, y, z;
};

struct OrcMap {
  std::vector<Pt> p;
  std::vector<uint32_t> id;
  std::vector<uint8_t> alive;
  uint32_t next_id = 0;
  float hash_edge = 0.5f;  // voxel hash for box searches (any edge works)
  std::unordered_map<uint64_t, std::vector<uint32_t>> hash;  // voxel -> slots

  static uint64_t key(int64_t a, int64_t b, int64_t c) {
    return ((uint64_t)(a & 0x1FFFFF) << 42) | ((uint64_t)(b & 0x1FFFFF) << 21) | (uint64_t)(c & 0x1FFFFF);
  }
  int64_t cell(float v) const { return (int64_t)std::floor((double)v / (double)hash_edge); }
  void index(uint32_t s) {
    hash[key(cell(p[s].x), cell(p[s].y), cell(p[s].z))].push_back(s);
  }
  uint32_t push(const Pt& q, uint32_t i) {
    p.push_back(q);
    id.push_back(i);
    alive.push_back(1);
    const uint32_t s = (uint32_t)(p.size() - 1);
    index(s);
    return s;
  }
  // alive slots inside the half-open box [lo, hi) (ikd_Tree.cpp:1320-1330 predicate)
  void box(const float lo[3], const float hi[3], std::vector<uint32_t>& out) const {
    out.clear();
    const int64_t a0 = cell(lo[0]) - 1, a1 = cell(hi[0]) + 1;
    const int64_t b0 = cell(lo[1]) - 1, b1 = cell(hi[1]) + 1;
    const int64_t c0 = cell(lo[2]) - 1, c1 = cell(hi[2]) + 1;
    for (int64_t a = a0; a <= a1; ++a)
      for (int64_t b = b0; b <= b1; ++b)
        for (int64_t c = c0; c <= c1; ++c) {
          auto it = hash.find(key(a, b, c));
          if (it == hash.end()) continue;
          for (uint32_t s : it->second) {
            if (!alive[s]) continue;
            const Pt& q = p[s];
            if (lo[0] <= q.x && hi[0] > q.x && lo[1] <= q.y && hi[1] > q.y && lo[2] <= q.z && hi[2] > q.z)
              out.push_back(s);
          }
        }
  }
};

inline float calc_dist(const Pt& a, const Pt& b) {  // ikd_Tree.cpp:1539-1544
  return (a.x - b.x) * (a.x - b.x) + (a.y - b.y) * (a.y - b.y) + (a.z - b.z) * (a.z - b.z);
}

inline bool same_point(const Pt& a, const Pt& b) {  // ikd_Tree.cpp:1533-1536
  return std::fabs(a.x - b.x) < 1e-6 && std::fabs(a.y - b.y) < 1e-6 && std::fabs(a.z - b.z) < 1e-6;
}

// Eigen Quaternion::toRotationMatrix (q = w, x, y, z)
void quat_matrix(const double* q, double R[9]) {
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
}

inline void matvec(const double R[9], const double v[3], double o[3]) {
  for (int i = 0; i < 3; ++i) o[i] = (R[3 * i] * v[0] + R[3 * i + 1] * v[1]) + R[3 * i + 2] * v[2];
}

// Add_Points (ikd_Tree.cpp:419-512) on the set; returns tmp_counter
int64_t add_points(OrcMap& m, const std::vector<Pt>& pts, bool downsample, float ds) {
  int64_t counter = 0;
  std::vector<uint32_t> store;
  // new slots whose point is still alive get ids at the end, in list order
  std::vector<uint32_t> new_slots;
  for (const Pt& q : pts) {
    if (!downsample) {
      new_slots.push_back(m.push(q, 0xFFFFFFFFu));
      continue;
    }
    float lo[3], hi[3];
    const float c[3] = {q.x, q.y, q.z};
    for (int a = 0; a < 3; ++a) {
      lo[a] = std::floor(c[a] / ds) * ds;
      hi[a] = lo[a] + ds;
    }
    Pt mid;
    mid.x = (float)(lo[0] + (hi[0] - lo[0]) / 2.0);
    mid.y = (float)(lo[1] + (hi[1] - lo[1]) / 2.0);
    mid.z = (float)(lo[2] + (hi[2] - lo[2]) / 2.0);
    m.box(lo, hi, store);
    // storage order: ascending id; a point added earlier in this call (id
    // not assigned yet: 0xFFFFFFFF) comes last, above every stored id
    std::sort(store.begin(), store.end(), [&](uint32_t a, uint32_t b) { return m.id[a] < m.id[b]; });
    float min_dist = calc_dist(q, mid);
    int64_t win = -1;  // -1: the new point
    for (uint32_t s : store) {
      const float d = calc_dist(m.p[s], mid);
      if (d < min_dist) {  // strict <: the first minimum in storage order
        min_dist = d;
        win = s;
      }
    }
    const Pt wp = win < 0 ? q : m.p[(size_t)win];
    if (store.size() > 1 || same_point(q, wp)) {
      for (uint32_t s : store)
        if ((int64_t)s != win) m.alive[s] = 0;
      if (win < 0) new_slots.push_back(m.push(q, 0xFFFFFFFFu));
      counter++;
    }
  }
  for (uint32_t s : new_slots)
    if (m.alive[s]) m.id[s] = m.next_id++;
  return counter;
}

}  // namespace

extern "C" {

void* orc_map_new(const float* x, const float* y, const float* z, int64_t n, float hash_edge) {
  OrcMap* m = new OrcMap;
  m->hash_edge = hash_edge > 0 ? hash_edge : 0.5f;
  m->p.reserve(n);
  for (int64_t i = 0; i < n; ++i) m->push(Pt{x[i], y[i], z[i]}, (uint32_t)i);
  m->next_id = (uint32_t)n;
  return m;
}

void orc_map_free(void* h) { delete static_cast<OrcMap*>(h); }

int64_t orc_map_size(void* h) {
  const OrcMap& m = *static_cast<OrcMap*>(h);
  int64_t k = 0;
  for (uint8_t a : m.alive) k += a;
  return k;
}

// alive points in ascending id
int64_t orc_map_dump(void* h, float* x, float* y, float* z, uint32_t* ids) {
  const OrcMap& m = *static_cast<OrcMap*>(h);
  std::vector<std::pair<uint32_t, uint32_t>> order;
  for (size_t s = 0; s < m.p.size(); ++s)
    if (m.alive[s]) order.push_back({m.id[s], (uint32_t)s});
  std::sort(order.begin(), order.end());
  for (size_t k = 0; k < order.size(); ++k) {
    const Pt& q = m.p[order[k].second];
    x[k] = q.x;
    y[k] = q.y;
    z[k] = q.z;
    ids[k] = order[k].first;
  }
  return (int64_t)order.size();
}

int64_t orc_map_add(void* h, const float* x, const float* y, const float* z, int64_t n, int downsample,
                    float ds) {
  std::vector<Pt> pts((size_t)n);
  for (int64_t i = 0; i < n; ++i) pts[i] = Pt{x[i], y[i], z[i]};
  return add_points(*static_cast<OrcMap*>(h), pts, downsample != 0, ds);
}

// Delete_Point_Boxes: boxes are n x 6 (min x, y, z, max x, y, z); returns
// the number of points deleted
int64_t orc_map_delete_boxes(void* h, const float* boxes, int64_t nb) {
  OrcMap& m = *static_cast<OrcMap*>(h);
  int64_t k = 0;
  for (int64_t b = 0; b < nb; ++b) {
    const float* lo = boxes + 6 * b;
    const float* hi = lo + 3;
    for (size_t s = 0; s < m.p.size(); ++s) {
      if (!m.alive[s]) continue;
      const Pt& q = m.p[s];
      if (lo[0] <= q.x && hi[0] > q.x && lo[1] <= q.y && hi[1] > q.y && lo[2] <= q.z && hi[2] > q.z) {
        m.alive[s] = 0;
        ++k;
      }
    }
  }
  return k;
}

// pointBodyToWorld (laserMapping.cpp:276-287): rotation matrices from the
// quaternions (Sophus SO3::matrix = Eigen toRotationMatrix), double, to float
void orc_body_to_world_mat(const double* state26, const float* bx, const float* by, const float* bz,
                           int64_t n, float* wx, float* wy, float* wz) {
  double R[9], RL[9];
  quat_matrix(state26 + 3, R);
  quat_matrix(state26 + 7, RL);
  const double* pos = state26;
  const double* tli = state26 + 11;
  for (int64_t i = 0; i < n; ++i) {
    const double pb[3] = {(double)bx[i], (double)by[i], (double)bz[i]};
    double a[3], w[3];
    matvec(RL, pb, a);
    for (int k = 0; k < 3; ++k) a[k] = a[k] + tli[k];
    matvec(R, a, w);
    wx[i] = (float)(w[0] + pos[0]);
    wy[i] = (float)(w[1] + pos[1]);
    wz[i] = (float)(w[2] + pos[2]);
  }
}

// map_incremental (laserMapping.cpp:382-433).  nbr_ids: n x 5 ids of the
// last search's Nearest_Points (-1: none); counts[0] = |PointToAdd|,
// counts[1] = |PointNoNeedDownsample|, counts[2] = Add_Points' counter.
int orc_map_incremental(void* h, const double* state26, const float* bx, const float* by, const float* bz,
                        int64_t n, const int32_t* nbr_ids, double filter_size_map_min, int ekf_inited,
                        float ds, int64_t* counts) {
  OrcMap& m = *static_cast<OrcMap*>(h);
  std::unordered_map<uint32_t, uint32_t> slot_of;
  slot_of.reserve(m.p.size());
  for (size_t s = 0; s < m.p.size(); ++s)
    if (m.alive[s]) slot_of[m.id[s]] = (uint32_t)s;
  std::vector<float> wx(n), wy(n), wz(n);
  orc_body_to_world_mat(state26, bx, by, bz, n, wx.data(), wy.data(), wz.data());
  std::vector<Pt> to_add, no_ds;
  const double fs = filter_size_map_min;
  for (int64_t i = 0; i < n; ++i) {
    const Pt p{wx[i], wy[i], wz[i]};
    std::vector<Pt> near;
    for (int j = 0; j < 5; ++j) {
      const int32_t id = nbr_ids[5 * i + j];
      if (id < 0) break;
      auto it = slot_of.find((uint32_t)id);
      if (it == slot_of.end()) return -1;  // a neighbour id the map does not hold
      near.push_back(m.p[it->second]);
    }
    if (!near.empty() && ekf_inited) {
      bool need_add = true;
      Pt mid;
      mid.x = (float)(std::floor((double)p.x / fs) * fs + 0.5 * fs);
      mid.y = (float)(std::floor((double)p.y / fs) * fs + 0.5 * fs);
      mid.z = (float)(std::floor((double)p.z / fs) * fs + 0.5 * fs);
      const float dist = calc_dist(p, mid);
      if (std::fabs(near[0].x - mid.x) > 0.5 * fs && std::fabs(near[0].y - mid.y) > 0.5 * fs &&
          std::fabs(near[0].z - mid.z) > 0.5 * fs) {
        no_ds.push_back(p);
        continue;
      }
      for (int j = 0; j < 5; ++j) {
        if ((int)near.size() < 5) break;
        if (calc_dist(near[j], mid) < dist) {
          need_add = false;
          break;
        }
      }
      if (need_add) to_add.push_back(p);
    } else {
      to_add.push_back(p);
    }
  }
  counts[0] = (int64_t)to_add.size();
  counts[1] = (int64_t)no_ds.size();
  counts[2] = add_points(m, to_add, true, ds);
  add_points(m, no_ds, false, ds);
  return 0;
}

// lasermap_fov_segment (laserMapping.cpp:309-365) on the local-map box
// (float vertex_min / vertex_max, in/out) at the LiDAR position pos_lid;
// writes up to 3 boxes to remove (6 floats each), returns their number.
int orc_fov_segment(const double* pos_lid, float* box_min, float* box_max, int* initialized, double cube_len,
                    float det_range, float* boxes) {
  const float MOV_THRESHOLD = 1.5f;
  if (!*initialized) {
    for (int i = 0; i < 3; ++i) {
      box_min[i] = (float)(pos_lid[i] - cube_len / 2.0);
      box_max[i] = (float)(pos_lid[i] + cube_len / 2.0);
    }
    *initialized = 1;
    return 0;
  }
  float dist[3][2];
  bool need_move = false;
  for (int i = 0; i < 3; ++i) {
    dist[i][0] = (float)std::fabs(pos_lid[i] - box_min[i]);
    dist[i][1] = (float)std::fabs(pos_lid[i] - box_max[i]);
    if (dist[i][0] <= MOV_THRESHOLD * det_range || dist[i][1] <= MOV_THRESHOLD * det_range) need_move = true;
  }
  if (!need_move) return 0;
  float nmin[3], nmax[3];
  std::memcpy(nmin, box_min, sizeof nmin);
  std::memcpy(nmax, box_max, sizeof nmax);
  const float mov_dist = (float)std::max((cube_len - 2.0 * MOV_THRESHOLD * det_range) * 0.5 * 0.9,
                                         double(det_range * (MOV_THRESHOLD - 1)));
  int nb = 0;
  for (int i = 0; i < 3; ++i) {
    float tmin[3], tmax[3];
    std::memcpy(tmin, box_min, sizeof tmin);
    std::memcpy(tmax, box_max, sizeof tmax);
    if (dist[i][0] <= MOV_THRESHOLD * det_range) {
      nmax[i] -= mov_dist;
      nmin[i] -= mov_dist;
      tmin[i] = box_max[i] - mov_dist;
    } else if (dist[i][1] <= MOV_THRESHOLD * det_range) {
      nmax[i] += mov_dist;
      nmin[i] += mov_dist;
      tmax[i] = box_min[i] + mov_dist;
    } else {
      continue;
    }
    for (int k = 0; k < 3; ++k) {
      boxes[6 * nb + k] = tmin[k];
      boxes[6 * nb + 3 + k] = tmax[k];
    }
    ++nb;
  }
  std::memcpy(box_min, nmin, sizeof nmin);
  std::memcpy(box_max, nmax, sizeof nmax);
  return nb;
}

}  // extern "C"
