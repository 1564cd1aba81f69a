// slio_oracle.cpp — CPU ORACLE (test infrastructure only).
//
// A from-scratch CPU restatement of the reference's hot path, used ONLY by
// tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the
// checker.  The product (agi_lidar_slam_amd/) never links or calls it.
//
// What it restates (all paths relative to /root/reference/src/S-FAST_LIO):
//   * KD_TREE::BuildTree (include/ikd-Tree/ikd_Tree.cpp:597-650, longest-axis
//     split, std::nth_element at mid = (l+r)>>1) and Update's subtree ranges
//     (:1320-1460) for a freshly built static tree;
//   * KD_TREE::Nearest_Search (:370-402) + Search (:960-1101) branch-and-bound
//     with calc_box_dist (:1547-1569), calc_dist (:1539-1544) and the
//     MANUAL_HEAP / PointType_CMP max-heap (ikd_Tree.h:88-168): strict-`<`
//     replacement, tie-break on x within 1e-10, output ascending;
//   * esti_plane (include/common_lib.h:102-134) via a restatement of Eigen's
//     ColPivHouseholderQR solve, sums taken left-to-right;
//   * esekf::h_share_model (include/esekfom.hpp:106-227): body->world with
//     quaternion rotation, kNN gate, plane, residual gate s > 0.9, Jacobian rows;
//   * esekf::update_iterated_dyn_share_modified (:270-346) incl. the 24 x m
//     gain K formed explicitly as the reference does (reference_gain = 1);
//   * Sophus::SO3 @ a621ff exp/log and Eigen quaternion helpers.
//
// PARITY STATUS: the reference cannot be compiled here (ROS, PCL, Eigen and
// Sophus are absent; ikd_Tree.h includes <pcl/point_types.h>) and ships no
// tests or fixtures, so this oracle is NOT pinned by reference outputs
// ("parity unpinned").  Its kNN is cross-checked against scipy's cKDTree
// (an independent exact kNN) in tests/test_oracle.py and its plane fit against
// numpy least squares; see DESIGN.md "Oracle and parity".
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include <omp.h>

namespace {

// ------------------------------------------------------------------ kd-tree
struct Node {
  int32_t pt;        // map point index
  int32_t left = -1, right = -1;
  float lo[3], hi[3];
};

struct Tree {
  std::vector<float> x, y, z;
  std::vector<Node> nodes;
  int32_t root = -1;
  const float* coord(int a) const { return a == 0 ? x.data() : a == 1 ? y.data() : z.data(); }
};

int32_t build_rec(Tree& T, std::vector<int32_t>& st, int l, int r) {
  if (l > r) return -1;
  const int mid = (l + r) >> 1;
  float mn[3] = {INFINITY, INFINITY, INFINITY};
  float mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  for (int i = l; i <= r; ++i) {
    const int32_t p = st[i];
    mn[0] = std::min(mn[0], T.x[p]);
    mn[1] = std::min(mn[1], T.y[p]);
    mn[2] = std::min(mn[2], T.z[p]);
    mx[0] = std::max(mx[0], T.x[p]);
    mx[1] = std::max(mx[1], T.y[p]);
    mx[2] = std::max(mx[2], T.z[p]);
  }
  float range[3];
  for (int i = 0; i < 3; ++i) range[i] = mx[i] - mn[i];
  int axis = 0;
  for (int i = 1; i < 3; ++i)
    if (range[i] > range[axis]) axis = i;
  const float* c = T.coord(axis);
  std::nth_element(st.begin() + l, st.begin() + mid, st.begin() + r + 1,
                   [c](int32_t a, int32_t b) { return c[a] < c[b]; });
  const int32_t id = (int32_t)T.nodes.size();
  T.nodes.push_back(Node{});
  T.nodes[id].pt = st[mid];
  const int32_t L = build_rec(T, st, l, mid - 1);
  const int32_t R = build_rec(T, st, mid + 1, r);
  Node& nd = T.nodes[id];
  nd.left = L;
  nd.right = R;
  const int32_t p = nd.pt;
  const float px[3] = {T.x[p], T.y[p], T.z[p]};
  for (int a = 0; a < 3; ++a) {
    float lo = px[a], hi = px[a];
    if (L >= 0) {
      lo = std::min(lo, T.nodes[L].lo[a]);
      hi = std::max(hi, T.nodes[L].hi[a]);
    }
    if (R >= 0) {
      lo = std::min(lo, T.nodes[R].lo[a]);
      hi = std::max(hi, T.nodes[R].hi[a]);
    }
    nd.lo[a] = lo;
    nd.hi[a] = hi;
  }
  return id;
}

struct Cand {
  float dist;
  float x;     // PointType_CMP tie-break coordinate
  int32_t pt;
};

// PointType_CMP::operator< (ikd_Tree.h:96-99)
inline bool cmp_less(const Cand& a, const Cand& b) {
  if (std::fabs(a.dist - b.dist) < 1e-10) return a.x < b.x;
  return a.dist < b.dist;
}

// MANUAL_HEAP (ikd_Tree.h:103-168): max-heap with a hard capacity
struct Heap {
  Cand h[16];
  int size = 0, cap;
  explicit Heap(int c) : cap(c) {}
  void push(const Cand& p) {
    if (size >= cap) return;
    int i = size;
    h[i] = p;
    Cand tmp = h[i];
    while (i > 0) {
      const int anc = (i - 1) / 2;
      if (cmp_less(h[anc], tmp)) {
        h[i] = h[anc];
        i = anc;
      } else {
        break;
      }
    }
    h[i] = tmp;
    ++size;
  }
  void pop() {
    if (size == 0) return;
    h[0] = h[size - 1];
    --size;
    int i = 0, l = 1;
    Cand tmp = h[0];
    while (l < size) {
      if (l + 1 < size && cmp_less(h[l], h[l + 1])) ++l;
      if (cmp_less(tmp, h[l])) {
        h[i] = h[l];
        i = l;
        l = 2 * i + 1;
      } else {
        break;
      }
    }
    h[i] = tmp;
  }
  const Cand& top() const { return h[0]; }
};

inline float box_dist(const Tree& T, int32_t n, float qx, float qy, float qz) {
  if (n < 0) return INFINITY;
  const Node& nd = T.nodes[n];
  float d = 0.0f;
  if (qx < nd.lo[0]) d += (qx - nd.lo[0]) * (qx - nd.lo[0]);
  if (qx > nd.hi[0]) d += (qx - nd.hi[0]) * (qx - nd.hi[0]);
  if (qy < nd.lo[1]) d += (qy - nd.lo[1]) * (qy - nd.lo[1]);
  if (qy > nd.hi[1]) d += (qy - nd.hi[1]) * (qy - nd.hi[1]);
  if (qz < nd.lo[2]) d += (qz - nd.lo[2]) * (qz - nd.lo[2]);
  if (qz > nd.hi[2]) d += (qz - nd.hi[2]) * (qz - nd.hi[2]);
  return d;
}

void search(const Tree& T, int32_t n, int k, float qx, float qy, float qz, Heap& q) {
  if (n < 0) return;
  const float max_sq = INFINITY;
  const float cur = box_dist(T, n, qx, qy, qz);
  if (cur > max_sq) return;
  const Node& nd = T.nodes[n];
  {
    const int32_t p = nd.pt;
    const float dx = qx - T.x[p], dy = qy - T.y[p], dz = qz - T.z[p];
    const float dist = dx * dx + dy * dy + dz * dz;
    if (dist <= max_sq && (q.size < k || dist < q.top().dist)) {
      if (q.size >= k) q.pop();
      q.push(Cand{dist, T.x[p], p});
    }
  }
  const float dl = box_dist(T, nd.left, qx, qy, qz);
  const float dr = box_dist(T, nd.right, qx, qy, qz);
  if (q.size < k || (dl < q.top().dist && dr < q.top().dist)) {
    if (dl <= dr) {
      search(T, nd.left, k, qx, qy, qz, q);
      if (q.size < k || dr < q.top().dist) search(T, nd.right, k, qx, qy, qz, q);
    } else {
      search(T, nd.right, k, qx, qy, qz, q);
      if (q.size < k || dl < q.top().dist) search(T, nd.left, k, qx, qy, qz, q);
    }
  } else {
    if (dl < q.top().dist) search(T, nd.left, k, qx, qy, qz, q);
    if (dr < q.top().dist) search(T, nd.right, k, qx, qy, qz, q);
  }
}

// Nearest_Search: returns k_found, fills ascending outputs
int nearest(const Tree& T, float qx, float qy, float qz, int k, int32_t* idx, float* sqd) {
  Heap q(2 * k);
  search(T, T.root, k, qx, qy, qz, q);
  const int kf = std::min(k, q.size);
  for (int i = kf - 1; i >= 0; --i) {
    idx[i] = q.top().pt;
    sqd[i] = q.top().dist;
    q.pop();
  }
  for (int i = kf; i < k; ++i) {
    idx[i] = -1;
    sqd[i] = INFINITY;
  }
  return kf;
}

// ------------------------------------------------------------------ plane
// Eigen ColPivHouseholderQR<Matrix<float,5,3>>::solve(-1) restated with
// left-to-right sums; then common_lib.h:244-257.
void qr_solve_m1(const float nb[5][3], float sol[3]) {
  const float eps = 1.1920928955078125e-07f;
  const float tiny = 1.17549435082228750797e-38f;
  float a[3][5];
  for (int c = 0; c < 3; ++c)
    for (int r = 0; r < 5; ++r) a[c][r] = nb[r][c];
  float nd[3], nu[3];
  for (int c = 0; c < 3; ++c) {
    float s = a[c][0] * a[c][0];
    for (int r = 1; r < 5; ++r) s = s + a[c][r] * a[c][r];
    nd[c] = std::sqrt(s);
    nu[c] = nd[c];
  }
  float mx = nu[0];
  for (int c = 1; c < 3; ++c)
    if (nu[c] > mx) mx = nu[c];
  const float tt = mx * eps;
  const float thr_helper = (tt * tt) / 5.0f;
  const float downdate_thr = std::sqrt(eps);
  int nzp = 3;
  int trans[3];
  float hc[3];
  for (int k = 0; k < 3; ++k) {
    int big = k;
    float bv = nu[k];
    for (int j = k + 1; j < 3; ++j)
      if (nu[j] > bv) {
        bv = nu[j];
        big = j;
      }
    if (nzp == 3 && bv * bv < thr_helper * (float)(5 - k)) nzp = k;
    trans[k] = big;
    if (big != k) {
      for (int r = 0; r < 5; ++r) std::swap(a[k][r], a[big][r]);
      std::swap(nu[k], nu[big]);
      std::swap(nd[k], nd[big]);
    }
    float tail = 0.0f;
    for (int r = k + 1; r < 5; ++r) tail = (r == k + 1) ? a[k][r] * a[k][r] : tail + a[k][r] * a[k][r];
    const float c0 = a[k][k];
    float tau, beta;
    if (tail <= tiny) {
      tau = 0.0f;
      beta = c0;
      for (int r = k + 1; r < 5; ++r) a[k][r] = 0.0f;
    } else {
      beta = std::sqrt(c0 * c0 + tail);
      if (c0 >= 0.0f) beta = -beta;
      const float den = c0 - beta;
      for (int r = k + 1; r < 5; ++r) a[k][r] = a[k][r] / den;
      tau = (beta - c0) / beta;
    }
    a[k][k] = beta;
    hc[k] = tau;
    if (tau != 0.0f) {
      for (int j = k + 1; j < 3; ++j) {
        float t = 0.0f;
        for (int r = k + 1; r < 5; ++r) t = (r == k + 1) ? a[k][r] * a[j][r] : t + a[k][r] * a[j][r];
        t = t + a[j][k];
        a[j][k] = a[j][k] - tau * t;
        for (int r = k + 1; r < 5; ++r) a[j][r] = a[j][r] - (tau * a[k][r]) * t;
      }
    }
    for (int j = k + 1; j < 3; ++j) {
      if (nu[j] != 0.0f) {
        float temp = std::fabs(a[j][k]) / nu[j];
        temp = (1.0f + temp) * (1.0f - temp);
        temp = temp < 0.0f ? 0.0f : temp;
        const float q = nu[j] / nd[j];
        const float temp2 = temp * (q * q);
        if (temp2 <= downdate_thr) {
          float s = 0.0f;
          for (int r = k + 1; r < 5; ++r) s = (r == k + 1) ? a[j][r] * a[j][r] : s + a[j][r] * a[j][r];
          nd[j] = std::sqrt(s);
          nu[j] = nd[j];
        } else {
          nu[j] = nu[j] * std::sqrt(temp);
        }
      }
    }
  }
  int perm[3] = {0, 1, 2};
  for (int k = 0; k < 3; ++k) std::swap(perm[k], perm[trans[k]]);
  sol[0] = sol[1] = sol[2] = 0.0f;
  if (nzp > 0) {
    float c[5] = {-1.0f, -1.0f, -1.0f, -1.0f, -1.0f};
    for (int k = 0; k < nzp; ++k) {
      const float tau = hc[k];
      if (tau == 0.0f) continue;
      float t = 0.0f;
      for (int r = k + 1; r < 5; ++r) t = (r == k + 1) ? a[k][r] * c[r] : t + a[k][r] * c[r];
      t = t + c[k];
      c[k] = c[k] - tau * t;
      for (int r = k + 1; r < 5; ++r) c[r] = c[r] - (tau * a[k][r]) * t;
    }
    for (int i = nzp - 1; i >= 0; --i) {
      if (c[i] != 0.0f) {
        c[i] = c[i] / a[i][i];
        for (int r = 0; r < i; ++r) c[r] = c[r] - c[i] * a[i][r];
      }
    }
    for (int i = 0; i < nzp; ++i) sol[perm[i]] = c[i];
  }
}

bool esti_plane(const float nb[5][3], float threshold, float abcd[4]) {
  float sol[3];
  qr_solve_m1(nb, sol);
  const float n = std::sqrt((sol[0] * sol[0] + sol[1] * sol[1]) + sol[2] * sol[2]);
  abcd[0] = sol[0] / n;
  abcd[1] = sol[1] / n;
  abcd[2] = sol[2] / n;
  abcd[3] = (float)(1.0 / (double)n);
  for (int j = 0; j < 5; ++j) {
    const float r = ((abcd[0] * nb[j][0] + abcd[1] * nb[j][1]) + abcd[2] * nb[j][2]) + abcd[3];
    if (std::fabs(r) > threshold) return false;
  }
  return true;
}

// ------------------------------------------------------------------ SO3
struct Q {
  double w, x, y, z;
};

void qrot(const Q& q, const double v[3], double o[3]) {
  double u[3] = {q.y * v[2] - q.z * v[1], q.z * v[0] - q.x * v[2], q.x * v[1] - q.y * v[0]};
  for (int i = 0; i < 3; ++i) u[i] = u[i] + u[i];
  const double c[3] = {q.y * u[2] - q.z * u[1], q.z * u[0] - q.x * u[2], q.x * u[1] - q.y * u[0]};
  for (int i = 0; i < 3; ++i) o[i] = (v[i] + q.w * u[i]) + c[i];
}

void qmat(const Q& q, double R[9]) {
  const double tx = 2.0 * q.x, ty = 2.0 * q.y, tz = 2.0 * q.z;
  const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
  const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
  const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
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

Q qmul(const Q& a, const Q& b) {
  return Q{a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z,
           a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y,
           a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z,
           a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x};
}

Q qnorm(const Q& q) {
  const double n = std::sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
  return Q{q.w / n, q.x / n, q.y / n, q.z / n};
}

Q so3_exp(const double w[3]) {
  const double th = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
  const double re = std::cos(0.5 * th);
  double im;
  if (th < 1e-10) {
    const double t2 = th * th;
    im = 0.5 - 0.0208333 * t2 + 0.000260417 * t2 * t2;
  } else {
    im = std::sin(0.5 * th) / th;
  }
  return qnorm(Q{re, im * w[0], im * w[1], im * w[2]});
}

void so3_log(const Q& q, double o[3]) {
  const double n = std::sqrt(q.x * q.x + q.y * q.y + q.z * q.z);
  double f;
  if (n < 1e-10)
    f = 2.0 / q.w - 2.0 * (n * n) / (q.w * (q.w * q.w));
  else if (std::fabs(q.w) < 1e-10)
    f = (q.w > 0 ? M_PI : -M_PI) / n;
  else
    f = 2.0 * std::atan(n / q.w) / n;
  o[0] = f * q.x;
  o[1] = f * q.y;
  o[2] = f * q.z;
}

Q q_from_mat(const double m[9]) {
  auto M = [&](int r, int c) { return m[r * 3 + c]; };
  double t = M(0, 0) + M(1, 1) + M(2, 2);
  Q q;
  if (t > 0.0) {
    t = std::sqrt(t + 1.0);
    q.w = 0.5 * t;
    t = 0.5 / t;
    q.x = (M(2, 1) - M(1, 2)) * t;
    q.y = (M(0, 2) - M(2, 0)) * t;
    q.z = (M(1, 0) - M(0, 1)) * t;
  } else {
    int i = 0;
    if (M(1, 1) > M(0, 0)) i = 1;
    if (M(2, 2) > M(i, i)) i = 2;
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    t = std::sqrt(M(i, i) - M(j, j) - M(k, k) + 1.0);
    double v[3];
    v[i] = 0.5 * t;
    t = 0.5 / t;
    q.w = (M(k, j) - M(j, k)) * t;
    v[j] = (M(j, i) + M(i, j)) * t;
    v[k] = (M(k, i) + M(i, k)) * t;
    q.x = v[0];
    q.y = v[1];
    q.z = v[2];
  }
  return q;
}

// state layout = slio_state: pos3 rot4 rli4 tli3 vel3 bg3 ba3 grav3 (26 doubles)
struct State {
  double pos[3];
  Q rot;
  Q rli;
  double tli[3], vel[3], bg[3], ba[3], grav[3];
};

void state_load(const double* s, State& x) {
  std::memcpy(x.pos, s, 24);
  x.rot = Q{s[3], s[4], s[5], s[6]};
  x.rli = Q{s[7], s[8], s[9], s[10]};
  std::memcpy(x.tli, s + 11, 24);
  std::memcpy(x.vel, s + 14, 24);
  std::memcpy(x.bg, s + 17, 24);
  std::memcpy(x.ba, s + 20, 24);
  std::memcpy(x.grav, s + 23, 24);
}

void state_store(const State& x, double* s) {
  std::memcpy(s, x.pos, 24);
  s[3] = x.rot.w;
  s[4] = x.rot.x;
  s[5] = x.rot.y;
  s[6] = x.rot.z;
  s[7] = x.rli.w;
  s[8] = x.rli.x;
  s[9] = x.rli.y;
  s[10] = x.rli.z;
  std::memcpy(s + 11, x.tli, 24);
  std::memcpy(s + 14, x.vel, 24);
  std::memcpy(s + 17, x.bg, 24);
  std::memcpy(s + 20, x.ba, 24);
  std::memcpy(s + 23, x.grav, 24);
}

void boxminus_rot(const Q& a1, const Q& a2, double o[3]) {
  double R1[9], R2[9], M[9];
  qmat(a1, R1);
  qmat(a2, R2);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      M[i * 3 + j] = R2[0 * 3 + i] * R1[0 * 3 + j] + R2[1 * 3 + i] * R1[1 * 3 + j] +
                     R2[2 * 3 + i] * R1[2 * 3 + j];
  so3_log(q_from_mat(M), o);
}

void boxminus(const State& x1, const State& x2, double d[24]) {
  for (int i = 0; i < 3; ++i) {
    d[i] = x1.pos[i] - x2.pos[i];
    d[9 + i] = x1.tli[i] - x2.tli[i];
    d[12 + i] = x1.vel[i] - x2.vel[i];
    d[15 + i] = x1.bg[i] - x2.bg[i];
    d[18 + i] = x1.ba[i] - x2.ba[i];
    d[21 + i] = x1.grav[i] - x2.grav[i];
  }
  boxminus_rot(x1.rot, x2.rot, d + 3);
  boxminus_rot(x1.rli, x2.rli, d + 6);
}

State boxplus(const State& x, const double* f) {
  State r = x;
  for (int i = 0; i < 3; ++i) {
    r.pos[i] = x.pos[i] + f[i];
    r.tli[i] = x.tli[i] + f[9 + i];
    r.vel[i] = x.vel[i] + f[12 + i];
    r.bg[i] = x.bg[i] + f[15 + i];
    r.ba[i] = x.ba[i] + f[18 + i];
    r.grav[i] = x.grav[i] + f[21 + i];
  }
  r.rot = qnorm(qmul(x.rot, so3_exp(f + 3)));
  r.rli = qnorm(qmul(x.rli, so3_exp(f + 6)));
  return r;
}

bool inverse(int N, const std::vector<double>& A, std::vector<double>& out) {
  std::vector<double> a(N * 2 * N);
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < N; ++j) {
      a[i * 2 * N + j] = A[i * N + j];
      a[i * 2 * N + N + j] = (i == j) ? 1.0 : 0.0;
    }
  for (int c = 0; c < N; ++c) {
    int p = c;
    for (int r = c + 1; r < N; ++r)
      if (std::fabs(a[r * 2 * N + c]) > std::fabs(a[p * 2 * N + c])) p = r;
    if (a[p * 2 * N + c] == 0.0) return false;
    if (p != c)
      for (int j = 0; j < 2 * N; ++j) std::swap(a[c * 2 * N + j], a[p * 2 * N + j]);
    const double inv = 1.0 / a[c * 2 * N + c];
    for (int j = 0; j < 2 * N; ++j) a[c * 2 * N + j] *= inv;
    for (int r = 0; r < N; ++r) {
      if (r == c) continue;
      const double f = a[r * 2 * N + c];
      if (f == 0.0) continue;
      for (int j = 0; j < 2 * N; ++j) a[r * 2 * N + j] -= f * a[c * 2 * N + j];
    }
  }
  out.assign(N * N, 0.0);
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < N; ++j) out[i * N + j] = a[i * 2 * N + N + j];
  return true;
}

// ------------------------------------------------------------------ h_share_model
struct PassIO {
  const float *bx, *by, *bz;
  int64_t n;
  int32_t* nbr_idx;  // n*5 (kept across passes like Nearest_Points)
  float* nbr_sqd;
  float* plane;      // n*4
  uint8_t* sel;      // n (point_selected_surf)
  float* resid;      // n
};

// one measurement pass; returns m; fills H (m x 12) and h (m) when non-null
int64_t h_share_model(const Tree& T, const State& x, PassIO& io, bool do_search, bool extrinsic,
                      float plane_thr, float max_sqd, int nthreads, std::vector<double>* H,
                      std::vector<double>* hv) {
  const int64_t n = io.n;
  double Rm[9], RLm[9];
  qmat(x.rot, Rm);
  qmat(x.rli, RLm);
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 256)
  for (int64_t i = 0; i < n; ++i) {
    const double pb[3] = {(double)io.bx[i], (double)io.by[i], (double)io.bz[i]};
    double a[3], w[3];
    qrot(x.rli, pb, a);
    for (int k = 0; k < 3; ++k) a[k] = a[k] + x.tli[k];
    qrot(x.rot, a, w);
    const float qx = (float)(w[0] + x.pos[0]);
    const float qy = (float)(w[1] + x.pos[1]);
    const float qz = (float)(w[2] + x.pos[2]);
    if (do_search) {
      const int kf = nearest(T, qx, qy, qz, 5, io.nbr_idx + i * 5, io.nbr_sqd + i * 5);
      io.sel[i] = (kf < 5) ? 0 : (io.nbr_sqd[i * 5 + 4] > max_sqd ? 0 : 1);
      for (int k = 0; k < 4; ++k) io.plane[i * 4 + k] = NAN;
    }
    io.resid[i] = NAN;
    if (!io.sel[i]) continue;
    io.sel[i] = 0;
    float nb[5][3];
    for (int j = 0; j < 5; ++j) {
      const int32_t p = io.nbr_idx[i * 5 + j];
      nb[j][0] = T.x[p];
      nb[j][1] = T.y[p];
      nb[j][2] = T.z[p];
    }
    float abcd[4];
    if (esti_plane(nb, plane_thr, abcd)) {
      for (int k = 0; k < 4; ++k) io.plane[i * 4 + k] = abcd[k];
      const float pd2 = ((abcd[0] * qx + abcd[1] * qy) + abcd[2] * qz) + abcd[3];
      const double nrm = std::sqrt((pb[0] * pb[0] + pb[1] * pb[1]) + pb[2] * pb[2]);
      const float s = (float)(1.0 - (0.9 * (double)std::fabs(pd2)) / std::sqrt(nrm));
      if ((double)s > 0.9) {
        io.sel[i] = 1;
        io.resid[i] = pd2;
      }
    } else {
      for (int k = 0; k < 4; ++k) io.plane[i * 4 + k] = NAN;
    }
  }
  // compaction + Jacobian rows in index order (esekfom.hpp:176-226)
  int64_t m = 0;
  for (int64_t i = 0; i < n; ++i) m += io.sel[i] ? 1 : 0;
  if (H) {
    H->assign(m * 12, 0.0);
    hv->assign(m, 0.0);
    int64_t r = 0;
    for (int64_t i = 0; i < n; ++i) {
      if (!io.sel[i]) continue;
      const double pb[3] = {(double)io.bx[i], (double)io.by[i], (double)io.bz[i]};
      double pI[3];
      qrot(x.rli, pb, pI);
      for (int k = 0; k < 3; ++k) pI[k] = pI[k] + x.tli[k];
      const double nv[3] = {(double)io.plane[i * 4 + 0], (double)io.plane[i * 4 + 1],
                            (double)io.plane[i * 4 + 2]};
      double C[3];
      for (int k = 0; k < 3; ++k) C[k] = Rm[0 * 3 + k] * nv[0] + (Rm[1 * 3 + k] * nv[1] + Rm[2 * 3 + k] * nv[2]);
      const double A[3] = {0.0 * C[0] + (-pI[2] * C[1] + pI[1] * C[2]),
                           pI[2] * C[0] + (0.0 * C[1] + -pI[0] * C[2]),
                           -pI[1] * C[0] + (pI[0] * C[1] + 0.0 * C[2])};
      double B[3] = {0.0, 0.0, 0.0};
      if (extrinsic) {
        const double S[9] = {0.0, -pb[2], pb[1], pb[2], 0.0, -pb[0], -pb[1], pb[0], 0.0};
        double M[9];
        for (int a = 0; a < 3; ++a)
          for (int b = 0; b < 3; ++b)
            M[a * 3 + b] = S[a * 3 + 0] * RLm[b * 3 + 0] +
                           (S[a * 3 + 1] * RLm[b * 3 + 1] + S[a * 3 + 2] * RLm[b * 3 + 2]);
        for (int a = 0; a < 3; ++a) B[a] = M[a * 3 + 0] * C[0] + (M[a * 3 + 1] * C[1] + M[a * 3 + 2] * C[2]);
      }
      double* row = H->data() + r * 12;
      row[0] = nv[0];
      row[1] = nv[1];
      row[2] = nv[2];
      // esekfom.hpp:213-221: [n, A, B, C] with extrinsic_est, [n, A, 0 x 6] without
      for (int k = 0; k < 3; ++k) {
        row[3 + k] = A[k];
        row[6 + k] = B[k];
        row[9 + k] = extrinsic ? C[k] : 0.0;
      }
      (*hv)[r] = -(double)io.resid[i];
      ++r;
    }
  }
  return m;
}

}  // namespace

// ====================================================================== C-ABI
extern "C" {

void* orc_tree_build(const float* x, const float* y, const float* z, int64_t n) {
  Tree* T = new Tree();
  T->x.assign(x, x + n);
  T->y.assign(y, y + n);
  T->z.assign(z, z + n);
  T->nodes.reserve(n);
  std::vector<int32_t> st(n);
  for (int64_t i = 0; i < n; ++i) st[i] = (int32_t)i;
  T->root = build_rec(*T, st, 0, (int)n - 1);
  return T;
}

void orc_tree_free(void* t) { delete (Tree*)t; }

int orc_knn(void* t, const float* qx, const float* qy, const float* qz, int64_t nq, int k,
            int32_t* idx, float* sqd, int nthreads) {
  const Tree* T = (const Tree*)t;
  if (k < 1 || k > 8) return -1;
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 256)
  for (int64_t i = 0; i < nq; ++i) nearest(*T, qx[i], qy[i], qz[i], k, idx + i * k, sqd + i * k);
  return 0;
}

void orc_qr_solve_m1(const float* nb15, float* sol) {
  float nb[5][3];
  for (int j = 0; j < 5; ++j)
    for (int k = 0; k < 3; ++k) nb[j][k] = nb15[3 * j + k];
  qr_solve_m1(nb, sol);
}

int orc_esti_plane(const float* nb15, float threshold, float* abcd) {
  float nb[5][3];
  for (int j = 0; j < 5; ++j)
    for (int c = 0; c < 3; ++c) nb[j][c] = nb15[j * 3 + c];
  return esti_plane(nb, threshold, abcd) ? 1 : 0;
}

// world query points of a scan for a state (esekfom.hpp:128-132)
int orc_body_to_world(const double* state26, const float* bx, const float* by, const float* bz,
                      int64_t n, float* wx, float* wy, float* wz) {
  State x;
  state_load(state26, x);
  for (int64_t i = 0; i < n; ++i) {
    const double pb[3] = {(double)bx[i], (double)by[i], (double)bz[i]};
    double a[3], w[3];
    qrot(x.rli, pb, a);
    for (int k = 0; k < 3; ++k) a[k] = a[k] + x.tli[k];
    qrot(x.rot, a, w);
    wx[i] = (float)(w[0] + x.pos[0]);
    wy[i] = (float)(w[1] + x.pos[1]);
    wz[i] = (float)(w[2] + x.pos[2]);
  }
  return 0;
}

// One h_share_model pass + sequential H^T H / H^T h sums (91 = 78 + 12 + m).
// nbr/plane/sel arrays are in/out exactly like the reference's globals.
int orc_pass(void* t, const double* state26, const float* bx, const float* by, const float* bz,
             int64_t n, int do_search, int extrinsic, float plane_thr, float max_sqd,
             int32_t* nbr_idx, float* nbr_sqd, float* plane, uint8_t* sel, float* resid,
             double* out91, double* rows14, int nthreads) {
  State x;
  state_load(state26, x);
  PassIO io{bx, by, bz, n, nbr_idx, nbr_sqd, plane, sel, resid};
  std::vector<double> H, hv;
  const int64_t m = h_share_model(*(const Tree*)t, x, io, do_search != 0, extrinsic != 0,
                                  plane_thr, max_sqd, nthreads, &H, &hv);
  if (rows14) {  // per-point rows [h_x (12), -pd2, 1] in point order, zeros if unselected
    std::memset(rows14, 0, sizeof(double) * 14 * n);
    int64_t r = 0;
    for (int64_t i = 0; i < n; ++i) {
      if (!sel[i]) continue;
      for (int j = 0; j < 12; ++j) rows14[i * 14 + j] = H[r * 12 + j];
      rows14[i * 14 + 12] = hv[r];
      rows14[i * 14 + 13] = 1.0;
      ++r;
    }
  }
  int k = 0;
  for (int i = 0; i < 12; ++i)
    for (int j = i; j < 12; ++j) {
      double s = 0.0;
      for (int64_t r = 0; r < m; ++r) s = s + H[r * 12 + i] * H[r * 12 + j];
      out91[k++] = s;
    }
  for (int i = 0; i < 12; ++i) {
    double s = 0.0;
    for (int64_t r = 0; r < m; ++r) s = s + H[r * 12 + i] * hv[r];
    out91[k++] = s;
  }
  out91[90] = (double)m;
  return 0;
}

// Full update_iterated_dyn_share_modified (esekfom.hpp:270-346).
// mode 0: reference control flow; mode 1: exactly maximum_iter passes with
// search every pass.  reference_gain 1 forms the 24 x m K like the reference.
// stats[0..4] = passes, searches, valid_passes, converged, last_m.
int orc_ikf_update(void* t, const float* bx, const float* by, const float* bz, int64_t n,
                   double* state26, double* P, double R, int maximum_iter, int extrinsic,
                   int mode, float plane_thr, float max_sqd, int reference_gain, int nthreads,
                   int32_t* nbr_idx, float* nbr_sqd, uint8_t* sel, int64_t* stats) {
  const Tree& T = *(const Tree*)t;
  State x;
  state_load(state26, x);
  const State x_prop = x;
  std::vector<float> plane(n * 4, NAN), resid(n, NAN);
  std::vector<uint8_t> sel_v(n, 0);
  std::vector<int32_t> idx_v(n * 5, -1);
  std::vector<float> sqd_v(n * 5, INFINITY);
  PassIO io{bx, by, bz, n, idx_v.data(), sqd_v.data(), plane.data(), sel_v.data(), resid.data()};
  bool converge = true;
  int tcount = 0;
  int64_t st[5] = {0, 0, 0, 0, 0};
  std::vector<double> KH(576, 0.0);
  std::vector<double> Pm(P, P + 576);
  const int first = mode == 0 ? -1 : 0;
  bool done = false;
  for (int i = first; i < maximum_iter && !done; ++i) {
    const bool search = mode == 1 ? true : converge;
    std::vector<double> H, hv;
    const int64_t m = h_share_model(T, x, io, search, extrinsic != 0, plane_thr, max_sqd,
                                    nthreads, &H, &hv);
    st[0]++;
    st[1] += search ? 1 : 0;
    st[4] = m;
    if (m < 1) continue;
    st[2]++;
    double dx_new[24];
    boxminus(x, x_prop, dx_new);
    // HTH (12x12 block), exactly H^T H
    std::vector<double> HTH(144, 0.0);
    for (int a = 0; a < 12; ++a)
      for (int b = 0; b < 12; ++b) {
        double s = 0.0;
        for (int64_t r = 0; r < m; ++r) s += H[r * 12 + a] * H[r * 12 + b];
        HTH[a * 12 + b] = s;
      }
    std::vector<double> Pinv, A(576), Kf;
    if (!inverse(24, Pm, Pinv)) return -2;
    for (int a = 0; a < 24; ++a)
      for (int b = 0; b < 24; ++b)
        A[a * 24 + b] = ((a < 12 && b < 12) ? HTH[a * 12 + b] : 0.0) / R + Pinv[a * 24 + b];
    if (!inverse(24, A, Kf)) return -2;
    double Kh[24];
    std::fill(KH.begin(), KH.end(), 0.0);
    if (reference_gain) {
      // K = K_front[:, :12] * H^T / R  (24 x m), then K*h and K*H
      std::vector<double> K(24 * m);
      for (int a = 0; a < 24; ++a)
        for (int64_t r = 0; r < m; ++r) {
          double s = 0.0;
          for (int j = 0; j < 12; ++j) s += Kf[a * 24 + j] * H[r * 12 + j];
          K[a * m + r] = s / R;
        }
      for (int a = 0; a < 24; ++a) {
        double s = 0.0;
        for (int64_t r = 0; r < m; ++r) s += K[a * m + r] * hv[r];
        Kh[a] = s;
        for (int b = 0; b < 12; ++b) {
          double u = 0.0;
          for (int64_t r = 0; r < m; ++r) u += K[a * m + r] * H[r * 12 + b];
          KH[a * 24 + b] = u;
        }
      }
    } else {
      double HTh[12];
      for (int j = 0; j < 12; ++j) {
        double s = 0.0;
        for (int64_t r = 0; r < m; ++r) s += H[r * 12 + j] * hv[r];
        HTh[j] = s;
      }
      for (int a = 0; a < 24; ++a) {
        double s = 0.0;
        for (int j = 0; j < 12; ++j) s += Kf[a * 24 + j] * HTh[j];
        Kh[a] = s / R;
        for (int b = 0; b < 12; ++b) {
          double u = 0.0;
          for (int j = 0; j < 12; ++j) u += Kf[a * 24 + j] * HTH[j * 12 + b];
          KH[a * 24 + b] = u / R;
        }
      }
    }
    double dx[24];
    for (int a = 0; a < 24; ++a) {
      double s = 0.0;
      for (int b = 0; b < 24; ++b) s += (KH[a * 24 + b] - (a == b ? 1.0 : 0.0)) * dx_new[b];
      dx[a] = Kh[a] + s;
    }
    x = boxplus(x, dx);
    if (mode == 1) {
      if (i == maximum_iter - 1) done = true;
      continue;
    }
    converge = true;
    for (int j = 0; j < 24; ++j)
      if (std::fabs(dx[j]) > 0.001) {
        converge = false;
        break;
      }
    if (converge) tcount++;
    if (!tcount && i == maximum_iter - 2) converge = true;
    if (tcount > 1 || i == maximum_iter - 1) done = true;
  }
  if (st[2] > 0 && (done || mode == 1)) {
    std::vector<double> Pn(576, 0.0);
    for (int a = 0; a < 24; ++a)
      for (int b = 0; b < 24; ++b) {
        double s = 0.0;
        for (int c = 0; c < 24; ++c) s += ((a == c ? 1.0 : 0.0) - KH[a * 24 + c]) * Pm[c * 24 + b];
        Pn[a * 24 + b] = s;
      }
    std::memcpy(P, Pn.data(), sizeof(double) * 576);
  }
  st[3] = converge ? 1 : 0;
  state_store(x, state26);
  if (nbr_idx) std::memcpy(nbr_idx, idx_v.data(), sizeof(int32_t) * 5 * n);
  if (nbr_sqd) std::memcpy(nbr_sqd, sqd_v.data(), sizeof(float) * 5 * n);
  if (sel) std::memcpy(sel, sel_v.data(), n);
  if (stats) std::memcpy(stats, st, sizeof(st));
  return 0;
}

}  // extern "C"
