// slio_ikf.cpp — host C++ IKF driver: the patched
// esekf::update_iterated_dyn_share_modified (esekfom.hpp:270-346).
//
// Each pass runs the device measurement model (slio_iterate_async) and reads
// back only the fixed-order sums H^T H (78), H^T h (12) and m.  The 24 x m
// gain K of the reference is never formed:
//   K * h       = K_front[:, :12] * (H^T h) / R
//   (K * H)[:, :12] = K_front[:, :12] * (H^T H) / R
// and K_front[:, :12] = G S^-1 comes from a 12x12 Cholesky (see filter_step):
// all algebraically identical to esekfom.hpp:306-319.  The control flow
// (passes i = -1 .. maximum_iter-1, re-search only after a converged pass or
// forced at i == maximum_iter-2, skip on effct_feat_num < 1, final
// P = (I - KH) P) follows esekfom.hpp:292-345 line for line.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstring>

#include "slio_common.hpp"
#include "slio_so3.hpp"

namespace slio {
void* internal_stream(slio_handle h);  // slio_device.hip
}

using namespace slio;

namespace {

constexpr double kEpsi = 0.001;  // esekfom.hpp:17

Quat q_of(const double q[4]) { return Quat{q[0], q[1], q[2], q[3]}; }
void q_to(const Quat& q, double o[4]) {
  o[0] = q.w;
  o[1] = q.x;
  o[2] = q.y;
  o[3] = q.z;
}

void boxplus(const slio_state& x, const double f[24], slio_state& r) {
  for (int i = 0; i < 3; ++i) {
    r.pos[i] = x.pos[i] + f[i];
    r.tli[i] = x.tli[i] + f[9 + i];
    r.vel[i] = x.vel[i] + f[12 + i];
    r.bg[i] = x.bg[i] + f[15 + i];
    r.ba[i] = x.ba[i] + f[18 + i];
    r.grav[i] = x.grav[i] + f[21 + i];
  }
  q_to(qnormalized(qmul(q_of(x.rot), so3_exp(f + 3))), r.rot);
  q_to(qnormalized(qmul(q_of(x.rli), so3_exp(f + 6))), r.rli);
}

void boxminus(const slio_state& x1, const slio_state& x2, double d[24]) {
  for (int i = 0; i < 3; ++i) {
    d[i] = x1.pos[i] - x2.pos[i];
    d[9 + i] = x1.tli[i] - x2.tli[i];
    d[12 + i] = x1.vel[i] - x2.vel[i];
    d[15 + i] = x1.bg[i] - x2.bg[i];
    d[18 + i] = x1.ba[i] - x2.ba[i];
    d[21 + i] = x1.grav[i] - x2.grav[i];
  }
  so3_boxminus(q_of(x1.rot), q_of(x2.rot), d + 3);
  so3_boxminus(q_of(x1.rli), q_of(x2.rli), d + 6);
}

slio_pose pose_of(const slio_state& x) {
  slio_pose p;
  std::memcpy(p.rot, x.rot, sizeof(p.rot));
  std::memcpy(p.pos, x.pos, sizeof(p.pos));
  std::memcpy(p.rli, x.rli, sizeof(p.rli));
  std::memcpy(p.tli, x.tli, sizeof(p.tli));
  return p;
}

// One filter update from the pass sums (esekfom.hpp:303-321), updating x and
// returning K H [:, :12] (K H [:, 12:] = 0) and dx.  With M = H^T H / R and
// the push-through identity (P^-1 + E^T M E)^-1 E^T = G S^-1,
// S = P11^-1 + M (SPD), G = P[:, :12] P11^-1:
//   K h + (K H - I) dx_new = G S^-1 v - dx_new,  v = H^T h / R + M dx_new[:12]
//   K H [:, :12] = G S^-1 M
// one 12 x 12 Cholesky per pass instead of the reference's two 24 x 24
// inverses (esekfom.hpp:311).  The device filter step (ikf_solve_block,
// slio_device.hip) performs the same operations in the same order.
bool filter_step(const slio_state& x_prop, const double* P11i, const double* G, double R,
                 const double HTH[78], const double HTh[12], slio_state& x, double K12[288],
                 double dx[24]) {
  double dx_new[24];
  boxminus(x, x_prop, dx_new);
  double M[144], S[144];
  for (int r = 0; r < 12; ++r)
    for (int c = 0; c < 12; ++c) {
      const int i = r <= c ? r : c, j = r <= c ? c : r;
      const double m = HTH[i * 12 - (i * (i - 1)) / 2 + (j - i)] / R;
      M[r * 12 + c] = m;
      S[r * 12 + c] = P11i[r * 12 + c] + m;
    }
  double v[12];
  for (int r = 0; r < 12; ++r) {
    double s2 = 0.0;
    for (int k = 0; k < 12; ++k) s2 = std::fma(M[r * 12 + k], dx_new[k], s2);
    v[r] = HTh[r] / R + s2;
  }
  // S = L L^T (right-looking, column j scaled by 1 / L[j][j])
  double L[144], invd[12];
  std::memcpy(L, S, sizeof(L));
  for (int j = 0; j < 12; ++j) {
    const double d = L[j * 12 + j];
    if (!(d > 0.0)) return false;
    const double ljj = std::sqrt(d);
    const double inv = 1.0 / ljj;
    invd[j] = inv;
    L[j * 12 + j] = ljj;
    for (int i = j + 1; i < 12; ++i) L[i * 12 + j] = L[i * 12 + j] * inv;
    for (int k = j + 1; k < 12; ++k)
      for (int i = k; i < 12; ++i) L[i * 12 + k] = std::fma(-L[i * 12 + j], L[k * 12 + j], L[i * 12 + k]);
  }
  // S y = v
  double r[12], y[12];
  std::memcpy(r, v, sizeof(r));
  for (int j = 0; j < 12; ++j) {
    const double zj = r[j] * invd[j];
    r[j] = zj;
    for (int i = j + 1; i < 12; ++i) r[i] = std::fma(-L[i * 12 + j], zj, r[i]);
  }
  for (int j = 11; j >= 0; --j) {
    const double yj = r[j] * invd[j];
    y[j] = yj;
    for (int i = 0; i < j; ++i) r[i] = std::fma(-L[j * 12 + i], yj, r[i]);
  }
  for (int q = 0; q < 24; ++q) {
    double s2 = 0.0;
    for (int k = 0; k < 12; ++k) s2 = std::fma(G[q * 12 + k], y[k], s2);
    dx[q] = s2 - dx_new[q];
  }
  // K H [:, :12] = G Z, Z = S^-1 M (column by column)
  double Z[144];
  for (int c = 0; c < 12; ++c) {
    double zc[12];
    for (int j = 0; j < 12; ++j) {
      double s2 = M[j * 12 + c];
      for (int k = 0; k < j; ++k) s2 = std::fma(-L[j * 12 + k], zc[k], s2);
      zc[j] = s2 * invd[j];
    }
    for (int j = 11; j >= 0; --j) {
      double s2 = zc[j];
      for (int k = j + 1; k < 12; ++k) s2 = std::fma(-L[k * 12 + j], zc[k], s2);
      zc[j] = s2 * invd[j];
    }
    for (int j = 0; j < 12; ++j) Z[j * 12 + c] = zc[j];
  }
  for (int q = 0; q < 24; ++q)
    for (int c = 0; c < 12; ++c) {
      double s2 = 0.0;
      for (int k = 0; k < 12; ++k) s2 = std::fma(G[q * 12 + k], Z[k * 12 + c], s2);
      K12[q * 12 + c] = s2;
    }
  slio_state xn;
  boxplus(x, dx, xn);
  x = xn;
  return true;
}

// P = (I - K H) P = P - K H [:, :12] P[:12, :]  (esekfom.hpp:341-343)
void covariance_update(double* P, const double K12[288]) {
  double Pn[576];
  for (int a = 0; a < 24; ++a)
    for (int b = 0; b < 24; ++b) {
      double s2 = 0.0;
      for (int k = 0; k < 12; ++k) s2 = std::fma(K12[a * 12 + k], P[k * 24 + b], s2);
      Pn[a * 24 + b] = P[a * 24 + b] - s2;
    }
  std::memcpy(P, Pn, sizeof(Pn));
}

}  // namespace

// Information-form constants of one update (P_ is fixed until its end) on
// the first D error-state components (D = 12, or 6 when H's columns 6..11
// are zero): P_DD^-1 = (P[:D, :D])^-1 (D x D) and G = P[:, :D] P_DD^-1
// (24 x D), both row-major and packed.  The device-resident update
// (slio_ikf_update_device) uses exactly these.
bool slio::info_constants(const double* P, int D, double P11i[144], double G[288]) {
  if (D != 6 && D != 12) return false;
  double PDD[144];
  for (int r = 0; r < D; ++r)
    for (int q = 0; q < D; ++q) PDD[r * D + q] = P[r * 24 + q];
  if (!(D == 12 ? invert<12>(PDD, P11i) : invert<6>(PDD, P11i))) return false;
  for (int r = 0; r < 24; ++r)
    for (int q = 0; q < D; ++q) {
      double v = 0.0;
      for (int k = 0; k < D; ++k) v += P[r * 24 + k] * P11i[k * D + q];
      G[r * D + q] = v;
    }
  return true;
}


extern "C" {

int slio_state_boxplus(const slio_state* x, const double dx[24], slio_state* out) {
  if (!x || !dx || !out) return SLIO_EINVAL;
  slio_state r = *x;
  boxplus(*x, dx, r);
  *out = r;
  return SLIO_OK;
}

int slio_state_boxminus(const slio_state* x1, const slio_state* x2, double dx[24]) {
  if (!x1 || !x2 || !dx) return SLIO_EINVAL;
  boxminus(*x1, *x2, dx);
  return SLIO_OK;
}

int slio_ikf_update(slio_handle h, slio_state* x, double P[576], double R, int maximum_iter,
                    int extrinsic_est, int mode, slio_allreduce_fn reduce, void* reduce_ctx,
                    slio_ikf_stats* stats) {
  if (!h || !x || !P || !(R > 0.0) || maximum_iter < 1 ||
      (mode != SLIO_MODE_REFERENCE && mode != SLIO_MODE_FIXED)) {
    set_error("slio_ikf_update: bad arguments");
    return SLIO_EINVAL;
  }
  slio_ikf_stats st{};
  const slio_state x_prop = *x;
  bool converge = true;  // dyn_share.converge (esekfom.hpp:282)
  int t = 0;
  double K12[288];
  double dx[24];
  double P11i[144], G[288];
  if (!info_constants(P, 12, P11i, G)) {
    set_error("slio_ikf_update: singular covariance block P[:12, :12]");
    return SLIO_EINVAL;
  }
  double sup[SLIO_NSUPER * SLIO_NPROD];
  const int first = (mode == SLIO_MODE_REFERENCE) ? -1 : 0;
  double dev_ms = 0.0;
  for (int i = first; i < maximum_iter; ++i) {
    const bool search = (mode == SLIO_MODE_FIXED) ? true : converge;
    const slio_pose pose = pose_of(*x);
    const auto t0 = std::chrono::steady_clock::now();
    double* d_super = nullptr;
    int rc = slio_iterate_async(h, &pose, search ? 1 : 0, extrinsic_est, &d_super);
    if (rc) return rc;
    if (reduce) {
      rc = reduce(reduce_ctx, d_super, (int64_t)SLIO_NSUPER * SLIO_NPROD, internal_stream(h));
      if (rc) {
        set_error("slio_ikf_update: reduce callback failed");
        return SLIO_EDEVICE;
      }
    }
    rc = slio_super_download(h, sup);
    if (rc) return rc;
    dev_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    double HTH[SLIO_NHTH], HTh[12];
    int64_t m = 0;
    slio_reduce_super(sup, HTH, HTh, &m);
    ++st.passes;
    st.searches += search ? 1 : 0;
    st.last_m = m;
    if (m < 1) {  // dyn_share.valid = false -> continue (esekfom.hpp:187-191, 297-299)
      continue;
    }
    ++st.valid_passes;
    if (!filter_step(x_prop, P11i, G, R, HTH, HTh, *x, K12, dx)) {
      set_error("slio_ikf_update: singular covariance");
      return SLIO_EINVAL;
    }
    if (mode == SLIO_MODE_FIXED) {
      if (i == maximum_iter - 1) break;
      continue;
    }
    converge = true;
    for (int j = 0; j < 24; ++j)
      if (std::fabs(dx[j]) > kEpsi) {
        converge = false;
        break;
      }
    if (converge) ++t;
    if (!t && i == maximum_iter - 2) converge = true;
    if (t > 1 || i == maximum_iter - 1) {
      covariance_update(P, K12);
      st.converged = converge ? 1 : 0;
      st.device_ms = dev_ms;
      if (stats) *stats = st;
      return SLIO_OK;
    }
  }
  if (mode == SLIO_MODE_FIXED && st.valid_passes > 0) covariance_update(P, K12);
  st.converged = converge ? 1 : 0;
  st.device_ms = dev_ms;
  if (stats) *stats = st;
  return SLIO_OK;
}

}  // extern "C"
