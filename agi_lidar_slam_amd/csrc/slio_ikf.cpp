// slio_ikf.cpp — host C++ IKF driver: the patched
// esekf::update_iterated_dyn_share_modified (esekfom.hpp:270-346).
//
// Each pass runs the device measurement model (slio_iterate_async) and reads
// back only the fixed-order sums H^T H (78), H^T h (12) and m.  The 24 x m
// gain K of the reference is never formed:
//   K * h       = K_front[:, :12] * (H^T h) / R
//   (K * H)[:, :12] = K_front[:, :12] * (H^T H) / R
// and K_front[:, :12] comes from a 12x12 inverse (see filter_step): all
// algebraically identical to esekfom.hpp:306-319.  The control flow
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
// returning K H and dx.  K_front[:, :12] = (H^T H / R + P^-1)^-1 [:, :12] is
// evaluated with the push-through identity
//   (P^-1 + E^T M E)^-1 E^T = P E^T (I + M E P E^T)^-1,  M = H^T H / R,
// i.e. K12 = P[:, :12] (I + M P11)^-1: one 12x12 inverse, no P^-1 (the
// reference inverts two 24x24 matrices per pass, esekfom.hpp:311).  The
// device kernel k_ikf_solve uses exactly this operation order.
bool filter_step(const slio_state& x_prop, const double* P, double R, const double HTH[78],
                 const double HTh[12], slio_state& x, double KH[576], double dx[24]) {
  double dx_new[24];
  boxminus(x, x_prop, dx_new);
  double M[144];
  int k = 0;
  for (int i = 0; i < 12; ++i)
    for (int j = i; j < 12; ++j) {
      const double v = HTH[k] / R;
      M[i * 12 + j] = v;
      M[j * 12 + i] = v;
      ++k;
    }
  double B[144], X[144];
  for (int r = 0; r < 12; ++r)
    for (int j = 0; j < 12; ++j) {
      double s = 0.0;
      for (int q = 0; q < 12; ++q) s += M[r * 12 + q] * P[q * 24 + j];
      B[r * 12 + j] = (r == j ? 1.0 : 0.0) + s;
    }
  if (!invert<12>(B, X)) return false;
  double K12[288];
  for (int r = 0; r < 24; ++r)
    for (int c = 0; c < 12; ++c) {
      double s = 0.0;
      for (int q = 0; q < 12; ++q) s += P[r * 24 + q] * X[q * 12 + c];
      K12[r * 12 + c] = s;
    }
  double Kh[24];
  for (int r = 0; r < 24; ++r) {
    double s = 0.0;
    for (int j = 0; j < 12; ++j) s += K12[r * 12 + j] * HTh[j];
    Kh[r] = s / R;
    for (int c = 0; c < 24; ++c) {
      double v = 0.0;
      if (c < 12)
        for (int j = 0; j < 12; ++j) v += K12[r * 12 + j] * M[j * 12 + c];
      KH[r * 24 + c] = v;
    }
  }
  for (int i = 0; i < 24; ++i) {
    double s = 0.0;
    for (int j = 0; j < 24; ++j) s += (KH[i * 24 + j] - (i == j ? 1.0 : 0.0)) * dx_new[j];
    dx[i] = Kh[i] + s;
  }
  slio_state xn;
  boxplus(x, dx, xn);
  x = xn;
  return true;
}

}  // namespace

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
  double KH[576];
  double dx[24];
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
    if (!filter_step(x_prop, P, R, HTH, HTh, *x, KH, dx)) {
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
      // P = (I - KH) * P  (esekfom.hpp:341-343)
      double Pn[576];
      for (int a = 0; a < 24; ++a)
        for (int b = 0; b < 24; ++b) {
          double s = 0.0;
          for (int c = 0; c < 24; ++c) s += ((a == c ? 1.0 : 0.0) - KH[a * 24 + c]) * P[c * 24 + b];
          Pn[a * 24 + b] = s;
        }
      std::memcpy(P, Pn, sizeof(Pn));
      st.converged = converge ? 1 : 0;
      st.device_ms = dev_ms;
      if (stats) *stats = st;
      return SLIO_OK;
    }
  }
  if (mode == SLIO_MODE_FIXED && st.valid_passes > 0) {
    double Pn[576];
    for (int a = 0; a < 24; ++a)
      for (int b = 0; b < 24; ++b) {
        double s = 0.0;
        for (int c = 0; c < 24; ++c) s += ((a == c ? 1.0 : 0.0) - KH[a * 24 + c]) * P[c * 24 + b];
        Pn[a * 24 + b] = s;
      }
    std::memcpy(P, Pn, sizeof(Pn));
  }
  st.converged = converge ? 1 : 0;
  st.device_ms = dev_ms;
  if (stats) *stats = st;
  return SLIO_OK;
}

}  // extern "C"
