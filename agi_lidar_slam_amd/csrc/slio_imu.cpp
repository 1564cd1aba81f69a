// slio_imu.cpp -- host side of ImuProcess::UndistortPcl
// (src/S-FAST_LIO/src/IMU_Processing.hpp:253-402): the forward propagation of
// the filter over the frame's IMU samples with esekf::predict
// (include/esekfom.hpp:82-95; get_f / df_dx / df_dw of use-ikfom.hpp:45-124),
// which is a short sequential 24-D recursion, and the IMUpose table
// (Pose6D, common_lib.h) it produces.  The per-point back-propagation over
// that table runs on the device (slio_device.hip, k_undistort).
#include <cmath>
#include <cstring>

#include "slio_common.hpp"
#include "slio_so3.hpp"

using namespace slio;

namespace {

constexpr double kG = 9.81;  // common_lib.h G_m_s2

Quat qof(const double q[4]) { return Quat{q[0], q[1], q[2], q[3]}; }

// x [+] dx (esekfom.hpp:59-73) on the host
void boxplus24(slio_state& x, const double d[24]) {
  for (int k = 0; k < 3; ++k) {
    x.pos[k] = x.pos[k] + d[k];
    x.tli[k] = x.tli[k] + d[9 + k];
    x.vel[k] = x.vel[k] + d[12 + k];
    x.bg[k] = x.bg[k] + d[15 + k];
    x.ba[k] = x.ba[k] + d[18 + k];
    x.grav[k] = x.grav[k] + d[21 + k];
  }
  const Quat r = qnormalized(qmul(qof(x.rot), so3_exp(d + 3)));
  const Quat l = qnormalized(qmul(qof(x.rli), so3_exp(d + 6)));
  x.rot[0] = r.w, x.rot[1] = r.x, x.rot[2] = r.y, x.rot[3] = r.z;
  x.rli[0] = l.w, x.rli[1] = l.x, x.rli[2] = l.y, x.rli[3] = l.z;
}

}  // namespace

extern "C" {

int slio_ikf_predict(slio_state* x, double P[576], double dt, const double Q[144], const double acc[3],
                     const double gyr[3]) {
  if (!x || !P || !Q || !acc || !gyr) {
    set_error("slio_ikf_predict: bad arguments");
    return SLIO_EINVAL;
  }
  double R[9];
  qmatrix(qof(x->rot), R);
  // get_f (use-ikfom.hpp:45-66): vel, omega = gyro - bg, R (acc - ba) + grav
  double f[24] = {0};
  double am[3];
  for (int k = 0; k < 3; ++k) am[k] = acc[k] - x->ba[k];
  for (int i = 0; i < 3; ++i) {
    const double ai = (R[3 * i] * am[0] + R[3 * i + 1] * am[1]) + R[3 * i + 2] * am[2];
    f[i] = x->vel[i];
    f[i + 3] = gyr[i] - x->bg[i];
    f[i + 12] = ai + x->grav[i];
  }
  // df_dx (use-ikfom.hpp:75-96) and df_dw (:105-117), before I + . * dt
  double Fx[576], Fw[288];
  std::memset(Fx, 0, sizeof Fx);
  std::memset(Fw, 0, sizeof Fw);
  const double hat[9] = {0.0, -am[2], am[1], am[2], 0.0, -am[0], -am[1], am[0], 0.0};
  for (int i = 0; i < 3; ++i) {
    Fx[i * 24 + 12 + i] = 1.0;           // (0, 12) I
    Fx[(12 + i) * 24 + 21 + i] = 1.0;    // (12, 21) I
    Fx[(3 + i) * 24 + 15 + i] = -1.0;    // (3, 15) -I
    for (int j = 0; j < 3; ++j) {
      // (12, 3) = -R * hat(acc - ba); (12, 18) = -R
      const double rh = ((-R[3 * i] * hat[j]) + (-R[3 * i + 1] * hat[3 + j])) + (-R[3 * i + 2] * hat[6 + j]);
      Fx[(12 + i) * 24 + 3 + j] = rh;
      Fx[(12 + i) * 24 + 18 + j] = -R[3 * i + j];
      Fw[(12 + i) * 12 + 3 + j] = -R[3 * i + j];  // (12, 3) -R
    }
    Fw[(3 + i) * 12 + i] = -1.0;       // (3, 0) -I
    Fw[(15 + i) * 12 + 6 + i] = 1.0;   // (15, 6) I
    Fw[(18 + i) * 12 + 9 + i] = 1.0;   // (18, 9) I
  }
  // x = x [+] f dt
  double fd[24];
  for (int k = 0; k < 24; ++k) fd[k] = f[k] * dt;
  boxplus24(*x, fd);
  // F = I + Fx dt; P = F P F^T + (dt Fw) Q (dt Fw)^T
  // Every product element is summed over k in ascending order from 0.0, as
  // esekf::predict's dense products do, except that terms whose F or G factor
  // is structurally zero are skipped: F = I + Fx dt has 51 possible non-zeros
  // of 576 and G = Fw dt 18 of 288 (df_dx / df_dw above).  A sum that starts
  // at +0.0 is never -0.0 under round-to-nearest (+0 + -0 = +0, x + -x = +0),
  // so adding a +-0 term leaves it unchanged: the same bits for finite P and
  // Q (an Inf or NaN in P no longer leaks through a zero factor).
  double F[576], FP[576], G[288], GQ[288], Pn[576];
  for (int i = 0; i < 24; ++i)
    for (int j = 0; j < 24; ++j) F[i * 24 + j] = (i == j ? 1.0 : 0.0) + Fx[i * 24 + j] * dt;
  for (int k = 0; k < 288; ++k) G[k] = dt * Fw[k];
  // the structurally non-zero columns of each row of F and G, ascending
  struct Nz {
    int fnz[24][8], fn[24], gnz[24][3], gn[24];
  };
  static const Nz nzt = [] {
    Nz z{};
    for (int i = 0; i < 24; ++i) {
      int* c = z.fnz[i];
      int n = 0;
      if (i < 3) {
        c[n++] = i;
        c[n++] = 12 + i;
      } else if (i < 6) {
        c[n++] = i;
        c[n++] = 12 + i;  // 15 + (i - 3)
      } else if (i >= 12 && i < 15) {
        for (int j = 3; j < 6; ++j) c[n++] = j;
        c[n++] = i;
        for (int j = 18; j < 21; ++j) c[n++] = j;
        c[n++] = 9 + i;  // 21 + (i - 12)
      } else {
        c[n++] = i;
      }
      z.fn[i] = n;
      int m = 0;
      if (i >= 3 && i < 6) z.gnz[i][m++] = i - 3;
      if (i >= 12 && i < 15)
        for (int j = 3; j < 6; ++j) z.gnz[i][m++] = j;
      if (i >= 15 && i < 18) z.gnz[i][m++] = i - 9;   // 6 + (i - 15)
      if (i >= 18 && i < 21) z.gnz[i][m++] = i - 9;   // 9 + (i - 18)
      z.gn[i] = m;
    }
    return z;
  }();
  const auto& fnz = nzt.fnz;
  const auto& fn = nzt.fn;
  const auto& gnz = nzt.gnz;
  const auto& gn = nzt.gn;
  // FP = F P (row i: the rows k of P with F[i][k] != 0, k ascending)
  for (int i = 0; i < 24; ++i) {
    double* r = FP + i * 24;
    for (int j = 0; j < 24; ++j) r[j] = 0.0;
    for (int t = 0; t < fn[i]; ++t) {
      const int k = fnz[i][t];
      const double f = F[i * 24 + k];
      const double* p = P + k * 24;
      for (int j = 0; j < 24; ++j) r[j] = r[j] + f * p[j];
    }
  }
  // GQ = G Q
  for (int i = 0; i < 24; ++i) {
    double* r = GQ + i * 12;
    for (int j = 0; j < 12; ++j) r[j] = 0.0;
    for (int t = 0; t < gn[i]; ++t) {
      const int k = gnz[i][t];
      const double gk = G[i * 12 + k];
      const double* q = Q + k * 12;
      for (int j = 0; j < 12; ++j) r[j] = r[j] + gk * q[j];
    }
  }
  // Pn = FP F^T + GQ G^T.  Element (i, j) sums FP[i][k] F[j][k] over the k of
  // row j of F (ascending), and GQ[i][k] G[j][k] separately, then adds the
  // two; computed as column j of Pn from the transposed FP / GQ so the 24
  // elements of a column go side by side
  double FPT[576], GQT[288], PnT[576], Bt[24];
  for (int i = 0; i < 24; ++i) {
    for (int k = 0; k < 24; ++k) FPT[k * 24 + i] = FP[i * 24 + k];
    for (int k = 0; k < 12; ++k) GQT[k * 24 + i] = GQ[i * 12 + k];
  }
  for (int j = 0; j < 24; ++j) {
    double* a = PnT + j * 24;
    for (int i = 0; i < 24; ++i) a[i] = Bt[i] = 0.0;
    for (int t = 0; t < fn[j]; ++t) {
      const int k = fnz[j][t];
      const double f = F[j * 24 + k];
      const double* c = FPT + k * 24;
      for (int i = 0; i < 24; ++i) a[i] = a[i] + c[i] * f;
    }
    for (int t = 0; t < gn[j]; ++t) {
      const int k = gnz[j][t];
      const double gk = G[j * 12 + k];
      const double* c = GQT + k * 24;
      for (int i = 0; i < 24; ++i) Bt[i] = Bt[i] + c[i] * gk;
    }
    for (int i = 0; i < 24; ++i) a[i] = a[i] + Bt[i];
  }
  for (int i = 0; i < 24; ++i)
    for (int j = 0; j < 24; ++j) Pn[i * 24 + j] = PnT[j * 24 + i];
  std::memcpy(P, Pn, sizeof Pn);
  return SLIO_OK;
}

int slio_imu_forward(const slio_imu_sample* imu, int nimu, double pcl_beg_time, double pcl_end_time,
                     double* last_lidar_end_time, double mean_acc_norm, const double cov_gyr[3],
                     const double cov_acc[3], const double cov_bias_gyr[3], const double cov_bias_acc[3],
                     double acc_s_last[3], double angvel_last[3], slio_state* x, double P[576],
                     slio_imu_pose* poses, int cap, int* npose) {
  if (!imu || nimu < 1 || !last_lidar_end_time || !(mean_acc_norm > 0.0) || !cov_gyr || !cov_acc ||
      !cov_bias_gyr || !cov_bias_acc || !acc_s_last || !angvel_last || !x || !P || !poses || !npose ||
      cap < nimu) {
    set_error("slio_imu_forward: bad arguments");
    return SLIO_EINVAL;
  }
  // IMU_Processing.hpp:255-270: v_imu = [last_imu_] + meas.imu (the caller's
  // imu array), the first pose is the filter state at the scan start
  const double imu_end_time = imu[nimu - 1].t;
  int k = 0;
  auto push = [&](double off, const double a[3], const double g[3]) {
    slio_imu_pose& q = poses[k++];
    q.offset_time = off;
    double R[9];
    qmatrix(qof(x->rot), R);
    for (int i = 0; i < 3; ++i) {
      q.acc[i] = a[i];
      q.gyr[i] = g[i];
      q.vel[i] = x->vel[i];
      q.pos[i] = x->pos[i];
    }
    std::memcpy(q.rot, R, sizeof R);
  };
  push(0.0, acc_s_last, angvel_last);
  // Q: process_noise_cov() with the diagonal blocks of this scan (:304-308)
  double Q[144] = {0};
  for (int i = 0; i < 3; ++i) {
    Q[i * 12 + i] = cov_gyr[i];
    Q[(3 + i) * 12 + 3 + i] = cov_acc[i];
    Q[(6 + i) * 12 + 6 + i] = cov_bias_gyr[i];
    Q[(9 + i) * 12 + 9 + i] = cov_bias_acc[i];
  }
  double in_acc[3] = {0, 0, 0}, in_gyr[3] = {0, 0, 0};
  for (int it = 0; it + 1 < nimu; ++it) {
    const slio_imu_sample& head = imu[it];
    const slio_imu_sample& tail = imu[it + 1];
    if (tail.t < *last_lidar_end_time) continue;  // :283
    for (int i = 0; i < 3; ++i) {
      in_gyr[i] = 0.5 * (head.gyr[i] + tail.gyr[i]);
      in_acc[i] = 0.5 * (head.acc[i] + tail.acc[i]);
      in_acc[i] = in_acc[i] * kG / mean_acc_norm;  // :294
    }
    const double dt = head.t < *last_lidar_end_time ? tail.t - *last_lidar_end_time : tail.t - head.t;
    if (int rc = slio_ikf_predict(x, P, dt, Q, in_acc, in_gyr)) return rc;
    // angvel_last, acc_s_last (:318-332)
    double a[3];
    for (int i = 0; i < 3; ++i) {
      angvel_last[i] = tail.gyr[i] - x->bg[i];
      a[i] = tail.acc[i] * kG / mean_acc_norm;
      a[i] = a[i] - x->ba[i];
    }
    double ra[3];
    qrotate(qof(x->rot), a, ra);  // imu_state.rot * v (Sophus: quaternion _transformVector)
    for (int i = 0; i < 3; ++i) acc_s_last[i] = ra[i] + x->grav[i];
    push(tail.t - pcl_beg_time, acc_s_last, angvel_last);
  }
  // :341-346: the last piece up to the scan end
  const double dt = std::fabs(pcl_end_time - imu_end_time);
  if (int rc = slio_ikf_predict(x, P, dt, Q, in_acc, in_gyr)) return rc;
  *last_lidar_end_time = pcl_end_time;
  *npose = k;
  return SLIO_OK;
}

}  // extern "C"
