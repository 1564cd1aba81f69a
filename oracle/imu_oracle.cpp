// CPU oracle of ImuProcess::UndistortPcl (TEST INFRASTRUCTURE ONLY: the
// product never links, loads or calls this).
//   forward propagation  src/S-FAST_LIO/src/IMU_Processing.hpp:253-346
//   esekf::predict       include/esekfom.hpp:82-95
//   get_f/df_dx/df_dw    include/use-ikfom.hpp:45-117
//   back-propagation     IMU_Processing.hpp:348-401 (the reference's backward
//                        double loop over IMU segments and time-sorted points,
//                        verbatim in structure: the first point, once reached,
//                        stays under the pointer and is compensated again by
//                        every earlier segment whose offset is below its time)
//   Sophus a621ff SO3::exp (expAndTheta, SMALL_EPS 1e-10, libm sin / cos),
//   SO3 * vector = Eigen _transformVector, SO3::matrix = toRotationMatrix.
// The time sort (std::sort with time_list, :266) is taken stable (ties by
// point index).  State: pos, rot (w x y z), rli, tli, vel, bg, ba, grav.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <numeric>
#include <vector>

namespace {

struct Q4 {
  double w, x, y, z;
};

Q4 mul(const Q4& a, const Q4& b) {
  return Q4{a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z, a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y,
            a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z, a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x};
}
Q4 normalized(const Q4& q) {
  const double n = std::sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
  return Q4{q.w / n, q.x / n, q.y / n, q.z / n};
}
Q4 so3_exp(const double o[3]) {  // Sophus a621ff expAndTheta
  const double theta = std::sqrt(o[0] * o[0] + o[1] * o[1] + o[2] * o[2]);
  const double half = 0.5 * theta;
  double imag;
  const double real = std::cos(half);
  if (theta < 1e-10) {
    const double t2 = theta * theta, t4 = t2 * t2;
    imag = 0.5 - 0.0208333 * t2 + 0.000260417 * t4;
  } else {
    imag = std::sin(half) / theta;
  }
  return normalized(Q4{real, imag * o[0], imag * o[1], imag * o[2]});
}
void matrix(const Q4& q, double R[9]) {  // Eigen toRotationMatrix
  const double tx = 2.0 * q.x, ty = 2.0 * q.y, tz = 2.0 * q.z;
  const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
  const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
  const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
  R[0] = 1.0 - (tyy + tzz), R[1] = txy - twz, R[2] = txz + twy;
  R[3] = txy + twz, R[4] = 1.0 - (txx + tzz), R[5] = tyz - twx;
  R[6] = txz - twy, R[7] = tyz + twx, R[8] = 1.0 - (txx + tyy);
}
void rotate(const Q4& q, const double v[3], double o[3]) {  // Eigen _transformVector
  double uv[3] = {q.y * v[2] - q.z * v[1], q.z * v[0] - q.x * v[2], q.x * v[1] - q.y * v[0]};
  for (double& u : uv) u = u + u;
  const double c[3] = {q.y * uv[2] - q.z * uv[1], q.z * uv[0] - q.x * uv[2], q.x * uv[1] - q.y * uv[0]};
  for (int k = 0; k < 3; ++k) o[k] = (v[k] + q.w * uv[k]) + c[k];
}

struct St {
  double s[26];  // pos 0, rot 3, rli 7, tli 11, vel 14, bg 17, ba 20, grav 23
  Q4 rot() const { return Q4{s[3], s[4], s[5], s[6]}; }
  Q4 rli() const { return Q4{s[7], s[8], s[9], s[10]}; }
};

void predict(St& x, double* P, double dt, const double* Q, const double acc[3], const double gyr[3]) {
  double R[9];
  matrix(x.rot(), R);
  double am[3], f[24] = {0};
  for (int k = 0; k < 3; ++k) am[k] = acc[k] - x.s[20 + k];
  for (int i = 0; i < 3; ++i) {
    f[i] = x.s[14 + i];
    f[3 + i] = gyr[i] - x.s[17 + i];
    f[12 + i] = ((R[3 * i] * am[0] + R[3 * i + 1] * am[1]) + R[3 * i + 2] * am[2]) + x.s[23 + i];
  }
  std::vector<double> Fx(576, 0.0), Fw(288, 0.0);
  const double hat[9] = {0.0, -am[2], am[1], am[2], 0.0, -am[0], -am[1], am[0], 0.0};
  for (int i = 0; i < 3; ++i) {
    Fx[i * 24 + 12 + i] = 1.0;
    Fx[(12 + i) * 24 + 21 + i] = 1.0;
    Fx[(3 + i) * 24 + 15 + i] = -1.0;
    for (int j = 0; j < 3; ++j) {
      double s = 0.0;
      for (int k = 0; k < 3; ++k) s = s + (-R[3 * i + k]) * hat[3 * k + j];
      Fx[(12 + i) * 24 + 3 + j] = s;
      Fx[(12 + i) * 24 + 18 + j] = -R[3 * i + j];
      Fw[(12 + i) * 12 + 3 + j] = -R[3 * i + j];
    }
    Fw[(3 + i) * 12 + i] = -1.0;
    Fw[(15 + i) * 12 + 6 + i] = 1.0;
    Fw[(18 + i) * 12 + 9 + i] = 1.0;
  }
  // boxplus(x, f dt)
  double d[24];
  for (int k = 0; k < 24; ++k) d[k] = f[k] * dt;
  for (int k = 0; k < 3; ++k) {
    x.s[k] += d[k];
    x.s[11 + k] += d[9 + k];
    x.s[14 + k] += d[12 + k];
    x.s[17 + k] += d[15 + k];
    x.s[20 + k] += d[18 + k];
    x.s[23 + k] += d[21 + k];
  }
  const Q4 r = normalized(mul(x.rot(), so3_exp(d + 3)));
  const Q4 l = normalized(mul(x.rli(), so3_exp(d + 6)));
  x.s[3] = r.w, x.s[4] = r.x, x.s[5] = r.y, x.s[6] = r.z;
  x.s[7] = l.w, x.s[8] = l.x, x.s[9] = l.y, x.s[10] = l.z;
  std::vector<double> F(576), G(288), FP(576, 0.0), GQ(288, 0.0), Pn(576);
  for (int i = 0; i < 24; ++i)
    for (int j = 0; j < 24; ++j) F[i * 24 + j] = (i == j ? 1.0 : 0.0) + Fx[i * 24 + j] * dt;
  for (int k = 0; k < 288; ++k) G[k] = dt * Fw[k];
  for (int i = 0; i < 24; ++i)
    for (int j = 0; j < 24; ++j) {
      double s = 0.0;
      for (int k = 0; k < 24; ++k) s = s + F[i * 24 + k] * P[k * 24 + j];
      FP[i * 24 + j] = s;
    }
  for (int i = 0; i < 24; ++i)
    for (int j = 0; j < 12; ++j) {
      double s = 0.0;
      for (int k = 0; k < 12; ++k) s = s + G[i * 12 + k] * Q[k * 12 + j];
      GQ[i * 12 + j] = s;
    }
  for (int i = 0; i < 24; ++i)
    for (int j = 0; j < 24; ++j) {
      double a = 0.0, b = 0.0;
      for (int k = 0; k < 24; ++k) a = a + FP[i * 24 + k] * F[j * 24 + k];
      for (int k = 0; k < 12; ++k) b = b + GQ[i * 12 + k] * G[j * 12 + k];
      Pn[i * 24 + j] = a + b;
    }
  std::memcpy(P, Pn.data(), 576 * sizeof(double));
}

struct Pose {
  double off, acc[3], gyr[3], vel[3], pos[3], rot[9];
};

}  // namespace

extern "C" int orc_imu_undistort(const double* imu7, int nimu, double pcl_beg, double pcl_end,
                                 double* last_lidar_end, double mean_acc_norm, const double* cov12,
                                 double* acc_s_last, double* angvel_last, double* state26, double* P,
                                 const float* x, const float* y, const float* z, const float* t, int64_t n,
                                 float* ox, float* oy, float* oz, float* ot, double* poses22, int* npose) {
  const double G_m_s2 = 9.81;
  St st;
  std::memcpy(st.s, state26, sizeof st.s);
  std::vector<Pose> IMUpose;
  auto push = [&](double off) {
    Pose p;
    p.off = off;
    double R[9];
    matrix(st.rot(), R);
    for (int k = 0; k < 3; ++k) {
      p.acc[k] = acc_s_last[k];
      p.gyr[k] = angvel_last[k];
      p.vel[k] = st.s[14 + k];
      p.pos[k] = st.s[k];
    }
    std::memcpy(p.rot, R, sizeof R);
    IMUpose.push_back(p);
  };
  push(0.0);
  double Q[144] = {0};
  for (int i = 0; i < 3; ++i) {
    Q[i * 12 + i] = cov12[i];
    Q[(3 + i) * 12 + 3 + i] = cov12[3 + i];
    Q[(6 + i) * 12 + 6 + i] = cov12[6 + i];
    Q[(9 + i) * 12 + 9 + i] = cov12[9 + i];
  }
  double in_acc[3] = {0, 0, 0}, in_gyr[3] = {0, 0, 0};
  const double imu_end = imu7[7 * (nimu - 1)];
  for (int it = 0; it + 1 < nimu; ++it) {
    const double* hd = imu7 + 7 * it;
    const double* tl = imu7 + 7 * (it + 1);
    if (tl[0] < *last_lidar_end) continue;
    for (int k = 0; k < 3; ++k) {
      in_gyr[k] = 0.5 * (hd[4 + k] + tl[4 + k]);
      in_acc[k] = 0.5 * (hd[1 + k] + tl[1 + k]);
      in_acc[k] = in_acc[k] * G_m_s2 / mean_acc_norm;
    }
    const double dt = hd[0] < *last_lidar_end ? tl[0] - *last_lidar_end : tl[0] - hd[0];
    predict(st, P, dt, Q, in_acc, in_gyr);
    double a[3];
    for (int k = 0; k < 3; ++k) {
      angvel_last[k] = tl[4 + k] - st.s[17 + k];
      a[k] = tl[1 + k] * G_m_s2 / mean_acc_norm - st.s[20 + k];
    }
    double ra[3];
    rotate(st.rot(), a, ra);
    for (int k = 0; k < 3; ++k) acc_s_last[k] = ra[k] + st.s[23 + k];
    push(tl[0] - pcl_beg);
  }
  predict(st, P, std::fabs(pcl_end - imu_end), Q, in_acc, in_gyr);
  *last_lidar_end = pcl_end;
  std::memcpy(state26, st.s, sizeof st.s);
  *npose = (int)IMUpose.size();
  for (size_t k = 0; k < IMUpose.size(); ++k) {
    double* o = poses22 + 22 * k;
    const Pose& p = IMUpose[k];
    o[0] = p.off;
    std::memcpy(o + 1, p.acc, 24);
    std::memcpy(o + 4, p.gyr, 24);
    std::memcpy(o + 7, p.vel, 24);
    std::memcpy(o + 10, p.pos, 24);
    std::memcpy(o + 13, p.rot, 72);
  }
  // step 5: backward over the time-sorted points
  std::vector<int64_t> ord(n);
  std::iota(ord.begin(), ord.end(), 0);
  std::stable_sort(ord.begin(), ord.end(), [&](int64_t a, int64_t b) { return t[a] < t[b]; });
  for (int64_t i = 0; i < n; ++i) {
    ox[i] = x[ord[i]];
    oy[i] = y[ord[i]];
    oz[i] = z[ord[i]];
    ot[i] = t[ord[i]];
  }
  if (n == 0) return 0;
  double Re[9], RL[9];
  matrix(st.rot(), Re);
  matrix(st.rli(), RL);
  const double* TL = st.s + 11;
  int64_t ip = n - 1;
  for (int kp = (int)IMUpose.size() - 1; kp > 0; --kp) {
    const Pose& hd = IMUpose[kp - 1];
    const Pose& tl = IMUpose[kp];
    for (; ot[ip] / double(1000) > hd.off; --ip) {
      const double dt = ot[ip] / double(1000) - hd.off;
      const double w[3] = {tl.gyr[0] * dt, tl.gyr[1] * dt, tl.gyr[2] * dt};
      double Ex[9], Ri[9];
      matrix(so3_exp(w), Ex);
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c)
          Ri[3 * r + c] = (hd.rot[3 * r] * Ex[c] + hd.rot[3 * r + 1] * Ex[3 + c]) + hd.rot[3 * r + 2] * Ex[6 + c];
      const double Pi[3] = {(double)ox[ip], (double)oy[ip], (double)oz[ip]};
      double Tei[3], a[3], b[3], cv[3], d[3];
      for (int k = 0; k < 3; ++k) Tei[k] = ((hd.pos[k] + hd.vel[k] * dt) + ((0.5 * tl.acc[k]) * dt) * dt) - st.s[k];
      for (int r = 0; r < 3; ++r) a[r] = ((RL[3 * r] * Pi[0] + RL[3 * r + 1] * Pi[1]) + RL[3 * r + 2] * Pi[2]) + TL[r];
      for (int r = 0; r < 3; ++r) b[r] = ((Ri[3 * r] * a[0] + Ri[3 * r + 1] * a[1]) + Ri[3 * r + 2] * a[2]) + Tei[r];
      for (int r = 0; r < 3; ++r) cv[r] = ((Re[r] * b[0] + Re[3 + r] * b[1]) + Re[6 + r] * b[2]) - TL[r];
      for (int r = 0; r < 3; ++r) d[r] = (RL[r] * cv[0] + RL[3 + r] * cv[1]) + RL[6 + r] * cv[2];
      ox[ip] = (float)d[0];
      oy[ip] = (float)d[1];
      oz[ip] = (float)d[2];
      if (ip == 0) break;
    }
  }
  return 0;
}
