// slio_so3.hpp — host-side restatement of the state algebra the IKF needs.
//
// The reference uses Sophus::SO3 from strasdat/Sophus @ a621ff (non-templated,
// README.md:41) on top of Eigen 3.3 quaternions; neither is in the image, so
// their published algorithms are restated here:
//   SO3::exp      = expAndTheta (unit quaternion from axis-angle, SMALL_EPS 1e-10)
//   SO3::log      = logAndTheta (atan-based, Hertzberg et al.)
//   SO3(Matrix3d) = Eigen Quaternion-from-rotation-matrix (trace branch)
//   SO3 * SO3     = Eigen quaternion product, then normalize()
//   SO3::matrix() = Eigen QuaternionBase::toRotationMatrix
//   SO3 * vector  = Eigen QuaternionBase::_transformVector
// Quaternions are stored (w, x, y, z) in this build.
#pragma once

#include <cmath>

#ifndef SLIO_HD
#if defined(__HIPCC__)
#define SLIO_HD __host__ __device__
#else
#define SLIO_HD
#endif
#endif

namespace slio {

struct Quat {
  double w = 1.0, x = 0.0, y = 0.0, z = 0.0;
};

SLIO_HD inline Quat qmul(const Quat& a, const Quat& b) {
  Quat r;
  r.w = a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z;
  r.x = a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y;
  r.y = a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z;
  r.z = a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x;
  return r;
}

SLIO_HD inline Quat qnormalized(const Quat& q) {
  const double n = sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
  return Quat{q.w / n, q.x / n, q.y / n, q.z / n};
}

// SO3 * vector: Eigen QuaternionBase::_transformVector
//   uv = vec x v; uv += uv; return v + w * uv + vec x uv
SLIO_HD inline void qrotate(const Quat& q, const double v[3], double o[3]) {
  double uv[3] = {q.y * v[2] - q.z * v[1], q.z * v[0] - q.x * v[2], q.x * v[1] - q.y * v[0]};
  uv[0] = uv[0] + uv[0];
  uv[1] = uv[1] + uv[1];
  uv[2] = uv[2] + uv[2];
  const double c[3] = {q.y * uv[2] - q.z * uv[1], q.z * uv[0] - q.x * uv[2], q.x * uv[1] - q.y * uv[0]};
  o[0] = (v[0] + q.w * uv[0]) + c[0];
  o[1] = (v[1] + q.w * uv[1]) + c[1];
  o[2] = (v[2] + q.w * uv[2]) + c[2];
}

// row-major 3x3
SLIO_HD inline void qmatrix(const Quat& q, double R[9]) {
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

// Eigen Quaternion(Matrix3) (Quaternion.h quaternionbase_assign_impl): trace
// branch, else i = argmax diagonal, j = (i+1)%3, k = (j+1)%3 -- written out per
// i so no local array is indexed at run time (that lowers to GPU scratch).
SLIO_HD inline Quat qfrom_matrix(const double m[9]) {
  const double m00 = m[0], m01 = m[1], m02 = m[2];
  const double m10 = m[3], m11 = m[4], m12 = m[5];
  const double m20 = m[6], m21 = m[7], m22 = m[8];
  Quat q;
  double t = m00 + m11 + m22;
  if (t > 0.0) {
    t = sqrt(t + 1.0);
    q.w = 0.5 * t;
    t = 0.5 / t;
    q.x = (m21 - m12) * t;
    q.y = (m02 - m20) * t;
    q.z = (m10 - m01) * t;
  } else if (!(m11 > m00) && !(m22 > m00)) {  // i = 0, j = 1, k = 2
    t = sqrt(m00 - m11 - m22 + 1.0);
    q.x = 0.5 * t;
    t = 0.5 / t;
    q.w = (m21 - m12) * t;
    q.y = (m10 + m01) * t;
    q.z = (m20 + m02) * t;
  } else if ((m11 > m00) && !(m22 > m11)) {  // i = 1, j = 2, k = 0
    t = sqrt(m11 - m22 - m00 + 1.0);
    q.y = 0.5 * t;
    t = 0.5 / t;
    q.w = (m02 - m20) * t;
    q.z = (m21 + m12) * t;
    q.x = (m01 + m10) * t;
  } else {  // i = 2, j = 0, k = 1
    t = sqrt(m22 - m00 - m11 + 1.0);
    q.z = 0.5 * t;
    t = 0.5 / t;
    q.w = (m10 - m01) * t;
    q.x = (m02 + m20) * t;
    q.y = (m12 + m21) * t;
  }
  return q;
}

constexpr double kSmallEps = 1e-10;

SLIO_HD inline Quat so3_exp(const double om[3]) {
  const double theta = sqrt(om[0] * om[0] + om[1] * om[1] + om[2] * om[2]);
  const double half = 0.5 * theta;
  double imag, real;
  if (theta < kSmallEps) {
    const double t2 = theta * theta;
    const double t4 = t2 * t2;
    imag = 0.5 - 0.0208333 * t2 + 0.000260417 * t4;  // Sophus a621ff's coefficients
    real = cos(half);
  } else if (half < 0.125) {
    // IKF increments: sin(h) / h and cos(h) by their Taylor series through
    // h^12 (remainder < 1e-22 relative at h = 0.125) -- no argument
    // reduction, a short dependent chain on the GPU
    const double u = half * half;
    const double sh = 1.0 + u * (-1.0 / 6 + u * (1.0 / 120 + u * (-1.0 / 5040 + u * (1.0 / 362880 +
                      u * (-1.0 / 39916800 + u * (1.0 / 6227020800.0))))));
    real = 1.0 + u * (-0.5 + u * (1.0 / 24 + u * (-1.0 / 720 + u * (1.0 / 40320 +
           u * (-1.0 / 3628800 + u * (1.0 / 479001600.0))))));
    imag = 0.5 * sh;
  } else {
    double sh;
    sincos(half, &sh, &real);  // one argument reduction for both
    imag = sh / theta;
  }
  return qnormalized(Quat{real, imag * om[0], imag * om[1], imag * om[2]});
}

SLIO_HD inline void so3_log(const Quat& q, double out[3]) {
  const double n = sqrt(q.x * q.x + q.y * q.y + q.z * q.z);
  const double w = q.w;
  double f;
  if (n < kSmallEps) {
    f = 2.0 / w - 2.0 * (n * n) / (w * (w * w));
  } else if (fabs(w) < kSmallEps) {
    f = (w > 0 ? M_PI : -M_PI) / n;
  } else {
    f = 2.0 * atan(n / w) / n;
  }
  out[0] = f * q.x;
  out[1] = f * q.y;
  out[2] = f * q.z;
}

// SO3(a.matrix()^T * b.matrix()).log()  (esekfom.hpp:242-246)
SLIO_HD inline void so3_boxminus(const Quat& b, const Quat& a, double out[3]) {
  double Ra[9], Rb[9], M[9];
  qmatrix(a, Ra);
  qmatrix(b, Rb);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      M[i * 3 + j] = Ra[0 * 3 + i] * Rb[0 * 3 + j] + Ra[1 * 3 + i] * Rb[1 * 3 + j] +
                     Ra[2 * 3 + i] * Rb[2 * 3 + j];
  so3_log(qfrom_matrix(M), out);
}

// In-place Gauss-Jordan inverse with partial pivoting of an n x n row-major
// matrix (stands in for Eigen's PartialPivLU-based inverse()). Returns false
// on an exactly singular pivot.
template <int N>
inline bool invert(const double* A, double* out) {
  using std::fabs;
  double a[N][2 * N];
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < N; ++j) {
      a[i][j] = A[i * N + j];
      a[i][N + j] = (i == j) ? 1.0 : 0.0;
    }
  for (int c = 0; c < N; ++c) {
    int p = c;
    double best = fabs(a[c][c]);
    for (int r = c + 1; r < N; ++r)
      if (fabs(a[r][c]) > best) {
        best = fabs(a[r][c]);
        p = r;
      }
    if (best == 0.0) return false;
    if (p != c)
      for (int j = 0; j < 2 * N; ++j) std::swap(a[c][j], a[p][j]);
    const double inv = 1.0 / a[c][c];
    for (int j = 0; j < 2 * N; ++j) a[c][j] *= inv;
    for (int r = 0; r < N; ++r) {
      if (r == c) continue;
      const double f = a[r][c];
      if (f == 0.0) continue;
      for (int j = 0; j < 2 * N; ++j) a[r][j] -= f * a[c][j];
    }
  }
  for (int i = 0; i < N; ++i)
    for (int j = 0; j < N; ++j) out[i * N + j] = a[i][N + j];
  return true;
}

}  // namespace slio
