// slio_s2m.cpp -- host side of LIO-SAM's LMOptimization
// (src/LIO-SAM/src/mapOptmization.cpp:1627-1700): the 6x6 Gauss-Newton step
// on the normal equations the device forms (slio_s2m_normal_equations), the
// degeneracy projection of the first iteration and the convergence test.
// OpenCV (cv::solve DECOMP_QR, cv::eigen, cv::Mat::inv) is third-party and
// absent; its algorithms are restated in float: Householder QR, the Jacobi
// eigensolver of hal::Jacobi, LU inverse with partial pivoting.
#include <cfloat>
#include <cmath>
#include <cstring>

#include <utility>

#include "slio_common.hpp"

using slio::set_error;

namespace {

// OpenCV lapack.cpp hypot
float cv_hypot(float a, float b) {
  a = std::fabs(a);
  b = std::fabs(b);
  if (a > b) {
    b /= a;
    return a * std::sqrt(1 + b * b);
  }
  if (b > 0) {
    a /= b;
    return b * std::sqrt(1 + a * a);
  }
  return 0;
}

// OpenCV hal::Jacobi (JacobiImpl_) on an n x n symmetric float matrix:
// eigenvalues W descending, eigenvectors the rows of V
void jacobi(float* A, int n, float* W, float* V) {
  const float eps = 1.1920928955078125e-07f;
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) V[i * n + j] = (i == j) ? 1.0f : 0.0f;
  int indR[8], indC[8];
  float mv;
  for (int k = 0; k < n; ++k) {
    W[k] = A[(n + 1) * k];
    if (k < n - 1) {
      int m = k + 1;
      mv = std::fabs(A[n * k + m]);
      for (int i = k + 2; i < n; ++i) {
        const float val = std::fabs(A[n * k + i]);
        if (mv < val) mv = val, m = i;
      }
      indR[k] = m;
    }
    if (k > 0) {
      int m = 0;
      mv = std::fabs(A[k]);
      for (int i = 1; i < k; ++i) {
        const float val = std::fabs(A[n * i + k]);
        if (mv < val) mv = val, m = i;
      }
      indC[k] = m;
    }
  }
  if (n > 1)
    for (int iters = 0; iters < n * n * 30; ++iters) {
      int k = 0;
      mv = std::fabs(A[indR[0]]);
      for (int i = 1; i < n - 1; ++i) {
        const float val = std::fabs(A[n * i + indR[i]]);
        if (mv < val) mv = val, k = i;
      }
      int l = indR[k];
      for (int i = 1; i < n; ++i) {
        const float val = std::fabs(A[n * indC[i] + i]);
        if (mv < val) mv = val, k = indC[i], l = i;
      }
      const float p = A[n * k + l];
      if (std::fabs(p) <= eps) break;
      float y = (float)((W[l] - W[k]) * 0.5);
      float t = std::fabs(y) + cv_hypot(p, y);
      float s = cv_hypot(p, t);
      const float c = t / s;
      s = p / s;
      t = (p / t) * p;
      if (y < 0) s = -s, t = -t;
      A[n * k + l] = 0;
      W[k] -= t;
      W[l] += t;
      float a0, b0;
#define SLIO_ROT(v0, v1) a0 = v0, b0 = v1, v0 = a0 * c - b0 * s, v1 = a0 * s + b0 * c
      for (int i = 0; i < k; ++i) SLIO_ROT(A[n * i + k], A[n * i + l]);
      for (int i = k + 1; i < l; ++i) SLIO_ROT(A[n * k + i], A[n * i + l]);
      for (int i = l + 1; i < n; ++i) SLIO_ROT(A[n * k + i], A[n * l + i]);
      for (int i = 0; i < n; ++i) SLIO_ROT(V[n * k + i], V[n * l + i]);
#undef SLIO_ROT
      for (int j = 0; j < 2; ++j) {
        const int idx = j == 0 ? k : l;
        if (idx < n - 1) {
          int m = idx + 1;
          mv = std::fabs(A[n * idx + m]);
          for (int i = idx + 2; i < n; ++i) {
            const float val = std::fabs(A[n * idx + i]);
            if (mv < val) mv = val, m = i;
          }
          indR[idx] = m;
        }
        if (idx > 0) {
          int m = 0;
          mv = std::fabs(A[idx]);
          for (int i = 1; i < idx; ++i) {
            const float val = std::fabs(A[n * i + idx]);
            if (mv < val) mv = val, m = i;
          }
          indC[idx] = m;
        }
      }
    }
  for (int k = 0; k < n - 1; ++k) {
    int m = k;
    for (int i = k + 1; i < n; ++i)
      if (W[m] < W[i]) m = i;
    if (k != m) {
      std::swap(W[m], W[k]);
      for (int i = 0; i < n; ++i) std::swap(V[n * m + i], V[n * k + i]);
    }
  }
}

// A x = b (6x6, float) by Householder QR.  false where OpenCV's QRImpl gives
// up (cv::solve DECOMP_QR -> hal::QR32f with eps = 10 * FLT_EPSILON: a
// diagonal entry of R below eps in magnitude)
bool qr_solve6(const float* A_in, const float* b_in, float* x) {
  float A[36], b[6];
  std::memcpy(A, A_in, sizeof A);
  std::memcpy(b, b_in, sizeof b);
  for (int k = 0; k < 6; ++k) {
    float nrm = 0;
    for (int i = k; i < 6; ++i) nrm += A[6 * i + k] * A[6 * i + k];
    nrm = std::sqrt(nrm);
    if (nrm == 0) return false;
    const float alpha = A[6 * k + k] > 0 ? -nrm : nrm;
    float v[6] = {0};
    for (int i = k; i < 6; ++i) v[i] = A[6 * i + k];
    v[k] -= alpha;
    float vv = 0;
    for (int i = k; i < 6; ++i) vv += v[i] * v[i];
    if (vv == 0) continue;
    for (int j = k; j < 6; ++j) {
      float d = 0;
      for (int i = k; i < 6; ++i) d += v[i] * A[6 * i + j];
      const float f = 2 * d / vv;
      for (int i = k; i < 6; ++i) A[6 * i + j] -= f * v[i];
    }
    float d = 0;
    for (int i = k; i < 6; ++i) d += v[i] * b[i];
    const float f = 2 * d / vv;
    for (int i = k; i < 6; ++i) b[i] -= f * v[i];
  }
  for (int i = 5; i >= 0; --i) {
    float s = b[i];
    for (int j = i + 1; j < 6; ++j) s -= A[6 * i + j] * x[j];
    if (std::fabs(A[6 * i + i]) < 10.0f * FLT_EPSILON) return false;
    x[i] = s / A[6 * i + i];
  }
  return true;
}

// inverse by LU with partial pivoting (cv::Mat::inv, DECOMP_LU)
bool inv6(const float* M, float* out) {
  float a[36], b[36];
  std::memcpy(a, M, sizeof a);
  for (int i = 0; i < 36; ++i) b[i] = (i % 7 == 0) ? 1.0f : 0.0f;
  for (int k = 0; k < 6; ++k) {
    int p = k;
    for (int i = k + 1; i < 6; ++i)
      if (std::fabs(a[6 * i + k]) > std::fabs(a[6 * p + k])) p = i;
    if (a[6 * p + k] == 0) return false;
    if (p != k)
      for (int j = 0; j < 6; ++j) {
        std::swap(a[6 * p + j], a[6 * k + j]);
        std::swap(b[6 * p + j], b[6 * k + j]);
      }
    for (int i = k + 1; i < 6; ++i) {
      const float f = a[6 * i + k] / a[6 * k + k];
      for (int j = k; j < 6; ++j) a[6 * i + j] -= f * a[6 * k + j];
      for (int j = 0; j < 6; ++j) b[6 * i + j] -= f * b[6 * k + j];
    }
  }
  for (int c = 0; c < 6; ++c)
    for (int i = 5; i >= 0; --i) {
      float s = b[6 * i + c];
      for (int j = i + 1; j < 6; ++j) s -= a[6 * i + j] * out[6 * j + c];
      out[6 * i + c] = s / a[6 * i + i];
    }
  return true;
}

}  // namespace

extern "C" int slio_s2m_lm_step(const float AtA[36], const float AtB[6], int64_t nsel, int iter_count,
                                float transform[6], int* is_degenerate, float matP[36], int* converged) {
  if (!AtA || !AtB || !transform || !is_degenerate || !matP || !converged) {
    set_error("slio_s2m_lm_step: bad arguments");
    return SLIO_EINVAL;
  }
  *converged = 0;
  if (nsel < 50) return 1;  // :1573-1576: too few correspondences, no update
  float X[6];
  // cv::solve(matAtA, matAtB, matX, DECOMP_QR) (:1620): on a (numerically)
  // singular A^T A it returns false with matX zeroed, and LMOptimization
  // ignores the return value -- a zero step, which then reads as converged
  if (!qr_solve6(AtA, AtB, X))
    for (float& v : X) v = 0.0f;
  if (iter_count == 0) {
    // :1633-1656: eigen-decomposition of A^T A; directions with eigenvalue
    // < 100 (smallest first) are not updated
    float A[36], E[6], V[36], V2[36];
    std::memcpy(A, AtA, sizeof A);
    jacobi(A, 6, E, V);
    std::memcpy(V2, V, sizeof V);
    *is_degenerate = 0;
    for (int i = 5; i >= 0; --i) {
      if (E[i] < 100.0f) {
        for (int j = 0; j < 6; ++j) V2[6 * i + j] = 0;
        *is_degenerate = 1;
      } else {
        break;
      }
    }
    float Vi[36];
    if (!inv6(V, Vi)) {
      set_error("slio_s2m_lm_step: singular eigenvector matrix");
      return SLIO_EINVAL;
    }
    for (int i = 0; i < 6; ++i)
      for (int j = 0; j < 6; ++j) {
        double s = 0;
        for (int k = 0; k < 6; ++k) s += (double)Vi[6 * i + k] * (double)V2[6 * k + j];
        matP[6 * i + j] = (float)s;
      }
  }
  if (*is_degenerate) {
    float X2[6];
    for (int i = 0; i < 6; ++i) {
      double s = 0;
      for (int k = 0; k < 6; ++k) s += (double)matP[6 * i + k] * (double)X[k];
      X2[i] = (float)s;
    }
    std::memcpy(X, X2, sizeof X);
  }
  for (int k = 0; k < 6; ++k) transform[k] += X[k];
  const float r2d = (float)(180.0 / M_PI);
  const float deltaR = std::sqrt(std::pow(X[0] * r2d, 2) + std::pow(X[1] * r2d, 2) + std::pow(X[2] * r2d, 2));
  const float deltaT = std::sqrt(std::pow(X[3] * 100, 2) + std::pow(X[4] * 100, 2) + std::pow(X[5] * 100, 2));
  *converged = (deltaR < 0.05 && deltaT < 0.05) ? 1 : 0;
  return SLIO_OK;
}
