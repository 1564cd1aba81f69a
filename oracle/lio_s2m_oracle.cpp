// CPU oracle of LIO-SAM's scan-to-map measurement model (TEST INFRASTRUCTURE
// ONLY: the product never links, loads or calls this).
//   pointAssociateToMap + trans2Affine3f   src/LIO-SAM/src/mapOptmization.cpp:359-373, 455-459
//     (pcl::getTransformation, float, trig correctly rounded)
//   cornerOptimization                     :1303-1432 (cv::eigen = OpenCV hal::Jacobi restated)
//   surfOptimization                       :1438-1515 (Eigen ColPivHouseholderQR: orc_qr_solve_m1)
//   combineOptimizationCoeffs + LMOptimization rows / A^T A / A^T B  :1517-1626
// The 5-NN lists come from the caller (oracle Tree on the same map).
// Parity unpinned: OpenCV / Eigen / PCL are absent; A^T A is summed in fp64
// in point order (corners, then surfs).
#include <cmath>
#include <cstdint>
#include <cstring>
#include <utility>

extern "C" void orc_qr_solve_m1(const float* nb15, float* sol);

namespace {

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
  for (int iters = 0; n > 1 && iters < n * n * 30; ++iters) {
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
    auto rot = [&](float& v0, float& v1) {
      const float a0 = v0, b0 = v1;
      v0 = a0 * c - b0 * s;
      v1 = a0 * s + b0 * c;
    };
    for (int i = 0; i < k; ++i) rot(A[n * i + k], A[n * i + l]);
    for (int i = k + 1; i < l; ++i) rot(A[n * k + i], A[n * i + l]);
    for (int i = l + 1; i < n; ++i) rot(A[n * k + i], A[n * l + i]);
    for (int i = 0; i < n; ++i) rot(V[n * k + i], V[n * l + i]);
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

}  // namespace

extern "C" {

void orc_s2m_transform(const float* tf, const float* bx, const float* by, const float* bz, int64_t n,
                       float* wx, float* wy, float* wz) {
  const float x = tf[3], y = tf[4], z = tf[5];
  auto fc = [](float a) { return (float)std::cos((double)a); };
  auto fs = [](float a) { return (float)std::sin((double)a); };
  const float A = fc(tf[2]), B = fs(tf[2]), C = fc(tf[1]), D = fs(tf[1]), E = fc(tf[0]), F = fs(tf[0]),
              DE = D * E, DF = D * F;
  const float m[12] = {A * C, A * DF - B * E, B * F + A * DE, x, B * C, A * E + B * DF, B * DE - A * F, y,
                       -D,    C * F,          C * E,          z};
  for (int64_t i = 0; i < n; ++i) {
    wx[i] = m[0] * bx[i] + m[1] * by[i] + m[2] * bz[i] + m[3];
    wy[i] = m[4] * bx[i] + m[5] * by[i] + m[6] * bz[i] + m[7];
    wz[i] = m[8] * bx[i] + m[9] * by[i] + m[10] * bz[i] + m[11];
  }
}

void orc_s2m_coeffs(int kind, const float* wx, const float* wy, const float* wz, int64_t n, const float* map_xyz,
                    const int32_t* idx, const float* sqd, float* coeff, uint8_t* sel) {
  for (int64_t i = 0; i < n; ++i) {
    float cf[4] = {0, 0, 0, 0};
    uint8_t ok = 0;
    const float x0 = wx[i], y0 = wy[i], z0 = wz[i];
    if (sqd[5 * i + 4] < 1.0) {
      float nb[15];
      for (int j = 0; j < 5; ++j)
        for (int k = 0; k < 3; ++k) nb[3 * j + k] = map_xyz[3 * (int64_t)idx[5 * i + j] + k];
      if (kind == 0) {
        float cx = 0, cy = 0, cz = 0;
        for (int j = 0; j < 5; ++j) {
          cx += nb[3 * j];
          cy += nb[3 * j + 1];
          cz += nb[3 * j + 2];
        }
        cx /= 5;
        cy /= 5;
        cz /= 5;
        float a11 = 0, a12 = 0, a13 = 0, a22 = 0, a23 = 0, a33 = 0;
        for (int j = 0; j < 5; ++j) {
          const float ax = nb[3 * j] - cx, ay = nb[3 * j + 1] - cy, az = nb[3 * j + 2] - cz;
          a11 += ax * ax;
          a12 += ax * ay;
          a13 += ax * az;
          a22 += ay * ay;
          a23 += ay * az;
          a33 += az * az;
        }
        a11 /= 5, a12 /= 5, a13 /= 5, a22 /= 5, a23 /= 5, a33 /= 5;
        float A[9] = {a11, a12, a13, a12, a22, a23, a13, a23, a33}, W[3], V[9];
        jacobi(A, 3, W, V);
        if (W[0] > 3 * W[1]) {
          const float x1 = cx + 0.1 * V[0], y1 = cy + 0.1 * V[1], z1 = cz + 0.1 * V[2];
          const float x2 = cx - 0.1 * V[0], y2 = cy - 0.1 * V[1], z2 = cz - 0.1 * V[2];
          const float a012 = std::sqrt(((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)) *
                                           ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)) +
                                       ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1)) *
                                           ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1)) +
                                       ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1)) *
                                           ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1)));
          const float l12 = std::sqrt((x1 - x2) * (x1 - x2) + (y1 - y2) * (y1 - y2) + (z1 - z2) * (z1 - z2));
          const float la = ((y1 - y2) * ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)) +
                            (z1 - z2) * ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1))) /
                           a012 / l12;
          const float lb = -((x1 - x2) * ((x0 - x1) * (y0 - y2) - (x0 - x2) * (y0 - y1)) -
                             (z1 - z2) * ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1))) /
                           a012 / l12;
          const float lc = -((x1 - x2) * ((x0 - x1) * (z0 - z2) - (x0 - x2) * (z0 - z1)) +
                             (y1 - y2) * ((y0 - y1) * (z0 - z2) - (y0 - y2) * (z0 - z1))) /
                           a012 / l12;
          const float ld2 = a012 / l12;
          const float s = 1 - 0.9 * std::fabs(ld2);
          cf[0] = s * la, cf[1] = s * lb, cf[2] = s * lc, cf[3] = s * ld2;
          ok = s > 0.1;
        }
      } else {
        float sol[3];
        orc_qr_solve_m1(nb, sol);
        float pa = sol[0], pb = sol[1], pc = sol[2], pd = 1;
        const float ps = std::sqrt(pa * pa + pb * pb + pc * pc);
        pa /= ps, pb /= ps, pc /= ps, pd /= ps;
        bool valid = true;
        for (int j = 0; j < 5; ++j)
          if (std::fabs(pa * nb[3 * j] + pb * nb[3 * j + 1] + pc * nb[3 * j + 2] + pd) > 0.2) {
            valid = false;
            break;
          }
        if (valid) {
          const float pd2 = pa * x0 + pb * y0 + pc * z0 + pd;
          const float s = 1 - 0.9 * std::fabs(pd2) / std::sqrt(std::sqrt(x0 * x0 + y0 * y0 + z0 * z0));
          cf[0] = s * pa, cf[1] = s * pb, cf[2] = s * pc, cf[3] = s * pd2;
          ok = s > 0.1;
        }
      }
    }
    std::memcpy(coeff + 4 * i, cf, sizeof cf);
    sel[i] = ok;
  }
}

// rows of the selected points of up to two clouds (corners first), fp64 sums
void orc_s2m_normal_equations(const float* tf, const float* const* body3, const float* const* coeff,
                              const uint8_t* const* sel, const int64_t* n, int nclouds, float* AtA, float* AtB,
                              int64_t* nsel) {
  auto fc = [](float a) { return (float)std::cos((double)a); };
  auto fs = [](float a) { return (float)std::sin((double)a); };
  const float srx = fs(tf[1]), crx = fc(tf[1]), sry = fs(tf[2]), cry = fc(tf[2]), srz = fs(tf[0]),
              crz = fc(tf[0]);
  double S[36] = {0}, B[6] = {0};
  int64_t cnt = 0;
  for (int q = 0; q < nclouds; ++q) {
    const float* bx = body3[3 * q];
    const float* by = body3[3 * q + 1];
    const float* bz = body3[3 * q + 2];
    for (int64_t i = 0; i < n[q]; ++i) {
      if (!sel[q][i]) continue;
      const float px = by[i], py = bz[i], pz = bx[i];
      const float* cs = coeff[q] + 4 * i;
      const float cx = cs[1], cy = cs[2], cz = cs[0], ci = cs[3];
      const float arx = (crx * sry * srz * px + crx * crz * sry * py - srx * sry * pz) * cx +
                        (-srx * srz * px - crz * srx * py - crx * pz) * cy +
                        (crx * cry * srz * px + crx * cry * crz * py - cry * srx * pz) * cz;
      const float ary = ((cry * srx * srz - crz * sry) * px + (sry * srz + cry * crz * srx) * py + crx * cry * pz) * cx +
                        ((-cry * crz - srx * sry * srz) * px + (cry * srz - crz * srx * sry) * py - crx * sry * pz) * cz;
      const float arz = ((crz * srx * sry - cry * srz) * px + (-cry * crz - srx * sry * srz) * py) * cx +
                        (crx * crz * px - crx * srz * py) * cy +
                        ((sry * srz + cry * crz * srx) * px + (crz * sry - cry * srx * srz) * py) * cz;
      const float a[6] = {arz, arx, ary, cz, cx, cy};
      for (int r = 0; r < 6; ++r) {
        for (int c = 0; c < 6; ++c) S[6 * r + c] += (double)a[r] * (double)a[c];
        B[r] += (double)a[r] * (double)(-ci);
      }
      ++cnt;
    }
  }
  for (int k = 0; k < 36; ++k) AtA[k] = (float)S[k];
  for (int k = 0; k < 6; ++k) AtB[k] = (float)B[k];
  *nsel = cnt;
}

}  // extern "C"
