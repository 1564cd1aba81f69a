// slio_plane.hpp — device restatement of esti_plane (common_lib.h:102-134).
//
// The reference solves A * n = -1 (A = the 5 neighbours, 5x3 float) with
// Eigen's ColPivHouseholderQR<Matrix<float,5,3>>::solve, normalises n and
// rejects the plane if any neighbour lies farther than `threshold` from it.
// Eigen 3.3.4+ is third-party and absent from the image, so this is a
// restatement of its published algorithm (ColPivHouseholderQR::computeInPlace
// with LAPACK xGEQPF norm downdating, makeHouseholder, applyHouseholderOnTheLeft,
// HouseholderSequence^T applied H_0 first, upper-triangular back substitution
// with the `rhs[i] != 0` guard, column permutation).  Every reduction is
// summed left-to-right: that is the build's canonical order, shared bit for
// bit with oracle/slio_oracle.cpp (Eigen's own order depends on packet width
// and runtime alignment, so parity with Eigen itself is at tolerance only).
// All indices are compile-time after unrolling so the 5x3 tile stays in
// VGPRs (runtime-indexed arrays would go to scratch).
#pragma once

#include <hip/hip_runtime.h>

namespace slio {

template <int C0, int C1>
__device__ __forceinline__ void cond_swap_cols(float (&a)[3][5], float (&nu)[3],
                                               float (&nd)[3], bool doit) {
#pragma unroll
  for (int r = 0; r < 5; ++r) {
    float x = a[C0][r], y = a[C1][r];
    a[C0][r] = doit ? y : x;
    a[C1][r] = doit ? x : y;
  }
  float x = nu[C0], y = nu[C1];
  nu[C0] = doit ? y : x;
  nu[C1] = doit ? x : y;
  x = nd[C0];
  y = nd[C1];
  nd[C0] = doit ? y : x;
  nd[C1] = doit ? x : y;
}

// nb[j] = (x, y, z) of neighbour j in ascending-distance order.
// Returns true and fills abcd when the plane is accepted.
// A x = -1 for the 5x3 A of the neighbours (ColPivHouseholderQR solve)
__device__ __forceinline__ void qr_solve_m1_dev(const float (&nb)[5][3], float (&sol)[3]) {
  constexpr float kEps = 1.1920928955078125e-07f;    // FLT_EPSILON
  constexpr float kTiny = 1.17549435082228750797e-38f; // FLT_MIN
  float a[3][5];
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int r = 0; r < 5; ++r) a[c][r] = nb[r][c];

  float nd[3], nu[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    float s = a[c][0] * a[c][0];
#pragma unroll
    for (int r = 1; r < 5; ++r) s = s + a[c][r] * a[c][r];
    nd[c] = sqrtf(s);
    nu[c] = nd[c];
  }
  float mx = nu[0];
  if (nu[1] > mx) mx = nu[1];
  if (nu[2] > mx) mx = nu[2];
  const float th_tmp = mx * kEps;
  const float threshold_helper = (th_tmp * th_tmp) / 5.0f;
  const float norm_downdate_threshold = sqrtf(kEps);

  int nzp = 3;
  int trans[3];
  float hc[3];

#pragma unroll
  for (int k = 0; k < 3; ++k) {
    // biggest remaining column norm, first maximum wins (Eigen maxCoeff)
    int big = k;
    float bv = nu[k];
#pragma unroll
    for (int j = k + 1; j < 3; ++j)
      if (nu[j] > bv) {
        bv = nu[j];
        big = j;
      }
    const float big_sq = bv * bv;
    if (nzp == 3 && big_sq < threshold_helper * (float)(5 - k)) nzp = k;
    trans[k] = big;
    if (k == 0) {
      cond_swap_cols<0, 1>(a, nu, nd, big == 1);
      cond_swap_cols<0, 2>(a, nu, nd, big == 2);
    } else if (k == 1) {
      cond_swap_cols<1, 2>(a, nu, nd, big == 2);
    }

    // makeHouseholderInPlace on a[k][k..4]
    float tail_sq = 0.0f;
#pragma unroll
    for (int r = k + 1; r < 5; ++r) tail_sq = (r == k + 1) ? a[k][r] * a[k][r] : tail_sq + a[k][r] * a[k][r];
    const float c0 = a[k][k];
    float tau, beta;
    if (tail_sq <= kTiny) {
      tau = 0.0f;
      beta = c0;
#pragma unroll
      for (int r = k + 1; r < 5; ++r) a[k][r] = 0.0f;
    } else {
      beta = sqrtf(c0 * c0 + tail_sq);
      if (c0 >= 0.0f) beta = -beta;
      const float den = c0 - beta;
#pragma unroll
      for (int r = k + 1; r < 5; ++r) a[k][r] = a[k][r] / den;
      tau = (beta - c0) / beta;
    }
    a[k][k] = beta;
    hc[k] = tau;

    // applyHouseholderOnTheLeft to the trailing columns
    if (tau != 0.0f) {
#pragma unroll
      for (int j = k + 1; j < 3; ++j) {
        float t = 0.0f;
#pragma unroll
        for (int r = k + 1; r < 5; ++r) t = (r == k + 1) ? a[k][r] * a[j][r] : t + a[k][r] * a[j][r];
        t = t + a[j][k];
        a[j][k] = a[j][k] - tau * t;
#pragma unroll
        for (int r = k + 1; r < 5; ++r) a[j][r] = a[j][r] - (tau * a[k][r]) * t;
      }
    }

    // column-norm downdate (LAPACK lawn176)
#pragma unroll
    for (int j = k + 1; j < 3; ++j) {
      if (nu[j] != 0.0f) {
        float temp = fabsf(a[j][k]) / nu[j];
        temp = (1.0f + temp) * (1.0f - temp);
        temp = temp < 0.0f ? 0.0f : temp;
        const float q = nu[j] / nd[j];
        const float temp2 = temp * (q * q);
        if (temp2 <= norm_downdate_threshold) {
          float s = 0.0f;
#pragma unroll
          for (int r = k + 1; r < 5; ++r) s = (r == k + 1) ? a[j][r] * a[j][r] : s + a[j][r] * a[j][r];
          nd[j] = sqrtf(s);
          nu[j] = nd[j];
        } else {
          nu[j] = nu[j] * sqrtf(temp);
        }
      }
    }
  }

  // column permutation from the transpositions
  int perm[3] = {0, 1, 2};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int t = trans[k];
    int pk = perm[k];
    int pt = (t == 0) ? perm[0] : (t == 1) ? perm[1] : perm[2];
    // swap perm[k] <-> perm[t]
#pragma unroll
    for (int q = 0; q < 3; ++q)
      if (q == t) perm[q] = pk;
    perm[k] = pt;
  }

  sol[0] = sol[1] = sol[2] = 0.0f;
  if (nzp > 0) {
    float c[5] = {-1.0f, -1.0f, -1.0f, -1.0f, -1.0f};
    // c = Q^T c : H_0 first
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      if (k < nzp && hc[k] != 0.0f) {
        const float tau = hc[k];
        float t = 0.0f;
#pragma unroll
        for (int r = k + 1; r < 5; ++r) t = (r == k + 1) ? a[k][r] * c[r] : t + a[k][r] * c[r];
        t = t + c[k];
        c[k] = c[k] - tau * t;
#pragma unroll
        for (int r = k + 1; r < 5; ++r) c[r] = c[r] - (tau * a[k][r]) * t;
      }
    }
    // upper-triangular back substitution on the leading nzp rows
#pragma unroll
    for (int i = 2; i >= 0; --i) {
      if (i < nzp && c[i] != 0.0f) {
        c[i] = c[i] / a[i][i];
#pragma unroll
        for (int r = 0; r < i; ++r) c[r] = c[r] - c[i] * a[i][r];
      }
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      if (i < nzp) {
        const int p = perm[i];
        sol[0] = (p == 0) ? c[i] : sol[0];
        sol[1] = (p == 1) ? c[i] : sol[1];
        sol[2] = (p == 2) ? c[i] : sol[2];
      }
    }
  }

}

__device__ __forceinline__ bool esti_plane_dev(const float (&nb)[5][3],
                                               float threshold, float (&abcd)[4]) {
  float sol[3];
  qr_solve_m1_dev(nb, sol);
  const float n = sqrtf((sol[0] * sol[0] + sol[1] * sol[1]) + sol[2] * sol[2]);
  abcd[0] = sol[0] / n;
  abcd[1] = sol[1] / n;
  abcd[2] = sol[2] / n;
  abcd[3] = (float)(1.0 / (double)n);
  bool ok = true;
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const float r = ((abcd[0] * nb[j][0] + abcd[1] * nb[j][1]) + abcd[2] * nb[j][2]) + abcd[3];
    if (fabsf(r) > threshold) ok = false;
  }
  return ok;
}

}  // namespace slio
