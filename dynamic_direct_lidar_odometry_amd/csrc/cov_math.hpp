// cov_math.hpp — per-point covariance math of calculate_covariances
// (reference include/nano_gicp/impl/nano_gicp_impl.hpp:392-437): the
// symmetric 3x3 eigen-decomposition behind the JacobiSVD regularisations,
// the 3x3 inverse of FROBENIUS, and the five regularisation methods.
#pragma once
#include <hip/hip_runtime.h>

namespace ddlo {

// ============================================================================
// small fp64 linear algebra (per lane)
// ============================================================================
// Symmetric 3x3 cyclic Jacobi eigen-decomposition: lam[j], V[j][i] = v_j[i].
// The whole 3x3 is rotated in place (its two triangles may drift apart by an
// ulp), operation for operation as oracle/cpu_ref.cpp sym_eig3: the
// regularised covariance of a (near-)isotropic neighbourhood depends on the
// last bit of the rotations, so device and oracle must share the sequence.
__device__ inline void sym_eig3(const double A[9], double lam[3], double V[3][3]) {
  double a[3][3] = {{A[0], A[1], A[2]}, {A[3], A[4], A[5]}, {A[6], A[7], A[8]}};
  double v[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
  for (int sweep = 0; sweep < 50; ++sweep) {
    const double off = fabs(a[0][1]) + fabs(a[0][2]) + fabs(a[1][2]);
    const double scale = fabs(a[0][0]) + fabs(a[1][1]) + fabs(a[2][2]);
    if (off <= 1e-300 || off <= scale * 1e-18) break;
#pragma unroll
    for (int pq = 0; pq < 3; ++pq) {
      const int p = pq == 2 ? 1 : 0;
      const int q = pq == 0 ? 1 : 2;
      const double apq = a[p][q];
      if (apq == 0.0) continue;
      const double theta = (a[q][q] - a[p][p]) / (2.0 * apq);
      const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
      const double c = 1.0 / sqrt(t * t + 1.0);
      const double s = t * c;
#pragma unroll
      for (int k = 0; k < 3; ++k) {   // A <- J^T A J
        const double akp = a[k][p], akq = a[k][q];
        a[k][p] = c * akp - s * akq;
        a[k][q] = s * akp + c * akq;
      }
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const double apk = a[p][k], aqk = a[q][k];
        a[p][k] = c * apk - s * aqk;
        a[q][k] = s * apk + c * aqk;
      }
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const double vkp = v[k][p], vkq = v[k][q];
        v[k][p] = c * vkp - s * vkq;
        v[k][q] = s * vkp + c * vkq;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    lam[j] = a[j][j];
#pragma unroll
    for (int i = 0; i < 3; ++i) V[j][i] = v[i][j];
  }
}

// 3x3 inverse by adjugate (general, row-major)
__device__ __forceinline__ void inv3(const double m[9], double r[9]) {
  const double c00 = m[4] * m[8] - m[5] * m[7];
  const double c01 = m[5] * m[6] - m[3] * m[8];
  const double c02 = m[3] * m[7] - m[4] * m[6];
  const double det = m[0] * c00 + m[1] * c01 + m[2] * c02;
  const double id = 1.0 / det;
  r[0] = c00 * id;
  r[1] = (m[2] * m[7] - m[1] * m[8]) * id;
  r[2] = (m[1] * m[5] - m[2] * m[4]) * id;
  r[3] = c01 * id;
  r[4] = (m[0] * m[8] - m[2] * m[6]) * id;
  r[5] = (m[2] * m[3] - m[0] * m[5]) * id;
  r[6] = c02 * id;
  r[7] = (m[1] * m[6] - m[0] * m[7]) * id;
  r[8] = (m[0] * m[4] - m[1] * m[3]) * id;
}

// regularisation of a covariance (nano_gicp_impl.hpp:401-437)
__device__ inline void regularize(const double C[9], int method, double out[6]) {
  double R[9];
  if (method == 0) {  // NONE
    for (int i = 0; i < 9; ++i) R[i] = C[i];
  } else if (method == 4) {  // FROBENIUS: ((C + 1e-3 I)^-1 / ||.||_F)^-1
    double Cl[9], Ci[9];
    for (int i = 0; i < 9; ++i) Cl[i] = C[i] + ((i % 4 == 0) ? 1e-3 : 0.0);
    inv3(Cl, Ci);
    double nrm = 0;
    for (int i = 0; i < 9; ++i) nrm += Ci[i] * Ci[i];
    nrm = sqrt(nrm);
    for (int i = 0; i < 9; ++i) Ci[i] /= nrm;
    inv3(Ci, R);
  } else {  // JacobiSVD route: U diag(vals) V^T with U col = sign(lambda) V col
    double lam[3], V[3][3];
    sym_eig3(C, lam, V);
    // order by |lambda| descending (stable for equal values: index order)
    int o0 = 0, o1 = 1, o2 = 2;
    if (fabs(lam[o1]) > fabs(lam[o0])) { int t = o0; o0 = o1; o1 = t; }
    if (fabs(lam[o2]) > fabs(lam[o1])) {
      int t = o1; o1 = o2; o2 = t;
      if (fabs(lam[o1]) > fabs(lam[o0])) { t = o0; o0 = o1; o1 = t; }
    }
    const int ord[3] = {o0, o1, o2};
    double sv[3], vals[3];
    for (int i = 0; i < 3; ++i) sv[i] = fabs(lam[ord[i]]);
    if (method == 3) {  // PLANE
      vals[0] = 1; vals[1] = 1; vals[2] = 1e-3;
    } else if (method == 1) {  // MIN_EIG
      for (int i = 0; i < 3; ++i) vals[i] = fmax(sv[i], 1e-3);
    } else {  // NORMALIZED_MIN_EIG
      for (int i = 0; i < 3; ++i) vals[i] = fmax(sv[i] / sv[0], 1e-3);
    }
    for (int i = 0; i < 9; ++i) R[i] = 0.0;
    for (int j = 0; j < 3; ++j) {
      const int oj = ord[j];
      const double sgn = lam[oj] < 0 ? -1.0 : 1.0;
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) R[3 * r + c] += sgn * V[oj][r] * vals[j] * V[oj][c];
    }
  }
  out[0] = R[0]; out[1] = R[1]; out[2] = R[2];
  out[3] = R[4]; out[4] = R[5]; out[5] = R[8];
}


}  // namespace ddlo
