// pose.hip — batched pose-only bundle adjustment on MI355X (gfx950).
//
// TrackLocalMap::OptimizeCameraPose (Core/MAGESLAM/Source/Tracking/TrackLocalMap.cpp:421-501) builds
// a fresh BundlerLib with ArePointsFixed, one free camera and one observation per map point, and
// runs StepBundleAdjustment(numIterations x huberWidth, maxOutlierErrorSquared) — every tracked frame,
// twice (:96-121).  Through the general BA path each of those tiny problems costs a dozen launches and
// a host round trip per LM trial; here a whole batch of them is ONE launch: one 256-thread workgroup
// per problem runs g2o's complete StepBundleAdjustment on device:
//   per step   linearise at the current pose (errors, Huber, the 6x6 Hpp / bp of J_pose^T w J_pose)
//              with one workgroup reduction; lambda = 1e-5 max diag at iteration 0 (computeLambdaInit)
//   per trial  (<= 10, OptimizationAlgorithmLevenberg::solve) lane 0 factors Hpp + lambda I (6x6
//              Cholesky; on failure x keeps the previous solve, as LinearSolverDense leaves it), the
//              trial pose exp(x) * T, computeScale; one reduction evaluates the trial chi2; accept /
//              reject exactly as g2o (rho, alpha, ni); a failed solve() ends the step loop
//   post-pass  (BundlerLib.cpp:385-446) each edge's squared error from the LAST evaluated state (g2o
//              keeps _error of the last computeActiveErrors, i.e. the last trial, even when it was
//              rejected) and the cheirality test at the current pose; outlier flags, mean of the kept.
// Points are fixed (ArePointsFixed): no Schur complement, the reduced system is the camera block.
#include <hip/hip_runtime.h>

#include <cstring>

#include <cfloat>
#include <cmath>

// FMA contraction for this file's device arithmetic (the library is built with -ffp-contract=off):
// the pose-only problem is a chain of short dependent fp64 sequences (per-trial 6x6 solve, exp map)
// whose length halves when a*b+c is one instruction.  Parity with the oracle is by tolerance and
// identical decisions (outliers, iterations, trials), which the reduction order already requires.
#pragma clang fp contract(fast)
#include "ba_math.hpp"
#include "common.hpp"

namespace mage {
namespace {

using namespace ba;

// threads per problem: 256 for large batches (2 problems per CU); MAGE_POSE_FEW_THREADS when the
// batch cannot fill the chip (the tracker's per-frame single problem).  Every thread runs the
// per-trial solve and exp map itself, so two waves per SIMD issue that chain twice: one wave per
// SIMD (256) halves it and the reductions, while the edge passes are issue-bound either way.
#ifndef MAGE_POSE_FEW_THREADS
#define MAGE_POSE_FEW_THREADS 256
#endif
constexpr int PB_THREADS_BATCH = 256, PB_THREADS_FEW = MAGE_POSE_FEW_THREADS;
// observations of a problem staged in LDS (X, Y, Z, info | u, v) when it has at most this many:
// every edge pass then reads LDS instead of L2 (a lane's edges are read by that lane only)
constexpr int POSE_STAGE = 2048;

#ifndef MAGE_POSE_STAMPS
#define MAGE_POSE_STAMPS 0  // tools/pose_stamps.py: phase stamps (s_memtime) of problem 0, thread 0
#endif
#if MAGE_POSE_STAMPS
__device__ unsigned long long g_pose_st[256];
#define PST(id)                                                                                                 \
    do {                                                                                                        \
        if (blockIdx.x == 0 && threadIdx.x == 0 && nst < 254)                                                   \
            g_pose_st[nst++] = ((unsigned long long)(id) << 56) | (__builtin_amdgcn_s_memtime() & 0xFFFFFFFFFFFFFFull); \
    } while (0)
#else
#define PST(id) \
    do {        \
    } while (0)
#endif

struct PoseParams {
    const float* pos3;    // per problem: view-space t
    const float* r9;      // per problem: rotation, Eigen column-major
    const float* intr4;   // per problem: cx, cy, fx, fy
    const uint32_t* obs_start;  // problems + 1
    const float* points3;       // per observation: map point (fixed)
    const float* uv;            // per observation
    const float* info;          // per observation: information scalar
    uint32_t nsteps;
    double huber;
    double max_err_sq;
    float* pos3_out;
    float* r9_out;
    double* qt7_out;      // optional fp64 state
    uint8_t* outlier;     // per observation
    float* mean_sq;       // per problem
    uint32_t* stats;      // optional: per problem {iterations, trials}
};

// SetCameraPose: Eigen::Quaternionf{Matrix3f}.normalized() in float, then SE3Quat(q, t) in double
// (BundlerLib.cpp:269-273; the same arithmetic as mage_ba_set_cameras)
__device__ void pose_from_input(const float* r9, const float* t3, double q[4], double t[3])
{
#pragma clang fp contract(off)
    float m[9];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) m[r * 3 + c] = r9[c * 3 + r];
    float qf[4];
    const float tr = m[0] + m[4] + m[8];
    if (tr > 0.f) {
        float s = sqrtf(tr + 1.0f);
        qf[3] = 0.5f * s;
        s = 0.5f / s;
        qf[0] = (m[7] - m[5]) * s;
        qf[1] = (m[2] - m[6]) * s;
        qf[2] = (m[3] - m[1]) * s;
    } else {
        int a = 0;
        if (m[4] > m[0]) a = 1;
        if (m[8] > m[a * 4]) a = 2;
        const int j = (a + 1) % 3, k = (j + 1) % 3;
        float s = sqrtf(m[a * 4] - m[j * 4] - m[k * 4] + 1.0f);
        qf[a] = 0.5f * s;
        s = 0.5f / s;
        qf[3] = (m[k * 3 + j] - m[j * 3 + k]) * s;
        qf[j] = (m[j * 3 + a] + m[a * 3 + j]) * s;
        qf[k] = (m[k * 3 + a] + m[a * 3 + k]) * s;
    }
    const float nrm = sqrtf(qf[0] * qf[0] + qf[1] * qf[1] + qf[2] * qf[2] + qf[3] * qf[3]);
    for (int k = 0; k < 4; k++) q[k] = (double)(qf[k] / nrm);
    d_se3_normalize(q);
    for (int k = 0; k < 3; k++) t[k] = (double)t3[k];
}

// ---- the trial's exp map (SE3Quat::exp(x) * T, g2o se3quat.h; ba_math.hpp d_oplus) with the
// square roots and divisions of its dependent chain as v_rsq_f64 + two Newton steps (~1 ulp):
// every thread runs this chain once per trial, and its length (~130 dependent fp64 operations,
// ~3.3k cycles with the IEEE sequences) is part of every trial's critical path.
__device__ __forceinline__ double rsqrt_nr(double x)
{
    const double h = 0.5 * x;
    double r = __builtin_amdgcn_rsq(x);
    r *= __builtin_fma(-h * r, r, 1.5);
    r *= __builtin_fma(-h * r, r, 1.5);
    return r;
}

template <int I>
__device__ __forceinline__ void quat_from_matrix_diag(const double* m, double q[4])
{
    constexpr int J = (I + 1) % 3, K = (J + 1) % 3;
    const double u = m[I * 4] - m[J * 4] - m[K * 4] + 1.0, r = rsqrt_nr(u);
    q[I] = 0.5 * (u * r);
    const double h = 0.5 * r;
    q[3] = (m[K * 3 + J] - m[J * 3 + K]) * h;
    q[J] = (m[J * 3 + I] + m[I * 3 + J]) * h;
    q[K] = (m[K * 3 + I] + m[I * 3 + K]) * h;
}

// Eigen Quaterniond(Matrix3d) (d_quat_from_matrix), static indices only
__device__ __forceinline__ void pose_quat_from_matrix(const double* m, double q[4])
{
    const double t = m[0] + m[4] + m[8];
    if (t > 0) {
        const double u = t + 1.0, r = rsqrt_nr(u);
        q[3] = 0.5 * (u * r);
        const double h = 0.5 * r;
        q[0] = (m[7] - m[5]) * h;
        q[1] = (m[2] - m[6]) * h;
        q[2] = (m[3] - m[1]) * h;
    } else {
        int i = 0;
        if (m[4] > m[0]) i = 1;
        if (m[8] > (i ? m[4] : m[0])) i = 2;
        if (i == 0)
            quat_from_matrix_diag<0>(m, q);
        else if (i == 1)
            quat_from_matrix_diag<1>(m, q);
        else
            quat_from_matrix_diag<2>(m, q);
    }
}

__device__ __forceinline__ void pose_normalize(double q[4])
{
    if (q[3] < 0)
        for (int i = 0; i < 4; i++) q[i] = -q[i];
    const double r = rsqrt_nr(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    for (int i = 0; i < 4; i++) q[i] *= r;
}

// T <- exp(u) * T (VertexSE3Expmap::oplusImpl); the same expressions as d_oplus
__device__ __forceinline__ void pose_oplus(double q[4], double t[3], const double u[6])
{
    const double w0 = u[0], w1 = u[1], w2 = u[2];
    const double x = w0 * w0 + w1 * w1 + w2 * w2;
    const double rs = rsqrt_nr(x), theta = x * rs;  // 1 / theta, theta
    const double O[9] = {0, -w2, w1, w2, 0, -w0, -w1, w0, 0};
    double O2[9];
#pragma unroll
    for (int r = 0; r < 3; r++)
#pragma unroll
        for (int c = 0; c < 3; c++) O2[r * 3 + c] = O[r * 3] * O[c] + O[r * 3 + 1] * O[3 + c] + O[r * 3 + 2] * O[6 + c];
    double R[9], V[9];
    if (x == 0 || theta < 0.00001) {
#pragma unroll
        for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0 ? 1.0 : 0.0) + O[i] + O2[i];
#pragma unroll
        for (int i = 0; i < 9; i++) V[i] = R[i];
    } else {
        double sn, cs;
        sincos(theta, &sn, &cs);
        const double i2 = rs * rs;
        const double a = sn * rs, b = (1 - cs) * i2, c = (theta - sn) * (i2 * rs);
#pragma unroll
        for (int i = 0; i < 9; i++) {
            const double I = (i % 4 == 0 ? 1.0 : 0.0);
            R[i] = I + a * O[i] + b * O2[i];
            V[i] = I + b * O[i] + c * O2[i];
        }
    }
    double eq[4], et[3];
    pose_quat_from_matrix(R, eq);
#pragma unroll
    for (int r = 0; r < 3; r++) et[r] = V[r * 3] * u[3] + V[r * 3 + 1] * u[4] + V[r * 3 + 2] * u[5];
    pose_normalize(eq);
    double rt[3];
    d_qrot(eq, t, rt);
    double nq[4];
    nq[3] = eq[3] * q[3] - eq[0] * q[0] - eq[1] * q[1] - eq[2] * q[2];
    nq[0] = eq[3] * q[0] + eq[0] * q[3] + eq[1] * q[2] - eq[2] * q[1];
    nq[1] = eq[3] * q[1] + eq[1] * q[3] + eq[2] * q[0] - eq[0] * q[2];
    nq[2] = eq[3] * q[2] + eq[2] * q[3] + eq[0] * q[1] - eq[1] * q[0];
    pose_normalize(nq);
#pragma unroll
    for (int i = 0; i < 4; i++) q[i] = nq[i];
#pragma unroll
    for (int i = 0; i < 3; i++) t[i] = et[i] + rt[i];
}

struct EdgeIn {
    double X[3], u, v, info;
};

// Reprojection error, robust chi2 and the pose normal-equation terms of one edge, added into acc
// (21 upper Hpp entries, 6 bp, rho0 at 27); also the post-pass inputs: ss = |e|^2 and the depth
// (cheirality: (R X + t)_z > 0 is the reference's (X + R^T t) . R^T z > 0).  Branch-free (Huber by
// selects), so two edges' chains interleave; one reciprocal of the depth serves the projection and
// the Jacobian.  This file is compiled with FMA contraction (see the pragma above): the terms are
// w J^T J and J^T (-w e) with the weight folded into one Jacobian row first (g2o's JtWJ order is
// not reproduced anyway: the sums run in another order than the oracle's, parity is by tolerance +
// identical decisions); the products with the structural zeros J[0][4] and J[1][3] are skipped
// (exact: every other operand is finite).
__device__ __forceinline__ void edge_terms(const EdgeIn& e, const double q[4], const double t[3], double f, double cx,
                                           double cy, double huber, double& ss, double& z, double (&acc)[32])
{
    double xc[3];
    d_qrot(q, e.X, xc);
    xc[0] += t[0];
    xc[1] += t[1];
    xc[2] += t[2];
    z = xc[2];
    const double iz = 1.0 / xc[2];
    const double xi = xc[0] * iz, yi = xc[1] * iz, fi = f * iz;
    const double ev0 = e.u - (xi * f + cx), ev1 = e.v - (yi * f + cy);
    ss = ev0 * ev0 + ev1 * ev1;
    const double chi2 = e.info * ss;
    // RobustKernelHuber; 1 / sqrt(chi2) by v_rsq_f64 + two Newton steps (only the outlier side
    // uses it: sqrt = chi2 / sqrt, rho1 = delta / sqrt) instead of an fp64 sqrt and a division
    const double dsqr = huber * huber, hc = 0.5 * chi2;
    double rs = __builtin_amdgcn_rsq(chi2);
    rs *= __builtin_fma(-hc * rs, rs, 1.5);
    rs *= __builtin_fma(-hc * rs, rs, 1.5);
    const bool in = chi2 <= dsqr;
    acc[27] += in ? chi2 : 2 * (chi2 * rs) * huber - dsqr;
    const double rho1 = in ? 1.0 : huber * rs;
    double Jp[12];
    jac_pose_q(xi, yi, fi, f, Jp);
    const double w = rho1 * e.info;
    const double or0 = -e.info * ev0 * rho1, or1 = -e.info * ev1 * rho1;
    double wj[12];
#pragma unroll
    for (int k = 0; k < 12; k++) wj[k] = Jp[k] * w;
#pragma unroll
    for (int r = 0; r < 6; r++)
#pragma unroll
        for (int c = r; c < 6; c++) {
            double& h = acc[r * 6 - r * (r - 1) / 2 + c - r];
            if (r != 4 && c != 4) h = __builtin_fma(wj[r], Jp[c], h);
            if (r != 3 && c != 3) h = __builtin_fma(wj[6 + r], Jp[6 + c], h);
        }
#pragma unroll
    for (int r = 0; r < 6; r++) {
        double& b = acc[21 + r];
        if (r != 4) b = __builtin_fma(Jp[r], or0, b);
        if (r != 3) b = __builtin_fma(Jp[6 + r], or1, b);
    }
}

// 64-bit lane exchanges for the butterfly below (all VALU: no LDS round trip per round)
template <int CTRL, int BANKS>
__device__ __forceinline__ double dpp_f64(double old, double v)
{
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v), o = __builtin_bit_cast(unsigned long long, old);
    const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp((int)(unsigned)o, (int)(unsigned)u, CTRL, 0xF, BANKS, false);
    const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp((int)(unsigned)(o >> 32), (int)(unsigned)(u >> 32), CTRL, 0xF,
                                                              BANKS, false);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
// (a, b) -> lanes l < H of each 2H-lane group: a(l) + a(l ^ H); lanes with bit H: b(l ^ H) + b(l)
// for H = 32 / 16 by v_permlane32_swap / v_permlane16_swap
template <int H>
__device__ __forceinline__ double xsum_swap(double a, double b)
{
    const unsigned long long ua = __builtin_bit_cast(unsigned long long, a), ub = __builtin_bit_cast(unsigned long long, b);
    unsigned a0, a1, b0, b1;
    if constexpr (H == 32) {
        const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)ua, (unsigned)ub, false, false);
        const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(ua >> 32), (unsigned)(ub >> 32), false, false);
        a0 = lo[0], b0 = lo[1], a1 = hi[0], b1 = hi[1];
    } else {
        const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)ua, (unsigned)ub, false, false);
        const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(ua >> 32), (unsigned)(ub >> 32), false, false);
        a0 = lo[0], b0 = lo[1], a1 = hi[0], b1 = hi[1];
    }
    return __builtin_bit_cast(double, ((unsigned long long)a1 << 32) | a0) +
           __builtin_bit_cast(double, ((unsigned long long)b1 << 32) | b0);
}

// fixed-order workgroup sum of acc[0..N) into out[0..N) (all threads read out afterwards).
// N > 4: butterfly reduce-scatter inside the wave (each round halves the values a lane holds:
// 16 + 8 + 4 + 2 + 1 + 1 exchanges instead of 6 per value; lane 2i ends with value i) on VALU
// lane exchanges — v_permlane32_swap / v_permlane16_swap for the 32- and 16-lane rounds (the swap
// itself pairs the kept and the sent value: no selects), DPP row_ror:8, row_shl/shr:4 by bank,
// quad_perm for the rest — then the per-wave partials in LDS
template <int PB_THREADS, int N>
__device__ __forceinline__ void wg_sum(double (&acc)[N], double (*red)[N], double* out)
{
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if constexpr (N > 4) {
        static_assert(N <= 32, "wg_sum: at most 32 values");
        double v[32];
#pragma unroll
        for (int k = 0; k < 32; k++) v[k] = k < N ? acc[k] : 0.0;
#pragma unroll
        for (int j = 0; j < 16; j++) v[j] = xsum_swap<32>(v[j], v[j + 16]);  // lane bit 5 -> value bit 4
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = xsum_swap<16>(v[j], v[j + 8]);  // lane bit 4 -> value bit 3
        {
            const bool up = (lane & 8) != 0;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const double send = up ? v[j] : v[j + 4], keep = up ? v[j + 4] : v[j];
                v[j] = keep + dpp_f64<0x128, 0xF>(0.0, send);  // row_ror:8 = lane ^ 8
            }
        }
        {
            const bool up = (lane & 4) != 0;
#pragma unroll
            for (int j = 0; j < 2; j++) {
                const double send = up ? v[j] : v[j + 2], keep = up ? v[j + 2] : v[j];
                // lane ^ 4: banks 0 / 2 read lane + 4 (row_shl:4), banks 1 / 3 lane - 4 (row_shr:4)
                const double x = dpp_f64<0x104, 0x5>(dpp_f64<0x114, 0xA>(0.0, send), send);
                v[j] = keep + x;
            }
        }
        {
            const bool up = (lane & 2) != 0;
            const double send = up ? v[0] : v[1], keep = up ? v[1] : v[0];
            v[0] = keep + dpp_f64<0x4E, 0xF>(0.0, send);  // quad_perm [2, 3, 0, 1] = lane ^ 2
        }
        const double s = v[0] + dpp_f64<0xB1, 0xF>(0.0, v[0]);  // quad_perm [1, 0, 3, 2] = lane ^ 1
        // value index of lane l: bits 5, 4, 3, 2, 1 of l -> bits 4, 3, 2, 1, 0
        if (!(lane & 1) && (lane >> 1) < N) red[wave][lane >> 1] = s;
    } else {
#pragma unroll
        for (int k = 0; k < N; k++) {
            double v = acc[k];
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
            if (lane == 0) red[wave][k] = v;
        }
    }
    __syncthreads();
    if (threadIdx.x < N) {
        double v = 0;
        for (int w = 0; w < PB_THREADS / kWave; w++) v += red[w][threadIdx.x];
        out[threadIdx.x] = v;
    }
    __syncthreads();
}

// The 6x6 solve of one trial, computed by every thread from the reduced system (no broadcast, no
// barrier): S = Hpp + lambda I, Cholesky (LLT) and the two triangular solves; on a non-positive
// pivot x keeps the previous solve (LinearSolverDense) and the trial is marked failed.  The
// diagonal of L is never stored: the factor and the solves use 1/L_jj only.
__device__ __forceinline__ bool pose_solve(const double* sum, double lam, double x[6])
{
    double L[36];
#pragma unroll
    for (int r = 0, k = 0; r < 6; r++)
#pragma unroll
        for (int c = r; c < 6; c++, k++) {
            L[r * 6 + c] = sum[k];
            L[c * 6 + r] = sum[k];
        }
#pragma unroll
    for (int r = 0; r < 6; r++) L[r * 6 + r] += lam;
    // fully unrolled (static register indexing, no scratch); a non-positive pivot only clears ok —
    // the rest of the factor is then unused, as after the oracle's break
    // 1/sqrt(d) by v_rsq_f64 + one Newton step (~1e-14 relative, as chol_tiles): the factor's
    // and the solves' divisions become multiplications, off the dependent f64 division sequence
    bool ok = true;
    double rinv[6];
#pragma unroll
    for (int j = 0; j < 6; j++) {
        double d = L[j * 6 + j];
#pragma unroll
        for (int k = 0; k < j; k++) d -= L[j * 6 + k] * L[j * 6 + k];
        ok = ok && d > 0;
        const double h = 0.5 * d;
        double r = __builtin_amdgcn_rsq(d);
        r *= __builtin_fma(-h * r, r, 1.5);
        rinv[j] = r;
#pragma unroll
        for (int i = j + 1; i < 6; i++) {
            double s = L[i * 6 + j];
#pragma unroll
            for (int k = 0; k < j; k++) s -= L[i * 6 + k] * L[j * 6 + k];
            L[i * 6 + j] = s * r;
        }
    }
    if (ok) {
        double y[6];
#pragma unroll
        for (int i = 0; i < 6; i++) {
            double s = sum[21 + i];
#pragma unroll
            for (int k = 0; k < i; k++) s -= L[i * 6 + k] * y[k];
            y[i] = s * rinv[i];
        }
#pragma unroll
        for (int i = 5; i >= 0; i--) {
            double s = y[i];
#pragma unroll
            for (int k = i + 1; k < 6; k++) s -= L[k * 6 + i] * y[k];
            y[i] = s * rinv[i];
        }
#pragma unroll
        for (int k = 0; k < 6; k++) x[k] = y[k];
    }
    return ok;
}

// One workgroup per problem.  Every thread keeps the LM state (pose, lambda, ni, the last solve)
// in registers and computes each trial's solve itself from the reduced system in LDS, so the only
// barriers are the reductions'.  The trial evaluation also accumulates the normal equations at the
// trial pose: when the trial is accepted they are the next step's linearisation (g2o linearises
// at the accepted state), so after step 0 a step costs one edge pass per trial.
//
// Post-pass folded into the edge passes (staged problems): BundlerLib's outlier pass reads each
// edge's error from the LAST evaluated state and the cheirality at the CURRENT pose, which is the
// last trial's pose if it was accepted, else the pose the current state was evaluated at.  Each
// pass therefore keeps per lane, for its edges, a bit "error above maxErrorSquare" and a bit
// "in front of the camera", and reduces the kept-edge sums (sum of ss, count) for both outcomes
// (slots 28-31 of the 32-value reduction, which the butterfly carries for free); after the loop
// the bits of the current pose give the outlier flags without another pass over the edges.
template <int PB_THREADS>
__global__ __launch_bounds__(PB_THREADS) void pose_ba_kernel(PoseParams p)
{
    __shared__ double red[PB_THREADS / kWave][32];
    __shared__ double sums[2][32];  // the linearisation at the current pose / at the trial pose
    // LM state: written by every thread with the same value (each thread computes it), so a
    // thread's reads follow its own writes and no barrier is needed; in LDS rather than registers
    // to keep them out of the edge loops' register budget
    __shared__ double s_cur[7], s_ev[7], s_x[6];  // current pose (q, t), last evaluated pose, last solve
    __shared__ float4 s_e0[POSE_STAGE];           // staged observations: X, Y, Z, info
    __shared__ float2 s_e1[POSE_STAGE];           // u, v
    const int pr = blockIdx.x, tid = threadIdx.x;
    [[maybe_unused]] int nst = 0;
    PST(0);
    const uint32_t e0 = p.obs_start[pr], e1 = p.obs_start[pr + 1];
    const int E = (int)(e1 - e0);
    const double f = p.intr4[4 * pr + 2], cx = p.intr4[4 * pr], cy = p.intr4[4 * pr + 1];
    // a lane's edges are observations tid + k PB_THREADS; staged (and post-pass bits) up to 32 per lane
    const bool staged = E <= POSE_STAGE && E <= 32 * PB_THREADS;
    // every load of the lane's edges in flight before the first LDS write (a loop of load ->
    // write pairs waited out one L2 round trip per edge), and before the initial pose
    constexpr int KS = POSE_STAGE / PB_THREADS;
    float4 ga[KS];
    float2 gb[KS];
    if (staged) {
#pragma unroll
        for (int k = 0; k < KS; k++) {
            const int i = tid + k * PB_THREADS;
            if (i < E) {
                const uint32_t g = e0 + i;
                ga[k] = make_float4(p.points3[3 * g], p.points3[3 * g + 1], p.points3[3 * g + 2], p.info[g]);
                gb[k] = make_float2(p.uv[2 * g], p.uv[2 * g + 1]);
            }
        }
    }
    {
        double q[4], t[3];
        pose_from_input(p.r9 + 9 * pr, p.pos3 + 3 * pr, q, t);
        for (int k = 0; k < 4; k++) s_cur[k] = q[k];
        for (int k = 0; k < 3; k++) s_cur[4 + k] = t[k];
        for (int k = 0; k < 6; k++) s_x[k] = 0;
    }
    if (staged) {
#pragma unroll
        for (int k = 0; k < KS; k++) {
            const int i = tid + k * PB_THREADS;
            if (i < E) {  // read back by the same thread: no barrier
                s_e0[i] = ga[k];
                s_e1[i] = gb[k];
            }
        }
    }
    PST(1);
    bool have_eval = false;
    double lambda = 0, ni = 2;
    const double maxe = p.max_err_sq;
    auto load_edge = [&](int i) {
        EdgeIn e;
        if (staged) {
            const float4 a = s_e0[i];
            const float2 b = s_e1[i];
            e.X[0] = a.x;
            e.X[1] = a.y;
            e.X[2] = a.z;
            e.info = a.w;
            e.u = b.x;
            e.v = b.y;
        } else {
            const uint32_t g = e0 + i;
            e.X[0] = p.points3[3 * g];
            e.X[1] = p.points3[3 * g + 1];
            e.X[2] = p.points3[3 * g + 2];
            e.u = p.uv[2 * g];
            e.v = p.uv[2 * g + 1];
            e.info = p.info[g];
        }
        return e;
    };
    // post-pass bits of the lane's edges: big (ss > maxErrorSquare) of the last pass, front (depth
    // > 0) of the last pass, and front at the current pose
    uint32_t big = 0, front = 0, front_cur = 0;
    // errors, robust chi2 and normal equations of every edge at pose qt = (q, t) -> sums[slot];
    // two edges per iteration (independent chains interleave)
    auto linearise = [&](const double* qt, int slot) {
        const double q[4] = {qt[0], qt[1], qt[2], qt[3]}, t[3] = {qt[4], qt[5], qt[6]};
        double acc[32];
#pragma unroll
        for (int k = 0; k < 32; k++) acc[k] = 0;
        uint32_t nb = 0, nf = 0, bit = 1;
        auto post = [&](double ss, double z) {
            const bool bg = ss > maxe, fr = z > 0;
            nb |= bg ? bit : 0u;
            nf |= fr ? bit : 0u;
            const bool keep_acc = fr && !bg, keep_rej = (front_cur & bit) && !bg;  // trial accepted / rejected
            acc[28] += keep_acc ? ss : 0.0;
            acc[29] += keep_acc ? 1.0 : 0.0;
            acc[30] += keep_rej ? ss : 0.0;
            acc[31] += keep_rej ? 1.0 : 0.0;
            bit <<= 1;
        };
        int i = tid;
        for (; i + PB_THREADS < E; i += 2 * PB_THREADS) {
            const EdgeIn a = load_edge(i), b = load_edge(i + PB_THREADS);
            double ssa, za, ssb, zb;
            edge_terms(a, q, t, f, cx, cy, p.huber, ssa, za, acc);
            edge_terms(b, q, t, f, cx, cy, p.huber, ssb, zb, acc);
            post(ssa, za);
            post(ssb, zb);
        }
        if (i < E) {
            double ss, z;
            edge_terms(load_edge(i), q, t, f, cx, cy, p.huber, ss, z, acc);
            post(ss, z);
        }
        big = nb;
        front = nf;
        PST(2);
        wg_sum<PB_THREADS, 32>(acc, red, sums[slot]);
        PST(3);
    };
    uint32_t iters = 0, trials = 0;
    int cur = 0;                // sums[cur]: the linearisation at the current pose
    int last = 0;               // sums[last]: the last pass's sums
    bool last_accepted = true;  // the last pass's pose is the current one
    // StepOptimizer::Step: no active vertex (no observations) -> useless, every Step fails
    for (uint32_t step = 0; E > 0 && step < p.nsteps; step++) {
        if (step == 0) {
            linearise(s_cur, cur);
            front_cur = front;
            double m = 0;
            for (int r = 0, k = 0; r < 6; k += 6 - r, r++) m = fmax(fabs(sums[cur][k]), m);
            lambda = 1e-5 * m;  // computeLambdaInit, tau 1e-5 (fresh BundlerLib: no user lambda)
            ni = 2;
        }
        double currentChi = sums[cur][27];
        double rho = 0;
        int qmax = 0;
        do {
            const double* S = sums[cur];
            double scale;
            bool ok;
            {
                double x[6];
                for (int k = 0; k < 6; k++) x[k] = s_x[k];
                ok = pose_solve(S, lambda, x);
                PST(9);
                double tq[4] = {s_cur[0], s_cur[1], s_cur[2], s_cur[3]}, tt[3] = {s_cur[4], s_cur[5], s_cur[6]};
                pose_oplus(tq, tt, x);
                for (int k = 0; k < 4; k++) s_ev[k] = tq[k];
                for (int k = 0; k < 3; k++) s_ev[4 + k] = tt[k];
                for (int k = 0; k < 6; k++) s_x[k] = x[k];
                double sc = 0;
                for (int k = 0; k < 6; k++) sc += x[k] * (lambda * x[k] + S[21 + k]);
                scale = sc + 1e-3;
            }
            PST(4);
            have_eval = true;
            linearise(s_ev, cur ^ 1);
            last = cur ^ 1;
            double tempChi = sums[cur ^ 1][27];
            if (!ok) tempChi = DBL_MAX;
            rho = (currentChi - tempChi) / scale;
            trials++;
            const bool accept = rho > 0 && isfinite(tempChi);
            last_accepted = accept;
            if (accept) {
                const double r3 = 2 * rho - 1;
                double alpha = 1. - r3 * r3 * r3;  // g2o: 1 - pow(2 rho - 1, 3)
                alpha = fmin(alpha, 2. / 3.);
                const double scaleFactor = fmax(1. / 3., alpha);
                lambda *= scaleFactor;
                ni = 2;
                for (int k = 0; k < 7; k++) s_cur[k] = s_ev[k];
                currentChi = tempChi;
                cur ^= 1;  // the trial's normal equations are the next step's linearisation
                front_cur = front;
            } else {
                lambda *= ni;
                ni *= 2;
            }
            qmax++;
            PST(5);
        } while (rho < 0 && qmax < 10);
        iters++;
        const bool ok = !(qmax == 10 || rho == 0 || !isfinite(lambda));
        if (!ok) break;
    }
    double cur_q[4] = {s_cur[0], s_cur[1], s_cur[2], s_cur[3]}, cur_t[3] = {s_cur[4], s_cur[5], s_cur[6]};
    double mean_num, mean_den;
    if (have_eval && staged) {
        // post-pass from the last pass's bits and sums (see above)
        uint32_t bit = 1;
        for (int i = tid; i < E; i += PB_THREADS, bit <<= 1)
            p.outlier[e0 + i] = ((front_cur & bit) && !(big & bit)) ? 0 : 1;
        mean_num = sums[last][last_accepted ? 28 : 30];
        mean_den = sums[last][last_accepted ? 29 : 31];
        PST(6);
    } else {
        // post-pass over the edges: errors of the last evaluated state (none: zero errors),
        // cheirality at the current pose
        double ev_q[4] = {s_ev[0], s_ev[1], s_ev[2], s_ev[3]}, ev_t[3] = {s_ev[4], s_ev[5], s_ev[6]};
        double qc[4] = {-cur_q[0], -cur_q[1], -cur_q[2], cur_q[3]};
        double it[3], fwd[3];
        d_qrot(qc, cur_t, it);
        const double zc[3] = {0, 0, 1};
        d_qrot(qc, zc, fwd);
        double acc2[2] = {0, 0};
        for (int i = tid; i < E; i += PB_THREADS) {
            const EdgeIn e = load_edge(i);
            double ss = 0, z, unused[32] = {};
            if (have_eval) edge_terms(e, ev_q, ev_t, f, cx, cy, p.huber, ss, z, unused);
            const double dot = (e.X[0] + it[0]) * fwd[0] + (e.X[1] + it[1]) * fwd[1] + (e.X[2] + it[2]) * fwd[2];
            const bool out = dot <= 0 || ss > maxe;
            p.outlier[e0 + i] = out ? 1 : 0;
            if (!out) {
                acc2[0] += ss;
                acc2[1] += 1;
            }
        }
        PST(6);
        wg_sum<PB_THREADS, 2>(acc2, reinterpret_cast<double(*)[2]>(red), sums[0]);
        mean_num = sums[0][0];
        mean_den = sums[0][1];
    }
    PST(7);
    if (tid == 0) {
        p.mean_sq[pr] = (float)(mean_num / mean_den);
        // GetPose (BundlerLib.cpp:457-465): t as float, R of the normalised quaternion as float
        double q[4] = {cur_q[0], cur_q[1], cur_q[2], cur_q[3]};
        const double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
        for (int k = 0; k < 4; k++) q[k] /= n;
        double R[9];
        d_qmat(q, R);
        for (int k = 0; k < 3; k++) p.pos3_out[3 * pr + k] = (float)cur_t[k];
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) p.r9_out[9 * pr + c * 3 + r] = (float)R[r * 3 + c];
        if (p.qt7_out) {
            for (int k = 0; k < 4; k++) p.qt7_out[7 * pr + k] = cur_q[k];
            for (int k = 0; k < 3; k++) p.qt7_out[7 * pr + 4 + k] = cur_t[k];
        }
        if (p.stats) {
            p.stats[2 * pr] = iters;
            p.stats[2 * pr + 1] = trials;
        }
    }
#if MAGE_POSE_STAMPS
    PST(8);
    if (blockIdx.x == 0 && threadIdx.x == 0) g_pose_st[255] = (unsigned long long)nst;
#endif
}

mage_status pose_launch(const PoseParams& p, uint32_t problems, hipStream_t st)
{
    if (problems == 0) return MAGE_OK;
    if (problems >= 512)
        launch("ba.pose_batch", pose_ba_kernel<PB_THREADS_BATCH>, dim3(problems), dim3(PB_THREADS_BATCH), 0, st, p);
    else
        launch("ba.pose_batch", pose_ba_kernel<PB_THREADS_FEW>, dim3(problems), dim3(PB_THREADS_FEW), 0, st, p);
    MAGE_HIP(hipGetLastError());
    return MAGE_OK;
}

}  // namespace
}  // namespace mage

extern "C" {

mage_status mage_ba_pose_batch_device(uint32_t problems, const float* d_pos3, const float* d_r9, const float* d_intr4,
                                      const uint32_t* d_obs_start, const float* d_points3, const float* d_uv,
                                      const float* d_info, uint32_t nsteps, float huber, float max_error_square,
                                      float* d_pos3_out, float* d_r9_out, double* d_qt7_out, uint8_t* d_outlier,
                                      float* d_mean_sq, uint32_t* d_stats, mage_stream stream)
{
    using namespace mage;
    if (problems == 0) return MAGE_OK;
    MAGE_REQUIRE(d_pos3 && d_r9 && d_intr4 && d_obs_start && d_points3 && d_uv && d_info && d_pos3_out && d_r9_out &&
                     d_outlier && d_mean_sq,
                 MAGE_EINVAL, "null buffer");
    MAGE_REQUIRE(huber >= 0.f, MAGE_EINVAL, "Huber widths must be nonnegative");
    PoseParams p{d_pos3, d_r9, d_intr4, d_obs_start, d_points3, d_uv, d_info, nsteps, (double)huber,
                 (double)max_error_square, d_pos3_out, d_r9_out, d_qt7_out, d_outlier, d_mean_sq, d_stats};
    return pose_launch(p, problems, (hipStream_t)stream);
}

mage_status mage_ba_pose_batch(uint32_t problems, const float* pos3, const float* r9, const float* intr4,
                               const uint32_t* obs_start, const float* points3, const float* uv, const float* info,
                               uint32_t nsteps, float huber, float max_error_square, float* pos3_out, float* r9_out,
                               double* qt7_out, uint8_t* outlier, float* mean_sq, uint32_t* stats, int device)
{
    using namespace mage;
    if (problems == 0) return MAGE_OK;
    MAGE_REQUIRE(pos3 && r9 && intr4 && obs_start && pos3_out && r9_out && mean_sq, MAGE_EINVAL, "null argument");
    MAGE_REQUIRE(obs_start[0] == 0, MAGE_EINVAL, "obs_start[0] must be 0");
    for (uint32_t k = 0; k < problems; k++)
        MAGE_REQUIRE(obs_start[k + 1] >= obs_start[k], MAGE_EINVAL, "obs_start must be non-decreasing");
    const uint32_t E = obs_start[problems];
    MAGE_REQUIRE(E == 0 || (points3 && uv && info && outlier), MAGE_EINVAL, "null observation arrays");
    MAGE_REQUIRE(huber >= 0.f, MAGE_EINVAL, "Huber widths must be nonnegative");
    mage_status r = bind_device(device);
    if (r != MAGE_OK) return r;
    HostScratch* sp = host_scratch(device, SCRATCH_POSE);
    if (!sp) return MAGE_EDEVICE;
    HostScratch& S = *sp;
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    const size_t P = problems;
    const size_t o_pos = 0, o_r9 = al(o_pos + 12 * P), o_in = al(o_r9 + 36 * P), o_os = al(o_in + 16 * P),
                 o_pt = al(o_os + 4 * (P + 1)), o_uv = al(o_pt + 12ull * E), o_inf = al(o_uv + 8ull * E),
                 o_pos2 = al(o_inf + 4ull * E), o_r92 = al(o_pos2 + 12 * P), o_qt = al(o_r92 + 36 * P),
                 o_out = al(o_qt + 56 * P), o_ms = al(o_out + E + 1), o_st = al(o_ms + 4 * P), total = o_st + 8 * P;
    if ((r = S.buf.reserve(total)) != MAGE_OK || (r = S.host.reserve(total)) != MAGE_OK) return r;
    char* b = S.buf.as<char>();
    char* h = S.host.as<char>();
    // inputs packed at their device offsets in pinned memory, one H2D copy
    auto put = [&](size_t off, const void* src, size_t n) {
        if (n) std::memcpy(h + off, src, n);
    };
    put(o_pos, pos3, 12 * P);
    put(o_r9, r9, 36 * P);
    put(o_in, intr4, 16 * P);
    put(o_os, obs_start, 4 * (P + 1));
    put(o_pt, points3, 12ull * E);
    put(o_uv, uv, 8ull * E);
    put(o_inf, info, 4ull * E);
    MAGE_HIP(hipMemcpyAsync(b, h, o_pos2, hipMemcpyHostToDevice, S.st));
    PoseParams p{reinterpret_cast<const float*>(b + o_pos), reinterpret_cast<const float*>(b + o_r9),
                 reinterpret_cast<const float*>(b + o_in), reinterpret_cast<const uint32_t*>(b + o_os),
                 reinterpret_cast<const float*>(b + o_pt), reinterpret_cast<const float*>(b + o_uv),
                 reinterpret_cast<const float*>(b + o_inf), nsteps, (double)huber, (double)max_error_square,
                 reinterpret_cast<float*>(b + o_pos2), reinterpret_cast<float*>(b + o_r92),
                 reinterpret_cast<double*>(b + o_qt), reinterpret_cast<uint8_t*>(b + o_out),
                 reinterpret_cast<float*>(b + o_ms), reinterpret_cast<uint32_t*>(b + o_st)};
    if ((r = pose_launch(p, problems, S.st)) != MAGE_OK) return r;
    // outputs: one D2H copy of the contiguous output region, then unpacked on the host
    MAGE_HIP(hipMemcpyAsync(h + o_pos2, b + o_pos2, total - o_pos2, hipMemcpyDeviceToHost, S.st));
    MAGE_HIP(hipStreamSynchronize(S.st));
    std::memcpy(pos3_out, h + o_pos2, 12 * P);
    std::memcpy(r9_out, h + o_r92, 36 * P);
    std::memcpy(mean_sq, h + o_ms, 4 * P);
    if (E) std::memcpy(outlier, h + o_out, E);
    if (qt7_out) std::memcpy(qt7_out, h + o_qt, 56 * P);
    if (stats) std::memcpy(stats, h + o_st, 8 * P);
    return MAGE_OK;
}

#if MAGE_POSE_STAMPS
// development build only (tools/pose_stamps.py): the phase stamps of the last launch's problem 0
mage_status mage_debug_pose_stamps(unsigned long long* out)
{
    MAGE_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(mage::g_pose_st), sizeof(mage::g_pose_st)));
    return MAGE_OK;
}
#endif

}  // extern "C"
