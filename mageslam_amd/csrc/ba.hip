// ba.hip — local bundle adjustment on MI355X (gfx950).  Replaces BundlerLib
// (Dependencies/BundlerLib/Source/BundlerLib.cpp) and the g2o machinery it drives
// (OptimizationAlgorithmLevenberg + BlockSolver_6_3 Schur + LinearSolverDense +
// EdgeProjectXYZ2UV / VertexSE3Expmap / VertexSBAPointXYZ / RobustKernelHuber), in fp64.
//
// Device-resident problem with CSR by point (edge order) and by camera (sorted by point id),
// filtered by a per-edge `active` byte so that outlier removal never rebuilds structure.
// One LM iteration (g2o solve(iteration)):
//   point_linearize   thread/point: errors of its edges (kept per edge, as g2o keeps _error),
//                     robust chi2, Hll, bl and Hpl_e = J_pose^T w J_point per edge
//   cam_linearize     workgroup/camera: Hpp, bp (recomputes J_pose; no per-edge 6x6 in HBM)
//   trial loop (<= 10; one pinned 128-byte control-block readback per trial decides accept /
//   reject on the host):
//     edge_schur      thread/point-edge: Dinv_p = (Hll + lambda I)^-1, db = Dinv bl (first edge
//                     of each point), Z_e = Hpl_e Dinv_p (6x3) for every edge
//     schur_chunks    per covisible camera pair (h1 <= h2) the Schur products (e1, e2) of its
//                     shared points, listed at initialisation and cut into 512-entry chunks: a
//                     workgroup per chunk (no dependent index walk), reduce-scatter sums, the
//                     last chunk of a pair adds the partials in order and writes the 6x6 block
//                     (+ Hpp + lambda I, rhs on h1 = h2); block rows grouped per XCD
//     chol_tiles      one workgroup, np <= 240: register-resident 16x16 upper tiles over 8
//                     waves; per step the owner factors the diagonal block (Cholesky, inverse
//                     and forward substitution in one column loop, look-ahead under the
//                     previous SYRK), TRSM and SYRK on f64 MFMA (v_mfma_f64_16x16x4f64), then a
//                     one-barrier-per-block backward solve.  cholesky_solve: np > 240 (LDS
//                     panels, in-place)
//     update_evaluate xl = Dinv (bl - Hpl^T xp), trial state = exp(xp) * T, p + xl
//                     (double-buffered: pop = no copy), and in the same point groups the errors +
//                     robust chi2 of the trial state;  reduce: chi2 and computeScale
//     outlier_pass    (last step of a StepBundleAdjustment only) speculatively on the trial
//                     and the current state, so the post-pass result is already on the host
// then the StepBundleAdjustment post-pass (BundlerLib.cpp:385-446): outlier indices from the
// speculative (or a fresh) outlier_pass, drop_edges clears their `active` byte.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <vector>

#include "ba_math.hpp"
#include "common.hpp"

namespace mage {
namespace {

using namespace ba;

constexpr int BA_THREADS = 256;

// A group of PG lanes per point (one edge per lane, strided): the edges' load chains run in
// parallel and the point sums close with a fixed shuffle tree (deterministic).
constexpr int PG = 32;

// components of the per-edge Schur records (edge_schur): Q = (x/z, y/z, f/z, W), G
constexpr int EQ_N = 9, EG_N = 6;

// StepBundleAdjustment post-pass results in the pinned control block: per candidate state the
// inlier (sum of |e|^2, count), the Cholesky failure flag and the outlier counts.
// Device-side counters of one trial (appends and the Cholesky failure flag); reduce3 copies them
// into the host-mapped OutlierCtl and zeroes them for the next trial (no memset per trial).
struct LiveCtl {
    int fail;
    uint32_t count[2];
    uint32_t pad;
};
struct OutlierCtl {
    double osum[2][2];
    int fail;
    uint32_t count[2];
    uint32_t ticket;
};

// The LM decision of a trial as reduce3 takes it on the device (OptimizationAlgorithmLevenberg::
// solve: rho = (chi_current - chi_trial) / (scale + 1e-3), accept when rho > 0 and chi_trial is
// finite; lambda *= max(1/3, min(2/3, 1 - (2 rho - 1)^3)) on accept, lambda *= ni on reject), so a
// linearisation of the next state can be queued before the host has read the trial back.  The
// host takes the same decision from the same doubles and adopts lam_next.
struct LmDev {
    double lam_next;
    int cur_next;
    int accept;
};

template <int N>
__device__ __forceinline__ void group_sum(double (&v)[N])
{
#pragma unroll
    for (int off = PG / 2; off > 0; off >>= 1)
#pragma unroll
        for (int k = 0; k < N; k++) v[k] += __shfl_xor(v[k], off);
}

// Butterfly reduce-scatter of N doubles over a group of LANES lanes (xor offsets LANES/2 .. 1):
// per step the lanes without the offset bit keep the first ceil(n/2) entries and the others the
// rest; each lane sends the half it gives up, so a step costs ceil(n/2) shuffles instead of n
// (42 entries over 64 lanes: 44 shuffles instead of 252).  Afterwards the lane holds the group
// total of entry rs_entry() in a[0] (-1: none).  Fixed order, deterministic.
template <int N, int LANES>
__device__ __forceinline__ int reduce_scatter(double (&a)[N], int lane)
{
    static_assert(N <= LANES, "one entry per lane at most");
    // the split sizes are uniform (n, h at compile time); `cnt` is the lane's count of real
    // entries in its range (the upper half of an odd range carries one zero pad)
    int lo = 0, cnt = N;
    int n = N;
#pragma unroll
    for (int off = LANES / 2; off > 0; off >>= 1) {
        const int h = (n + 1) / 2;
        const bool hi = (lane & off) != 0;
#pragma unroll
        for (int i = 0; i < h; i++) {
            const double up = (i + h < n) ? a[i + h] : 0.0;
            const double send = hi ? a[i] : up;
            const double keep = hi ? up : a[i];
            a[i] = keep + __shfl_xor(send, off);
        }
        if (hi) {
            lo += h;
            cnt -= h;
        } else {
            cnt = cnt < h ? cnt : h;
        }
        n = h;
    }
    return cnt > 0 ? lo : -1;
}

// The lane (within its group) that reduce_scatter<N, LANES> leaves entry k in.
template <int N, int LANES>
__host__ __device__ constexpr int rs_lane_of(int k)
{
    int lane = 0, lo = 0, n = N;
    for (int off = LANES / 2; off > 0; off >>= 1) {
        const int h = (n + 1) / 2;
        if (k >= lo + h) {
            lane |= off;
            lo += h;
        }
        n = h;
    }
    return lane;
}

// Eigen Matrix3d::inverse (cofactors)
__device__ __forceinline__ void d_inv3(const double m[9], double o[9])
{
    const double c0 = m[4] * m[8] - m[5] * m[7];
    const double c1 = m[5] * m[6] - m[3] * m[8];
    const double c2 = m[3] * m[7] - m[4] * m[6];
    const double det = m[0] * c0 + m[1] * c1 + m[2] * c2;
    const double id = 1.0 / det;
    o[0] = c0 * id;
    o[1] = (m[2] * m[7] - m[1] * m[8]) * id;
    o[2] = (m[1] * m[5] - m[2] * m[4]) * id;
    o[3] = c1 * id;
    o[4] = (m[0] * m[8] - m[2] * m[6]) * id;
    o[5] = (m[2] * m[3] - m[0] * m[5]) * id;
    o[6] = c2 * id;
    o[7] = (m[1] * m[6] - m[0] * m[7]) * id;
    o[8] = (m[0] * m[4] - m[1] * m[3]) * id;
}

// Outputs of a point pass.
struct PointOut {
    double* err;        // E x 2: edge errors (g2o keeps _error of the last evaluation)
    double* Hll;        // P x 9
    double* bl;         // P x 3
    double* Q;          // EQ_N x ecsr: x/z, y/z, f/z and W = w J_point (camera-major)
    double* G;          // EG_N x ecsr: W Dinv_p (linearisation with a known lambda)
    double* chi_part;   // P: robust chi2 of the point's edges
    double* maxd_part;  // P: max |diag Hll| (computeLambdaInit)
};

// The StepBundleAdjustment post-pass (BundlerLib.cpp:385-446) run speculatively inside the
// evaluation of the last trial, for two candidate states at once: list 0 = the evaluated (trial)
// state if it is accepted, list 1 = the current state if it is rejected (g2o's pop restores the
// vertices but keeps the trial's _error, so both lists test the trial errors).  An active edge
// behind the camera or with |e|^2 > maxErrorSquare is an outlier (index appended; the host sorts
// the short list into g2o's active-edge order); inliers add |e|^2 to block partials that reduce3
// sums in fixed order.
struct SpecPass {
    State cur;
    int on;
    double maxErrSq;
    uint32_t* out_list;  // [2][E]
    int E;
    double* part;        // [2 lists][2][gridDim.x]: inlier sum, count
    LiveCtl* ctl;
};

__device__ __forceinline__ double cheirality_at(const double q[4], const double t[3], const double X[3])
{
    // SE3Quat::inverse: q*, -(q* t); forward = q* (0,0,1)
    const double qc[4] = {-q[0], -q[1], -q[2], q[3]};
    double it[3], fwd[3];
    d_qrot(qc, t, it);
    const double z[3] = {0, 0, 1};
    d_qrot(qc, z, fwd);
    return (X[0] + it[0]) * fwd[0] + (X[1] + it[1]) * fwd[1] + (X[2] + it[2]) * fwd[2];
}

__device__ __forceinline__ double cheirality(const State& s, int c, int p)
{
    const double q[4] = {s.q[4 * c], s.q[4 * c + 1], s.q[4 * c + 2], s.q[4 * c + 3]};
    const double t[3] = {s.t[3 * c], s.t[3 * c + 1], s.t[3 * c + 2]};
    const double X[3] = {s.p[3 * p], s.p[3 * p + 1], s.p[3 * p + 2]};
    return cheirality_at(q, t, X);
}

// One point by a group of PG lanes (one edge per lane, strided): edge errors, robust chi2 and,
// when linearising (BlockSolver::buildSystem with BaseBinaryEdge::constructQuadraticForm, robust
// first-order weighting), Hll, bl and the per-edge Schur records Q; with a known lambda also
// G = W Dinv_p (what edge_schur computes), so the first trial needs no extra sweep.
template <bool LIN>
__device__ __forceinline__ void point_group(const Problem& pb, const State& s, int p, int sub, const PointOut& o,
                                            double lambda, bool with_g, const SpecPass* sp, double (&vs)[2],
                                            double (&vc)[2])
{
    const int free_p = LIN && pb.ptfree[p];
    double acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};  // H 00 01 02 11 12 22, g 0 1 2, chi
    double* H = acc;
    double* g = acc + 6;
    double& chi = acc[9];
    const long long es = pb.ecsr;
    const int e0 = pb.pstart[p], e1 = pb.pstart[p + 1];
    // the lane's edge for the G pass below, kept in registers when the point has at most PG edges
    // (one per lane): camera-CSR position (-1: none or a fixed camera) and W as stored in Q
    int c_ap = -1;
    double c_W[6] = {0, 0, 0, 0, 0, 0};
    const double Xp3[3] = {s.p[3 * p], s.p[3 * p + 1], s.p[3 * p + 2]};  // the group's point (no ept reload)
    for (int a = e0 + sub; a < e1; a += PG) {
        const int4 ent = pb.pe[a];  // (edge, camera, camera block, camera-CSR position)
        const int e = ent.x;
        if (!pb.active[e]) {
            // the Schur products read Q of every listed edge: a removed edge contributes zero
            if (LIN && ent.z >= 0) {
                c_ap = ent.w;
                if (free_p) {
                    double* q = o.Q + c_ap;
                    for (int k = 0; k < EQ_N; k++) q[k * es] = 0;
                }
            }
            continue;
        }
        double ev[2], xc[3], rho0, rho1;
        const int c = ent.y;
        {
            const double q[4] = {s.q[4 * c], s.q[4 * c + 1], s.q[4 * c + 2], s.q[4 * c + 3]};
            const double t[3] = {s.t[3 * c], s.t[3 * c + 1], s.t[3 * c + 2]};
            edge_eval_at(pb, e, c, q, t, Xp3, ev, xc, rho0, rho1);
        }
        if (o.err) {  // (a speculative linearisation after a rejected trial keeps the trial's errors)
            o.err[2 * e] = ev[0];
            o.err[2 * e + 1] = ev[1];
        }
        chi += rho0;
        if (!LIN) {
            if (sp) {
                const double sumSquares = ev[0] * ev[0] + ev[1] * ev[1];
#pragma unroll
                for (int k = 0; k < 2; k++) {
                    const double dot = cheirality(k == 0 ? s : sp->cur, c, p);
                    if (dot <= 0 || sumSquares > sp->maxErrSq) {
                        sp->out_list[(long long)k * sp->E + atomicAdd(&sp->ctl->count[k], 1u)] = (uint32_t)e;
                    } else {
                        vs[k] += sumSquares;
                        vc[k] += 1;
                    }
                }
            }
            continue;
        }
        const bool cam_free = ent.z >= 0;
        if (cam_free) c_ap = ent.w;
        if (!free_p) continue;
        const double f = pb.camk[3 * c];
        const double q[4] = {s.q[4 * c], s.q[4 * c + 1], s.q[4 * c + 2], s.q[4 * c + 3]};
        double R[9];
        d_qmat(q, R);
        const double iz = 1.0 / xc[2], xi = xc[0] * iz, yi = xc[1] * iz;  // one reciprocal (see jac_pose)
        const double tmp0[3] = {f, 0, -xi * f}, tmp1[3] = {0, f, -yi * f};
        double J[6];
        for (int k = 0; k < 3; k++) {
            J[k] = -iz * (tmp0[0] * R[k] + tmp0[1] * R[3 + k] + tmp0[2] * R[6 + k]);
            J[3 + k] = -iz * (tmp1[0] * R[k] + tmp1[1] * R[3 + k] + tmp1[2] * R[6 + k]);
        }
        const double inf = pb.info[e];
        const double w = rho1 * inf;
        const double or0 = -inf * ev[0] * rho1, or1 = -inf * ev[1] * rho1;
        g[0] += J[0] * or0 + J[3] * or1;
        g[1] += J[1] * or0 + J[4] * or1;
        g[2] += J[2] * or0 + J[5] * or1;
        H[0] += (J[0] * J[0] + J[3] * J[3]) * w;
        H[1] += (J[0] * J[1] + J[3] * J[4]) * w;
        H[2] += (J[0] * J[2] + J[3] * J[5]) * w;
        H[3] += (J[1] * J[1] + J[4] * J[4]) * w;
        H[4] += (J[1] * J[2] + J[4] * J[5]) * w;
        H[5] += (J[2] * J[2] + J[5] * J[5]) * w;
        if (cam_free) {
            // Hpl_e = Jp^T (w J): kept factored as (x/z, y/z, f/z) + W = w J (camera-major
            // component arrays; schur_chunks reads them coalesced)
            double* qo = o.Q + c_ap;
            qo[0] = xi;
            qo[es] = yi;
            qo[2 * es] = f * iz;
            for (int k = 0; k < 6; k++) {
                c_W[k] = J[k] * w;
                qo[(3 + k) * es] = c_W[k];
            }
        }
    }
    // group sums by reduce-scatter: lane `sub` ends up with entry k of acc (H 00 01 02 11 12 22,
    // g 0 1 2, chi) and writes it
    const int k = reduce_scatter<10, PG>(acc, sub);
    const double v = acc[0];
    const int gbase = (threadIdx.x & (kWave - 1)) & ~(PG - 1);
    if (LIN) {
        double h6[6];
#pragma unroll
        for (int j = 0; j < 6; j++) h6[j] = __shfl(v, gbase + rs_lane_of<10, PG>(j));
        if (sub == rs_lane_of<10, PG>(0)) o.maxd_part[p] = free_p ? fmax(fabs(h6[0]), fmax(fabs(h6[3]), fabs(h6[5]))) : 0.0;
        if (with_g) {
            // D_p = Hll_p + lambda I and its inverse exactly as edge_schur forms them from Hll
            double D[9] = {h6[0], h6[1], h6[2], h6[1], h6[3], h6[4], h6[2], h6[4], h6[5]}, Di[9];
            D[0] += lambda;
            D[4] += lambda;
            D[8] += lambda;
            d_inv3(D, Di);
            auto store_g = [&](int ap, const double (&W)[6]) {
                if (!free_p) {
                    for (int j = 0; j < EG_N; j++) o.G[j * es + ap] = 0;
                    return;
                }
#pragma unroll
                for (int i = 0; i < 2; i++)
#pragma unroll
                    for (int kk = 0; kk < 3; kk++)
                        o.G[(i * 3 + kk) * es + ap] = W[i * 3] * Di[kk] + W[i * 3 + 1] * Di[3 + kk] + W[i * 3 + 2] * Di[6 + kk];
            };
            if (e1 - e0 <= PG) {
                // the lane's one edge from registers (no dependent reload of pedges / ecam /
                // camh / epos / Q after the group reduction)
                if (c_ap >= 0) store_g(c_ap, c_W);
            } else {
                for (int a = e0 + sub; a < e1; a += PG) {
                    const int4 ent = pb.pe[a];
                    if (ent.z < 0) continue;
                    const int ap = ent.w;
                    double W[6];
#pragma unroll
                    for (int j = 0; j < 6; j++) W[j] = o.Q[(3 + j) * es + ap];
                    store_g(ap, W);
                }
            }
        }
    }
    if (k == 9) o.chi_part[p] = v;
    if (!LIN || k < 0 || k == 9) return;
    if (k >= 6) {
        o.bl[3 * p + (k - 6)] = v;
        return;
    }
    // packed upper (00 01 02 11 12 22) -> both symmetric positions of the 3x3
    constexpr int r_of[6] = {0, 0, 0, 1, 1, 2}, c_of[6] = {0, 1, 2, 1, 2, 2};
    double* Ho = o.Hll + 9 * (long long)p;
    const int r = r_of[k], c = c_of[k];
    Ho[3 * r + c] = v;
    Ho[3 * c + r] = v;
}

// Tether edges (thread per tether; a window carries a handful): error and chi2 = e^T Omega e
// into chi[t] (appended after the points' robust chi2); with `linearize`, the Jacobians —
// BaseMultiEdge::linearizeOplus central differences (delta 1e-9 through the exp-map oplus) for the
// distance / rotation constraints, EdgeSE3Expmap's adjoints for the transform — and the blocks
// H11 = J1^T Omega J1, H22, H12 = J1^T Omega J2, b_v = J_v^T (-Omega e) into out[t][TETHER_OUT].
__global__ __launch_bounds__(64) void tether_eval(const Tether* __restrict__ teth, int nt, State s, int linearize,
                                                  double* __restrict__ chi, double* __restrict__ out)
{
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= nt) return;
    const Tether T = teth[i];
    if (!T.active) {
        chi[i] = 0;
        return;
    }
    double q1[4], t1[3], q2[4], t2[3];
    for (int k = 0; k < 4; k++) {
        q1[k] = s.q[4 * T.c1 + k];
        q2[k] = s.q[4 * T.c2 + k];
    }
    for (int k = 0; k < 3; k++) {
        t1[k] = s.t[3 * T.c1 + k];
        t2[k] = s.t[3 * T.c2 + k];
    }
    double e[6];
    const int dim = d_tether_error(T, q1, t1, q2, t2, e);
    const double om = T.kind == 2 ? T.w : 1.0;
    double c2 = 0;
    for (int r = 0; r < dim; r++) c2 += e[r] * e[r];
    chi[i] = om * c2;
    if (!linearize) return;
    double J[2][36];
    if (T.kind == 2) {
        double a[4], at[3], b[4], bt[3], iq[4], it[3], mq[4], mt[3];
        d_se3_inv(T.mq, T.mt, mq, mt);  // Tij^-1
        d_se3_inv(q2, t2, iq, it);
        d_se3_mul(iq, it, T.mq, T.mt, a, at);  // Tj^-1 Tij
        d_se3_inv(q1, t1, iq, it);
        d_se3_mul(iq, it, mq, mt, b, bt);  // Ti^-1 Tij^-1
        d_se3_adj(a, at, false, J[0]);
        d_se3_adj(b, bt, true, J[1]);
    } else {
        const double delta = 1e-9, scalar = 1 / (2 * delta);
        for (int v = 0; v < 2; v++) {
            if ((v ? T.h2 : T.h1) < 0) continue;
            for (int d = 0; d < 6; d++) {
                double add[6] = {0, 0, 0, 0, 0, 0}, ep[6], em[6];
                double pq[4], pt[3];
                add[d] = delta;
                for (int k = 0; k < 4; k++) pq[k] = v ? q2[k] : q1[k];
                for (int k = 0; k < 3; k++) pt[k] = v ? t2[k] : t1[k];
                d_oplus(pq, pt, add);
                if (v) d_tether_error(T, q1, t1, pq, pt, ep);
                else d_tether_error(T, pq, pt, q2, t2, ep);
                add[d] = -delta;
                for (int k = 0; k < 4; k++) pq[k] = v ? q2[k] : q1[k];
                for (int k = 0; k < 3; k++) pt[k] = v ? t2[k] : t1[k];
                d_oplus(pq, pt, add);
                if (v) d_tether_error(T, q1, t1, pq, pt, em);
                else d_tether_error(T, pq, pt, q2, t2, em);
                J[v][d] = scalar * (ep[0] - em[0]);
            }
        }
    }
    double* o = out + (long long)i * TETHER_OUT;
    for (int v = 0; v < 2; v++) {
        if ((v ? T.h2 : T.h1) < 0) continue;
        const double* Jv = J[v];
        for (int r = 0; r < 6; r++) {
            double g = 0;
            for (int m = 0; m < dim; m++) g += Jv[m * 6 + r] * (-om * e[m]);
            o[108 + 6 * v + r] = g;
            for (int c = 0; c < 6; c++) {
                double h = 0;
                for (int m = 0; m < dim; m++) h += Jv[m * 6 + r] * Jv[m * 6 + c];
                o[36 * v + r * 6 + c] = h * om;
            }
        }
    }
    if (T.h1 >= 0 && T.h2 >= 0)
        for (int r = 0; r < 6; r++)
            for (int c = 0; c < 6; c++) {
                double h = 0;
                for (int m = 0; m < dim; m++) h += J[0][m * 6 + r] * J[1][m * 6 + c];
                o[72 + r * 6 + c] = h * om;
            }
}

// Block sum of `acc[N]` over a workgroup of T threads; the result lands in red[0][0..N).  Per
// wave a reduce-scatter (each lane ends with one entry), then the waves' partials in order.
template <int N, int T = BA_THREADS>
__device__ __forceinline__ void block_sum(double (&acc)[N], double (*red)[N])
{
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int k = reduce_scatter<N, kWave>(acc, lane);
    if (k >= 0) red[wave][k] = acc[0];
    __syncthreads();
    if (threadIdx.x < N) {
        double v = 0;
        for (int w = 0; w < T / kWave; w++) v += red[w][threadIdx.x];
        acc[0] = v;  // thread k keeps the total of entry k in acc[0]
    }
    __syncthreads();
    if (threadIdx.x < N) red[0][threadIdx.x] = acc[0];
    __syncthreads();
}

// Per free camera: Hpp (6x6, packed upper 21) and bp (6) partial sums from its active edges.
// CAM_CHUNKS workgroups per camera (block = h * CAM_CHUNKS + chunk) take interleaved slices of its
// edge list and write their partials; schur_finish (or linearize_finish) adds them in chunk order
// (no cross-workgroup hand-off inside the kernel).
constexpr int CAM_CHUNKS = 8;
constexpr int MAX_FREE_CAMS = 96;  // = CH_PANEL_ROWS / 6, the system-size limit checked at initialisation

__device__ __forceinline__ void cam_chunk(const Problem& pb, const State& s, const int* __restrict__ cam_of_block,
                                          double* __restrict__ part, int blk)  // part: [nb][CAM_CHUNKS][27]
{
    const int h = blk / CAM_CHUNKS, chunk = blk % CAM_CHUNKS;
    const int c = cam_of_block[h];
    __shared__ double red[BA_THREADS / kWave][27];
    double acc[27];
    for (int k = 0; k < 27; k++) acc[k] = 0;
    const double f = pb.camk[3 * c];
    // the block's camera pose once; an entry's point from cpt (no ecam / ept reload per edge)
    const double q[4] = {s.q[4 * c], s.q[4 * c + 1], s.q[4 * c + 2], s.q[4 * c + 3]};
    const double t[3] = {s.t[3 * c], s.t[3 * c + 1], s.t[3 * c + 2]};
    for (int a = pb.cstart[c] + chunk * BA_THREADS + threadIdx.x; a < pb.cstart[c + 1]; a += CAM_CHUNKS * BA_THREADS) {
        const int e = pb.cedges[a], pt = pb.cpt[a];
        if (!pb.active[e]) continue;
        double ev[2], xc[3], rho0, rho1;
        const double X[3] = {s.p[3 * pt], s.p[3 * pt + 1], s.p[3 * pt + 2]};
        edge_eval_at(pb, e, c, q, t, X, ev, xc, rho0, rho1);  // the same error point_group computes for e
        double Jp[12];
        jac_pose(xc, f, Jp);
        const double inf = pb.info[e];
        const double w = rho1 * inf;
        const double or0 = -inf * ev[0] * rho1, or1 = -inf * ev[1] * rho1;
        int k = 0;
        for (int r = 0; r < 6; r++)
            for (int cc = r; cc < 6; cc++) acc[k++] += (Jp[r] * Jp[cc] + Jp[6 + r] * Jp[6 + cc]) * w;
        for (int r = 0; r < 6; r++) acc[21 + r] += Jp[r] * or0 + Jp[6 + r] * or1;
    }
    block_sum<27>(acc, red);
    if (threadIdx.x < 27) part[((long long)h * CAM_CHUNKS + chunk) * 27 + threadIdx.x] = red[0][threadIdx.x];
}

// The linearisation sweep in one launch: blocks [0, npb) are point groups (point_group<true>),
// the rest camera chunks (CAM_CHUNKS per free camera: Hpp packed upper 21 + bp 6 partials,
// added in chunk order by schur_finish / linearize_finish).
__global__ __launch_bounds__(BA_THREADS) void linearize_kernel(Problem pb, State s, PointOut o, double lambda, int with_g,
                                                               int npb, const int* __restrict__ cam_of_block,
                                                               double* __restrict__ campart, State s1,
                                                               const LmDev* __restrict__ lm)
{
    if (lm) {
        // speculative: the state and lambda of the decision reduce3 just took (s = buffer 0, s1 =
        // buffer 1); after a rejection the state is unchanged and the trial's errors stay
        if (lm->cur_next == 1) s = s1;
        lambda = lm->lam_next;
        if (!lm->accept) o.err = nullptr;
    }
    if ((int)blockIdx.x >= npb) {
        cam_chunk(pb, s, cam_of_block, campart, blockIdx.x - npb);
        return;
    }
    const int gid = blockIdx.x * BA_THREADS + threadIdx.x;
    const int p = gid / PG, sub = gid % PG;
    if (p >= pb.P) return;  // whole groups
    double vs[2], vc[2];
    point_group<true>(pb, s, p, sub, o, lambda, with_g != 0, nullptr, vs, vc);
}

// After the linearisation (one workgroup): Hpp / bp of every free camera from its chunk partials,
// and out[0] = sum of the points' robust chi2, out[2] = max diagonal entry over Hll and Hpp
// (computeLambdaInit), with the fixed-order tree of reduce3.
__global__ __launch_bounds__(1024) void linearize_finish(int nb, const int* __restrict__ cam_of_block,
                                                         const double* __restrict__ part,
                                                         const double* __restrict__ chi, int P,
                                                         const double* __restrict__ maxd_pts,
                                                         const Tether* __restrict__ teth, int nt,
                                                         const double* __restrict__ tout,
                                                         double* __restrict__ Hpp, double* __restrict__ bp,
                                                         double* __restrict__ out)
{
    __shared__ double cams[MAX_FREE_CAMS][27];
    __shared__ double sa[1024], sm[1024];
    const int tid = threadIdx.x;
    for (int i = tid; i < nb * 27; i += 1024) {
        const int h = i / 27, k = i % 27;
        double v = 0;
        for (int q = 0; q < CAM_CHUNKS; q++) v += part[((long long)h * CAM_CHUNKS + q) * 27 + k];
        // tethers after the observations (g2o's addEdge order), each in its set order
        if (nt > 0) {
            int r = 0, c = k;
            if (k < 21)
                while (c >= 6 - r) {
                    c -= 6 - r;
                    r++;
                }
            for (int t = 0; t < nt; t++) {
                const Tether& T = teth[t];
                if (!T.active) continue;
                for (int vtx = 0; vtx < 2; vtx++) {
                    if ((vtx ? T.h2 : T.h1) != h) continue;
                    const double* o = tout + (long long)t * TETHER_OUT;
                    v += k < 21 ? o[36 * vtx + r * 6 + (r + c)] : o[108 + 6 * vtx + (k - 21)];
                }
            }
        }
        cams[h][k] = v;
    }
    __syncthreads();
    for (int i = tid; i < nb * 42; i += 1024) {
        const int h = i / 42, k = i % 42, c = cam_of_block[h];
        if (k < 36) {
            int r = k / 6, cc = k % 6;
            if (r > cc) {
                const int t = r;
                r = cc;
                cc = t;
            }
            Hpp[36 * (long long)c + k] = cams[h][r * 6 - r * (r - 1) / 2 + (cc - r)];
        } else {
            bp[6 * c + (k - 36)] = cams[h][21 + (k - 36)];
        }
    }
    double va = 0, vm = 0;
    for (int i = tid; i < P; i += 1024) {
        va += chi[i];
        vm = fmax(vm, maxd_pts[i]);
    }
    for (int i = tid; i < nt; i += 1024) va += chi[P + i];
    for (int h = tid; h < nb; h += 1024)
        for (int r = 0; r < 6; r++) vm = fmax(vm, fabs(cams[h][r * 6 - r * (r - 1) / 2]));
    sa[tid] = va;
    sm[tid] = vm;
    __syncthreads();
    for (int st = 512; st > 0; st >>= 1) {
        if (tid < st) {
            sa[tid] += sa[tid + st];
            sm[tid] = fmax(sm[tid], sm[tid + st]);
        }
        __syncthreads();
    }
    if (tid == 0) {
        out[0] = sa[0];
        out[1] = 0;
        out[2] = sm[0];
    }
}


// Fixed-order reduction of two sum arrays and one max array into out[0..2], a third sum array into
// outc[0] (the linearisation's chi2), and with ns > 0 the post-pass's per-block (sum, count)
// partials of its ns states into ctl->osum.
__global__ __launch_bounds__(1024) void reduce3(const double* __restrict__ a, int na,
                                                const double* __restrict__ b, int nb,
                                                const double* __restrict__ m, int nm,
                                                double* __restrict__ out,
                                                const double* __restrict__ c, int nc, double* __restrict__ outc,
                                                const double* __restrict__ opart, int oblocks, int ns,
                                                OutlierCtl* __restrict__ ctl, LiveCtl* __restrict__ live,
                                                unsigned* __restrict__ seq_out, unsigned seq,
                                                LmDev* __restrict__ lm, double lam, double ni, int cur,
                                                double cur_chi, double* __restrict__ lam_out)
{
    // the seven sums in one pass (strided per thread, fixed order), one reduce-scatter per wave,
    // then the 16 wave partials in order; the max separately (only linearize_finish's callers
    // need it, nm = 0 here in practice)
    __shared__ double red[1024 / kWave][8];
    __shared__ double smax[1024 / kWave];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    double v[7] = {0, 0, 0, 0, 0, 0, 0};  // a, b, c, osum[0] (sum, count), osum[1] (sum, count)
    double vm = 0;
    // Strided sums (thread tid adds elements tid, tid + 1024, ... of each array in order) with the
    // first loads of every array issued together (one array after another waited on each array's
    // loads in turn: 7 dependent memory round trips per launch on C3, 6.9 -> 6.0 us in
    // tools/ablate_ba.py); the tails past them follow.
    const double* segp[7] = {a, b, c, opart, opart + oblocks, opart + 2 * oblocks, opart + 3 * oblocks};
    const int segn[7] = {na, nb, nc, ns > 0 ? oblocks : 0, ns > 0 ? oblocks : 0, ns > 1 ? oblocks : 0,
                         ns > 1 ? oblocks : 0};
    constexpr int J3 = 6, J4 = 1;  // first loads per thread: point / camera arrays, block partials
    // branch-free: every load reads a valid address (an absent array reads the live block) and a
    // select drops what lies past the array, so no load waits inside a branch
    auto first = [&](int k, int j) {
        const int i = tid + 1024 * j, n = segn[k];
        const double* src = n > 0 ? segp[k] : reinterpret_cast<const double*>(live);
        const double x = src[min(i, max(n - 1, 0))];
        return i < n ? x : 0.0;
    };
    double t3[3][J3], t4[4][J4];
#pragma unroll
    for (int k = 0; k < 3; k++)
#pragma unroll
        for (int j = 0; j < J3; j++) t3[k][j] = first(k, j);
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
        for (int j = 0; j < J4; j++) t4[k][j] = first(3 + k, j);
#pragma unroll
    for (int k = 0; k < 3; k++)
#pragma unroll
        for (int j = 0; j < J3; j++) v[k] += t3[k][j];
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
        for (int j = 0; j < J4; j++) v[3 + k] += t4[k][j];
#pragma unroll
    for (int k = 0; k < 7; k++)
        for (int i = tid + 1024 * (k < 3 ? J3 : J4); i < segn[k]; i += 1024) v[k] += segp[k][i];
    for (int i = tid; i < nm; i += 1024) vm = fmax(vm, m[i]);
    const int e = reduce_scatter<7, kWave>(v, lane);
    if (e >= 0) red[wave][e] = v[0];
    for (int off = 32; off > 0; off >>= 1) vm = fmax(vm, __shfl_xor(vm, off));
    if (lane == 0) smax[wave] = vm;
    __syncthreads();
    if (tid < 7) {
        double t = 0;
        for (int w = 0; w < 1024 / kWave; w++) t += red[w][tid];
        red[0][tid] = t;
    } else if (tid == 7) {
        double t = 0;
        for (int w = 0; w < 1024 / kWave; w++) t = fmax(t, smax[w]);
        red[0][7] = t;
    }
    __syncthreads();
    if (tid == 0) {
        out[0] = red[0][0];
        out[1] = red[0][1];
        out[2] = red[0][7];
        if (nc > 0) outc[0] = red[0][2];
        for (int k = 0; k < ns; k++) {
            ctl->osum[k][0] = red[0][3 + 2 * k];
            ctl->osum[k][1] = red[0][4 + 2 * k];
        }
        if (lm) {
            // the trial's LM decision (see LmDev); the chi of the current state is the
            // linearisation's (reduced here) unless the host passed it
            const double tempChi = live->fail ? __DBL_MAX__ : red[0][0];
            const double currentChi = isnan(cur_chi) ? red[0][2] : cur_chi;
            double rho = currentChi - tempChi;
            const double scale = red[0][1] + 1e-3;
            rho /= scale;
            const bool acc = rho > 0 && isfinite(tempChi);
            double ln;
            if (acc) {
                double alpha = 1. - pow(2 * rho - 1, 3.0);
                alpha = fmin(alpha, 2. / 3.);
                ln = lam * fmax(1. / 3., alpha);
            } else {
                ln = lam * ni;
            }
            lm->lam_next = ln;
            lm->cur_next = acc ? 1 - cur : cur;
            lm->accept = acc ? 1 : 0;
            lam_out[0] = ln;
        }
        // the trial's counters to the host block, and zero for the next trial
        ctl->fail = live->fail;
        ctl->count[0] = live->count[0];
        ctl->count[1] = live->count[1];
        live->fail = 0;
        live->count[0] = 0;
        live->count[1] = 0;
        // completion word for the host's spin-wait: every result above reaches host memory first
        // (drained plain stores before the word measured the same, tools/ablate_ba.py)
        __threadfence_system();
        *reinterpret_cast<volatile unsigned*>(seq_out) = seq;
    }
}


// Per-edge factors of the Schur sweeps, camera-major component arrays (entry k of edge record a
// at k * ecsr + a, a = the edge's camera-CSR position):
//   Q (EQ_N = 9): x/z, y/z, f/z of the point in the camera (the pose Jacobian Jp, jac_pose_q)
//                 and W = w J_point (2x3), so Hpl_e = Jp^T W;
//   G (6):        G = W Dinv_p (2x3), so Z_e = Hpl_e Dinv_p = Jp^T G.
// A Schur product Z_e1 Hpl_e2^T = Jp1^T (G1 W2^T) Jp2 then reads 18 doubles instead of 36.

// Per camera-CSR entry a: D_p = Hll_p + lambda I, Dinv_p by cofactors (recomputed per entry) and
// G_a = W_a Dinv_p.  Entries of fixed cameras take no part; a point that lost its last edge gets
// G = 0.
__global__ __launch_bounds__(BA_THREADS) void edge_schur(Problem pb, const double* __restrict__ Hll,
                                                         const double* __restrict__ Q, double lambda,
                                                         double* __restrict__ G)
{
    const int a = blockIdx.x * BA_THREADS + threadIdx.x;
    if (a >= pb.ecsr) return;
    const int e = pb.cedges[a];
    if (pb.camh[pb.ecam[e]] < 0) return;
    const int p = pb.cpt[a];
    const long long es = pb.ecsr;
    if (!pb.ptfree[p]) {
        for (int k = 0; k < EG_N; k++) G[k * es + a] = 0;
        return;
    }
    double D[9], Di[9];
#pragma unroll
    for (int k = 0; k < 9; k++) D[k] = Hll[9 * (long long)p + k];
    D[0] += lambda;
    D[4] += lambda;
    D[8] += lambda;
    d_inv3(D, Di);
    double w[6];
#pragma unroll
    for (int k = 0; k < 6; k++) w[k] = Q[(3 + k) * es + a];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int k = 0; k < 3; k++)
            G[(i * 3 + k) * es + a] = w[i * 3] * Di[k] + w[i * 3 + 1] * Di[3 + k] + w[i * 3 + 2] * Di[6 + k];
}

// Schur complement (BlockSolver::solve's Schur loop), per covisible camera pair (h1 <= h2):
//   S[h1][h2] = delta(h1,h2) (Hpp_c1 + lambda I) - sum_p Hpl_{c1 p} Dinv_p Hpl_{c2 p}^T
//   rhs[h1]   = bp_c1 - sum_p Hpl_{c1 p} Dinv_p bl_p                          (h1 == h2 only)
// The products are enumerated once per initialisation: a pair's list holds (e1, e2) for every
// shared free point (c1's edge e1, c2's edge e2; on the diagonal every ordered pair of the
// camera's edges on the point), and the diagonal pair carries a second list of (e, p) for the rhs.
// Lists are cut into chunks of <= SC_CHUNK entries, one 256-thread workgroup per chunk: each
// thread loads its two entries, then Z_e1 = Hpl_e1 Dinv_p (edge_schur) and Hpl_e2 (or bl_p) with
// no further dependent load, accumulates the 6x6 (+ 6 rhs) in registers, and the chunk sum is
// a reduce-scatter + LDS tree.  Inactive edges have zero Hpl / Z (point_linearize, edge_schur),
// so no flag is read.  A pair of one chunk finishes in place; otherwise its chunks write partials
// and schur_finish adds them in chunk order (deterministic; a last-arriver ticket would need an
// agent-scope fence = a full L2 write-back per workgroup on gfx950).  XCD-aware: the chunks of
// one block row of S run on one XCD (block b on XCD b % 8), so Z_{c1 .} stays in that L2.
constexpr int SC_THREADS = 256;
constexpr int SC_CHUNK = 2 * SC_THREADS;

struct SchurChunk {
    int pair;   // -1: padding block
    int start;  // first entry
    int count;  // entries (<= SC_CHUNK); the rhs list's chunks have kind 1
    int kind;   // 0 products (e1, e2), 1 rhs (e, p)
    int slot;   // partial slot of this chunk (pairs of more than one chunk)
    int pad0, pad1, pad2;
};
struct SchurPair {
    int h1, h2, c1;
    int slot0, nslots;  // partial slots [slot0, slot0 + nslots); nslots = 1: finished in place
    int tbeg, tend;     // tether H12 blocks of this pair: ptlist[tbeg, tend)
    int c2;
};

// Entry k < 42 of a pair's sum -> S (both triangles; + Hpp + lambda I on the diagonal, + tether
// H12 blocks) or rhs (k >= 36, diagonal pairs: bp - sum).  `cam` is Hpp[k] (k < 36) or bp[k - 36]
// of the diagonal pair's camera.
__device__ __forceinline__ void schur_write(const SchurPair& pr, int k, double sum, double cam, double lambda, int np,
                                            const int* __restrict__ ptlist, const double* __restrict__ tout,
                                            double* __restrict__ S, double* __restrict__ rhs)
{
    const bool diag = pr.h1 == pr.h2;
    if (k < 36) {
        const int r = k / 6, c = k % 6;
        // a diagonal block's (r, c) and (c, r) sums add the same products in another order: only
        // the upper entry's value is written, to both triangles (one writer per address, so the
        // result does not depend on which store lands last)
        if (diag && r > c) return;
        double v = -sum;
        if (diag) v += cam + (r == c ? lambda : 0.0);
        // tether H12 blocks of this camera pair (code = 2 t + transposed)
        for (int j = pr.tbeg; j < pr.tend; j++) {
            const int code = ptlist[j];
            const double* H12 = tout + (long long)(code >> 1) * TETHER_OUT + 72;
            v += (code & 1) ? H12[c * 6 + r] : H12[r * 6 + c];
        }
        S[(long long)(6 * pr.h1 + r) * np + 6 * pr.h2 + c] = v;
        S[(long long)(6 * pr.h2 + c) * np + 6 * pr.h1 + r] = v;
    } else if (diag) {
        rhs[6 * pr.h1 + (k - 36)] = cam - sum;
    }
}

__global__ __launch_bounds__(SC_THREADS) void schur_chunks(const SchurChunk* __restrict__ chunks,
                                                           const SchurPair* __restrict__ pairs,
                                                           const int2* __restrict__ entries,
                                                           const double* __restrict__ G,
                                                           const double* __restrict__ Q,
                                                           const double* __restrict__ camk,
                                                           const double* __restrict__ bl, double lambda, int np, int ecsr,
                                                           const int* __restrict__ ptlist,
                                                           const double* __restrict__ tout,
                                                           double* __restrict__ part,
                                                           double* __restrict__ S, double* __restrict__ rhs)
{
    __shared__ double red[SC_THREADS / kWave][42];
    const SchurChunk ch = chunks[blockIdx.x];
    if (ch.pair < 0) return;
    const int t = threadIdx.x;
    const long long es = ecsr;
    double acc[42];
#pragma unroll
    for (int k = 0; k < 42; k++) acc[k] = 0;
    // both entries' indices first (padding -> the zero record), then every operand load
    // (a chunk of count 0 reads the list's padding entry; invalid lanes repeat the last entry)
    const int2 x0 = entries[ch.start + max(0, min(t, ch.count - 1))];
    const int2 x1 = entries[ch.start + max(0, min(t + SC_THREADS, ch.count - 1))];
    const bool v0 = t < ch.count, v1 = t + SC_THREADS < ch.count;
    const SchurPair pr = pairs[ch.pair];
    const double f1 = camk[3 * pr.c1], f2 = camk[3 * pr.c2];
    // records at camera-CSR positions, component arrays of stride es: consecutive entries of a
    // pair are (mostly) consecutive positions, so every load below is coalesced
    double q0[3], g0[6], q1[3], g1[6];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        q0[k] = Q[k * es + x0.x];
        q1[k] = Q[k * es + x1.x];
    }
#pragma unroll
    for (int k = 0; k < 6; k++) {
        g0[k] = G[k * es + x0.x];
        g1[k] = G[k * es + x1.x];
    }
    if (ch.kind == 0) {
        // Z_e1 Hpl_e2^T = Jp1^T (G1 W2^T) Jp2
        double r0[3], w0[6], r1[3], w1[6];
#pragma unroll
        for (int k = 0; k < 3; k++) {
            r0[k] = Q[k * es + x0.y];
            r1[k] = Q[k * es + x1.y];
        }
#pragma unroll
        for (int k = 0; k < 6; k++) {
            w0[k] = Q[(3 + k) * es + x0.y];
            w1[k] = Q[(3 + k) * es + x1.y];
        }
        auto product = [&](const double (&q)[3], const double (&g)[6], const double (&rq)[3], const double (&w)[6],
                           bool valid) {
            double J1[12], J2[12];
            jac_pose_q(q[0], q[1], q[2], f1, J1);
            jac_pose_q(rq[0], rq[1], rq[2], f2, J2);
            double M[4];
#pragma unroll
            for (int i = 0; i < 2; i++)
#pragma unroll
                for (int j = 0; j < 2; j++) M[i * 2 + j] = g[i * 3] * w[j * 3] + g[i * 3 + 1] * w[j * 3 + 1] + g[i * 3 + 2] * w[j * 3 + 2];
            if (!valid) M[0] = M[1] = M[2] = M[3] = 0;
            double T[12];
#pragma unroll
            for (int i = 0; i < 2; i++)
#pragma unroll
                for (int c = 0; c < 6; c++) T[i * 6 + c] = M[i * 2] * J2[c] + M[i * 2 + 1] * J2[6 + c];
#pragma unroll
            for (int r = 0; r < 6; r++)
#pragma unroll
                for (int c = 0; c < 6; c++) acc[r * 6 + c] = fma(J1[r], T[c], fma(J1[6 + r], T[6 + c], acc[r * 6 + c]));
        };
        product(q0, g0, r0, w0, v0);
        product(q1, g1, r1, w1, v1);
    } else {
        // Z_e bl_p = Jp^T (G bl_p)
        double b0[3], b1[3];
#pragma unroll
        for (int m = 0; m < 3; m++) {
            b0[m] = bl[3 * x0.y + m];
            b1[m] = bl[3 * x1.y + m];
        }
        auto term = [&](const double (&q)[3], const double (&g)[6], const double (&b)[3], bool valid) {
            double J[12];
            jac_pose_q(q[0], q[1], q[2], f1, J);
            double u0 = g[0] * b[0] + g[1] * b[1] + g[2] * b[2], u1 = g[3] * b[0] + g[4] * b[1] + g[5] * b[2];
            if (!valid) u0 = u1 = 0;
#pragma unroll
            for (int r = 0; r < 6; r++) acc[36 + r] = fma(J[r], u0, fma(J[6 + r], u1, acc[36 + r]));
        };
        term(q0, g0, b0, v0);
        term(q1, g1, b1, v1);
    }
    block_sum<42, SC_THREADS>(acc, red);  // red[0][k] = chunk total of entry k
    if (pr.nslots > 1 || pr.h1 == pr.h2) {  // schur_finish: partials in order, the camera blocks
        if (t < 42) part[(long long)ch.slot * 42 + t] = red[0][t];
        return;
    }
    if (t < 42) schur_write(pr, t, red[0][t], 0.0, lambda, np, ptlist, tout, S, rhs);
}

// Diagonal pairs and pairs of more than one chunk: entry t < 42 of a pair adds its chunk partials
// in chunk order.  A diagonal pair's camera block comes from the linearisation partials (chunk
// order, then the tethers in set order: g2o's addEdge order), written to Hpp / bp as well
// (update_state's computeScale reads bp).  A 64-lane wave per pair.
struct FinishArgs {
    const int* flist;
    int nf;  // pairs in flist (0: S and rhs are complete)
    const SchurPair* pairs;
    const double* part;
    const double* campart;
    const Tether* teth;
    int nt;
    double* Hpp;
    double* bp;
    double lambda;
    const int* ptlist;
    const double* tout;
    double* S;
    double* rhs;
};

__device__ __forceinline__ void finish_entry(const FinishArgs& a, const SchurPair& pr, int t, int np)
{
    double v = 0;
    for (int q0 = 0; q0 < pr.nslots; q0 += 8) {  // chunk order, the loads of 8 partials in flight together
        double x[8];
#pragma unroll
        for (int q = 0; q < 8; q++) x[q] = q0 + q < pr.nslots ? a.part[(long long)(pr.slot0 + q0 + q) * 42 + t] : 0.0;
#pragma unroll
        for (int q = 0; q < 8; q++)
            if (q0 + q < pr.nslots) v += x[q];
    }
    double cam = 0;
    if (pr.h1 == pr.h2) {
        const int h = pr.h1;
        int pk, r = 0, c = 0;  // packed upper index of (min, max), or 21 + rhs entry
        if (t < 36) {
            r = min(t / 6, t % 6);
            c = max(t / 6, t % 6);
            pk = r * 6 - r * (r - 1) / 2 + (c - r);
        } else {
            pk = 21 + (t - 36);
        }
        for (int q = 0; q < CAM_CHUNKS; q++) cam += a.campart[((long long)h * CAM_CHUNKS + q) * 27 + pk];
        for (int i = 0; i < a.nt; i++) {
            const Tether& T = a.teth[i];
            if (!T.active) continue;
            for (int vtx = 0; vtx < 2; vtx++) {
                if ((vtx ? T.h2 : T.h1) != h) continue;
                const double* o = a.tout + (long long)i * TETHER_OUT;
                cam += t < 36 ? o[36 * vtx + r * 6 + c] : o[108 + 6 * vtx + (t - 36)];
            }
        }
        if (t < 36) a.Hpp[36 * (long long)pr.c1 + t] = cam;
        else a.bp[6 * pr.c1 + (t - 36)] = cam;
    }
    schur_write(pr, t, v, cam, a.lambda, np, a.ptlist, a.tout, a.S, a.rhs);
}

__global__ __launch_bounds__(64) void schur_finish(FinishArgs a, int np)
{
    const SchurPair pr = a.pairs[a.flist[blockIdx.x]];
    if (threadIdx.x < 42) finish_entry(a, pr, threadIdx.x, np);
}

// Dense SPD solve S x = b in one workgroup, S of padded order np (multiple of 16, rows n..np-1
// set to identity here).  Right-looking Cholesky with 16-wide panels:
//   (1) the 16x16 diagonal block is factored in one wave's registers (shuffles, no barriers),
//   (2) panel TRSM one row per thread into an LDS copy of the panel,
//   (3) trailing update A22 -= L21 L21^T on f64 MFMA 16x16x4 tiles (lower triangle only).
// Then forward / backward substitution, each 16-block solved by one wave with shuffles.
constexpr int CH_THREADS = 1024;
constexpr int CH_WAVES = CH_THREADS / kWave;
constexpr int NB = 16;
constexpr int CH_PANEL_ROWS = 576;  // 96 free cameras
static_assert(CH_PANEL_ROWS / 6 == MAX_FREE_CAMS, "free-camera limit");

typedef double dbl4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(CH_THREADS) void cholesky_solve(double* __restrict__ S, int np, int n,
                                                             const double* __restrict__ b,
                                                             double* __restrict__ x,
                                                             int* __restrict__ fail)
{
    __shared__ double L11[NB][NB + 1];
    __shared__ double panel[CH_PANEL_ROWS][NB + 1];
    __shared__ double yv[NB];
    __shared__ int s_fail;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    for (long long idx = tid; idx < (long long)(np - n) * np; idx += CH_THREADS) {
        const int i = n + (int)(idx / np), k = (int)(idx % np);
        S[(long long)i * np + k] = (i == k) ? 1.0 : 0.0;
    }
    if (tid == 0) s_fail = 0;
    __syncthreads();
    for (int kb = 0; kb < np; kb += NB) {
        if (wave == 0) {
            const int l = lane;
            double a[NB];
#pragma unroll
            for (int k = 0; k < NB; k++) a[k] = (l < NB && k <= l) ? S[(long long)(kb + l) * np + kb + k] : 0.0;
            bool bad = false;
#pragma unroll
            for (int j = 0; j < NB; j++) {
                const double djj = __shfl(a[j], j);
                if (!(djj > 0)) bad = true;
                const double d = sqrt(djj);
                if (l == j) a[j] = d;
                if (l > j) a[j] = a[j] / d;
#pragma unroll
                for (int k = j + 1; k < NB; k++) {
                    const double lkj = __shfl(a[j], k);
                    if (l >= k) a[k] -= a[j] * lkj;
                }
            }
            if (l < NB) {
#pragma unroll
                for (int k = 0; k < NB; k++) {
                    L11[l][k] = k <= l ? a[k] : 0.0;
                    if (k <= l) S[(long long)(kb + l) * np + kb + k] = a[k];
                }
            }
            if (l == 0 && bad) s_fail = 1;
        }
        __syncthreads();
        if (s_fail) break;
        const int r0 = kb + NB, m = np - r0;
        for (int i = r0 + tid; i < np; i += CH_THREADS) {
            // keeps hipcc from hoisting the 136 loop-invariant L11 reads into registers (spills)
            asm volatile("" ::: "memory");
            double v[NB];
#pragma unroll
            for (int j = 0; j < NB; j++) v[j] = S[(long long)i * np + kb + j];
#pragma unroll
            for (int j = 0; j < NB; j++) {
                double s = v[j];
#pragma unroll
                for (int k = 0; k < j; k++) s -= v[k] * L11[j][k];
                v[j] = s / L11[j][j];
            }
#pragma unroll
            for (int j = 0; j < NB; j++) {
                S[(long long)i * np + kb + j] = v[j];
                panel[i - r0][j] = v[j];
            }
        }
        __syncthreads();
        const int mt = m / NB;
        const int ntiles = mt * (mt + 1) / 2;
        for (int t = wave; t < ntiles; t += CH_WAVES) {
            int ti = 0, rem = t;
            while (rem > ti) {
                rem -= ti + 1;
                ti++;
            }
            const int tk = rem;
            const int col = lane & 15, rb = lane >> 4;
            dbl4 c;
#pragma unroll
            for (int r = 0; r < 4; r++) c[r] = S[(long long)(r0 + ti * NB + rb + 4 * r) * np + r0 + tk * NB + col];
#pragma unroll
            for (int kk = 0; kk < NB / 4; kk++) {
                const double av = -panel[ti * NB + (lane & 15)][kk * 4 + (lane >> 4)];
                const double bv = panel[tk * NB + (lane & 15)][kk * 4 + (lane >> 4)];
                c = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, c, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 4; r++) S[(long long)(r0 + ti * NB + rb + 4 * r) * np + r0 + tk * NB + col] = c[r];
        }
        __syncthreads();
    }
    if (s_fail) {
        if (tid == 0) *fail = 1;
        return;
    }
    for (int i = tid; i < np; i += CH_THREADS) x[i] = i < n ? b[i] : 0.0;
    __syncthreads();
    // forward: L y = b
    for (int kb = 0; kb < np; kb += NB) {
        if (wave == 0) {
            const int l = lane & 15;
            double Lrow[NB];
#pragma unroll
            for (int k = 0; k < NB; k++) Lrow[k] = S[(long long)(kb + l) * np + kb + k];
            double s = x[kb + l], y = 0;
#pragma unroll
            for (int j = 0; j < NB; j++) {
                const double yj = __shfl(s / Lrow[j], j);
                if (l == j) y = yj;
                if (l > j) s -= Lrow[j] * yj;
            }
            if (lane < NB) {
                x[kb + l] = y;
                yv[l] = y;
            }
        }
        __syncthreads();
        for (int i = kb + NB + tid; i < np; i += CH_THREADS) {
            double s = 0;
#pragma unroll
            for (int j = 0; j < NB; j++) s += S[(long long)i * np + kb + j] * yv[j];
            x[i] -= s;
        }
        __syncthreads();
    }
    // backward: L^T x = y
    for (int kb = np - NB; kb >= 0; kb -= NB) {
        if (wave == 0) {
            const int l = lane & 15;
            double Lcol[NB];  // Lcol[k] = L[kb+k][kb+l]
#pragma unroll
            for (int k = 0; k < NB; k++) Lcol[k] = S[(long long)(kb + k) * np + kb + l];
            double s = x[kb + l], y = 0;
#pragma unroll
            for (int j = NB - 1; j >= 0; j--) {
                const double yj = __shfl(s / Lcol[j], j);
                if (l == j) y = yj;
                if (l < j) s -= Lcol[j] * yj;
            }
            if (lane < NB) {
                x[kb + l] = y;
                yv[l] = y;
            }
        }
        __syncthreads();
        for (int i = tid; i < kb; i += CH_THREADS) {
            double s = 0;
#pragma unroll
            for (int j = 0; j < NB; j++) s += S[(long long)(kb + j) * np + i] * yv[j];
            x[i] -= s;
        }
        __syncthreads();
    }
}

// Register-resident tiled Cholesky + solve for np <= 240 (the usual local-BA window: 40 free
// keyframes -> n = 240; larger systems use cholesky_solve).  S = U^T U in upper form: the upper
// 16x16 tiles (i <= j) of S live in the f64 MFMA accumulator layout of 15 tile waves (slots from
// the host's chol_tile_table; lane l holds rows (l >> 4) + 4r, column l & 15) next to one factor
// wave that holds no tile.  Every product sums over a tile's row index, which is exactly the B
// operand of v_mfma_f64_16x16x4f64 taken from those registers (k-step q = register q):
//   TRSM  U_kj = inv(L_kk) A_kj            (A operand inv(L_kk) from LDS; L = U^T)
//   SYRK  A_ij -= U_ki^T U_kj, k < i <= j  (both operands from the LDS panel of row-block k)
// Step k (tile waves): TRSM of row-block k into the double-buffered panel — the owner of (k, k+1)
// also owns (k+1, k+1): it solves (k, k+1) first, applies that tile's update to (k+1, k+1) and
// hands A_{k+1,k+1} to the factor wave (LDS + flag) — then the tile waves' own barrier (an LDS
// counter), the SYRKs, and the workgroup barrier.  The factor wave factors block k+1 (Cholesky +
// triangular inverse + forward substitution in one column loop) as soon as it is handed over,
// concurrently with the TRSM and SYRK phases, and meets the tile waves only at the end of the step.
// Factor wave and tile waves run separate code paths, so the factor's registers never add to the
// resident tiles'.  Measured at n = 240 (tools/ablate_ba.py): 95 us with 8 waves and the factor
// after the SYRK barrier, 74 us now (16 waves, 4 per SIMD).  Nothing of S leaves the chip between
// steps; the solves use the per-block inverses kept in LDS.
constexpr int CT_WAVES = 16;  // 4 per SIMD (15 tile waves x 8 resident tiles + the factor wave)
constexpr int CT_THREADS = CT_WAVES * kWave;
constexpr int CT_TW = CT_WAVES - 1;  // tile waves (wave CT_TW: the factor wave, which holds no tile)
constexpr int CT_MAXT = 15;
constexpr int CT_TPW = (CT_MAXT * (CT_MAXT + 1) / 2 + CT_TW - 1) / CT_TW;  // tiles per tile wave: 7 x 18 >= 120 upper tiles of np = 240
static_assert(CT_TW * CT_TPW >= CT_MAXT * (CT_MAXT + 1) / 2, "every upper tile has a slot");

// Broadcast of lane l's double (two v_readlane_b32: scalar result, no LDS crossbar).
__device__ __forceinline__ double readlane_f64(double v, int l)
{
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(u & 0xFFFFFFFFull), l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(u >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// One double through a 32-bit DPP move per half (bound_ctrl: lanes shifted in from outside the
// row read 0).
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v)
{
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(u & 0xFFFFFFFFull), CTRL, 0xF, 0xF, true);
    const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(u >> 32), CTRL, 0xF, 0xF, true);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
// Inclusive prefix sum over the 16 lanes of a DPP row (row_shr 1, 2, 4, 8): lane 15 of the row
// ends with the row total.
__device__ __forceinline__ double row_sum16(double v)
{
    v += dpp_f64<0x111>(v);
    v += dpp_f64<0x112>(v);
    v += dpp_f64<0x114>(v);
    v += dpp_f64<0x118>(v);
    return v;
}

__device__ __forceinline__ int upper_tile_index(int i, int j, int mt) { return i * mt - i * (i - 1) / 2 + (j - i); }

__global__ __launch_bounds__(CT_THREADS) void chol_tiles(const double* __restrict__ S, int np, int n,
                                                         const double* __restrict__ b, double* __restrict__ x,
                                                         int* __restrict__ fail, const uint16_t* __restrict__ tab)
{
    // inverse of L_kk = U_kk^T per diagonal block, column-major: invT[k][c][m] = inv(L_kk)[m][c]
    // (the factor writes a column with 16-byte stores; 18-double rows keep them aligned and the
    // MFMA / solve readers conflict-free)
    __shared__ __attribute__((aligned(16))) double invT[CT_MAXT][16][18];
    __shared__ double pan[2][CT_MAXT][16][17];    // U row-block k tiles (k, j)
    __shared__ __attribute__((aligned(16))) double dsc[16][18];  // the factor's scratch: A_kk transposed
    __shared__ __attribute__((aligned(16))) double vb[CT_MAXT * 16];  // b -> y -> x
    __shared__ int s_fail;
    __shared__ unsigned s_tile_bar;   // the TRSM-phase barrier count (CT_TW + 1 arrivals per step)
    __shared__ double cst[16][17], dst[16][17];  // A_{k,k+1}, A_{k+1,k+1} staged for the factor wave
    __shared__ uint16_t s_nz[CT_MAXT];  // structural row masks of U (chol_tile_table)
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: tile bookkeeping on the SALU
    const int mt = np >> 4, T = mt * (mt + 1) / 2;
    const int lr = lane >> 4, lc = lane & 15;  // accumulator layout: rows lr + 4r, column lc

    // tile coordinates of each slot (wave uniform, scalar registers), from the host's table
    // (chol_tile_table: tiles (d-1, d) and (d, d) share an owner)
    int tIJ[CT_TPW];  // ti | tj << 8, one scalar register per slot
#pragma unroll
    for (int sl = 0; sl < CT_TPW; sl++) {
        const int v = wave < CT_TW ? (int)tab[wave * CT_TPW + sl] : 0xFFFF;  // the factor wave holds no tile
        tIJ[sl] = v == 0xFFFF ? (mt | mt << 8) : v;                           // mt: no tile
    }
    (void)T;
    auto tile_of = [&](int sl, int& ti, int& tj) {
        ti = tIJ[sl] & 0xFF;
        tj = tIJ[sl] >> 8;
    };
    // --- the 16x16 diagonal block factor (the factor wave), from dsc ---
    auto factor_diag = [&](int k) {  // from dsc
        const int l = lane;
        // Right-looking Cholesky of the 16x16 block with the triangular inverse and the
        // forward substitution fused into the same column loop, one register array v[] over
        // three lane groups that all take the same update v[q] -= v[j] L[q][j]:
        //   lanes 0-15:  row l of A -> row l of L (entries above the diagonal are never read)
        //   lanes 16-31: column l-16 of I -> column l-16 of inv(L)
        //   lane 32:     vb_k (final: every block above has updated it) -> y_k, in place
        // Column j's L[q][j] are broadcast once with v_readlane (scalar registers).  Lane j's
        // own v[j] is the pivot d, so v[j] *= 1/sqrt(d) yields sqrt(d) there with no select.
        // (An LDS column broadcast instead measured 2x slower.)
        double v[16];
        const double* vbk = &vb[16 * k];
        const int c = l - 16;
        // one batch of unconditional 16-byte loads from a per-lane source (row l of A for
        // lanes 0-15, vb_k for the others), then per-lane selects
        double dq[16];
        {
            const double2* dr = reinterpret_cast<const double2*>(l < 16 ? &dsc[l][0] : vbk);
#pragma unroll
            for (int q = 0; q < 8; q++) {
                const double2 d2 = dr[q];
                dq[2 * q] = d2.x;
                dq[2 * q + 1] = d2.y;
            }
        }
#pragma unroll
        for (int q = 0; q < 16; q++)
            v[q] = l < 16 ? (q <= l ? dq[q] : 0.0) : (l < 32 ? (q == c ? 1.0 : 0.0) : (l == 32 ? dq[q] : 0.0));
        bool bad = false;
        // 1/sqrt by v_rsq_f64 + one Newton step (~1e-14 relative, no f64 sqrt / division
        // sequence on the column's critical path)
        auto rsq_newton = [&](double d) {
            if (!(d > 0)) bad = true;
            const double h = 0.5 * d;
            double r = __builtin_amdgcn_rsq(d);
            return r * __builtin_fma(-h * r, r, 1.5);
        };
        // Look-ahead: column j + 1 is updated first and its pivot's 1/sqrt chain starts right
        // away, so the chain (readlane -> rsq -> Newton -> scale, a run of dependent f64 ops)
        // overlaps the rest of column j's update instead of following it in issue order.
        double r = rsq_newton(readlane_f64(v[0], 0));
#pragma unroll
        for (int j = 0; j < 16; j++) {
            v[j] *= r;
            if (j < 15) {
                const double l1 = readlane_f64(v[j], j + 1);
                v[j + 1] = __builtin_fma(-v[j], l1, v[j + 1]);
                const double rn = rsq_newton(readlane_f64(v[j + 1], j + 1));
                double lq[16];
#pragma unroll
                for (int q = j + 2; q < 16; q++) lq[q] = readlane_f64(v[j], q);
#pragma unroll
                for (int q = j + 2; q < 16; q++) v[q] = __builtin_fma(-v[j], lq[q], v[q]);
                r = rn;
            }
            __builtin_amdgcn_sched_barrier(0);  // keep each column's broadcasts in its own window
        }
        if (l == 0 && bad) s_fail = 1;
        if (l >= 16 && l < 32) {
            double2* o = reinterpret_cast<double2*>(&invT[k][c][0]);
#pragma unroll
            for (int m = 0; m < 8; m++) o[m] = double2{v[2 * m], v[2 * m + 1]};
        }
        if (l == 32) {  // y_k replaces b_k in the solution vector
            double2* o = reinterpret_cast<double2*>(&vb[16 * k]);
#pragma unroll
            for (int m = 0; m < 8; m++) o[m] = double2{v[2 * m], v[2 * m + 1]};
        }
    };
    auto solve_block = [&](int k) {  // by one wave: vb_k := inv(U_kk) vb_k, inv(U) = inv(L)^T
        double xv = 0;
        if (lane < 16) {
            const double2* ir = reinterpret_cast<const double2*>(&invT[k][lane][0]);
            const double2* vr = reinterpret_cast<const double2*>(&vb[16 * k]);
#pragma unroll
            for (int c = 0; c < 8; c++) {
                const double2 a = ir[c], v2 = vr[c];
                xv += a.x * v2.x;
                xv += a.y * v2.y;
            }
        }
        __builtin_amdgcn_wave_barrier();
        if (lane < 16) vb[16 * k + lane] = xv;
    };
    if (wave == CT_TW) {
        // ===== the factor wave: it holds no tile, so none of the tile registers are live here.
        // Per step k it runs the critical chain alone: TRSM of (k, k+1) with its own inv(L_kk),
        // the update of (k+1, k+1) by it, and the factor of block k+1; the tile waves stage both
        // tiles for it at the end of step k-1 ---
        if (lane == 0) {
            s_fail = 0;
            s_tile_bar = 0;
        }
        dbl4 cA = {0, 0, 0, 0}, cD = {0, 0, 0, 0};  // A_{k,k+1}, A_{k+1,k+1} (accumulator layout)
        auto s_tile = [&](int ti, int tj) {  // tile (ti, tj) of S, padded with the identity
            dbl4 t;
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int row = 16 * ti + lr + 4 * r, col = 16 * tj + lc;
                t[r] = (row < n && col < n) ? S[(long long)row * np + col] : (row == col ? 1.0 : 0.0);
            }
            return t;
        };
        if (mt > 0) {
            // block 0 from S directly while the tile waves load their tiles (A_00 goes to dsc
            // transposed, as stage_diag writes it)
            if (lane < 16) {
#pragma unroll
                for (int q = 0; q < 16; q++)
                    dsc[lane][q] = (q < n && lane < n) ? S[(long long)q * np + lane] : (q == lane ? 1.0 : 0.0);
                vb[lane] = lane < n ? b[lane] : 0.0;
            }
            if (mt > 1) {
                cA = s_tile(0, 1);
                cD = s_tile(1, 1);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            factor_diag(0);
        }
        __syncthreads();  // tiles loaded, block 0 factored
        for (int k = 0; k < mt; k++) {
            if (s_fail) break;
            const int kn = k + 1, buf = k & 1;
            if (kn < mt) {
                if (k > 0)
#pragma unroll
                    for (int r = 0; r < 4; r++) {
                        cA[r] = cst[lr + 4 * r][lc];
                        cD[r] = dst[lr + 4 * r][lc];
                    }
                __builtin_amdgcn_s_setprio(3);  // the critical chain first on this SIMD
                // TRSM U_{k,k+1} = inv(L_kk) A_{k,k+1} into the panel, y_{k+1} -= U^T y_k
                dbl4 acc = {0, 0, 0, 0};
#pragma unroll
                for (int q = 0; q < 4; q++)
                    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(invT[k][4 * q + lr][lc], cA[q], acc, 0, 0, 0);
#pragma unroll
                for (int r = 0; r < 4; r++) pan[buf][kn][lr + 4 * r][lc] = acc[r];
                double pacc = 0;
#pragma unroll
                for (int r = 0; r < 4; r++) pacc = __builtin_fma(acc[r], vb[16 * k + lr + 4 * r], pacc);
                pacc += __shfl_xor(pacc, 16);
                pacc += __shfl_xor(pacc, 32);
                if (lr == 0) vb[16 * kn + lc] -= pacc;
                // arrive at the TRSM-phase barrier (row-block k of the panel)
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                if (lane == 0) __hip_atomic_fetch_add(&s_tile_bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __builtin_amdgcn_wave_barrier();  // U_{k,k+1} in the panel, read across lanes below
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                // A_{k+1,k+1} -= U^T U, into dsc transposed
#pragma unroll
                for (int q = 0; q < 4; q++)
                    cD = __builtin_amdgcn_mfma_f64_16x16x4f64(-pan[buf][kn][4 * q + lr][lc], pan[buf][kn][4 * q + lr][lc], cD,
                                                             0, 0, 0);
#pragma unroll
                for (int r = 0; r < 4; r++) dsc[lc][lr + 4 * r] = cD[r];
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                factor_diag(kn);
                __builtin_amdgcn_s_setprio(0);
            } else {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                if (lane == 0) __hip_atomic_fetch_add(&s_tile_bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            __syncthreads();  // end of step k
        }
        if (s_fail) return;
        for (int k = 0; k < (mt > 0 ? mt : 1); k++) __syncthreads();  // the backward solve's barriers
        return;
    }

    // ===== the tile waves =====
    dbl4 C[CT_TPW];
#pragma unroll
    for (int sl = 0; sl < CT_TPW; sl++) {
        int ti, tj;
        tile_of(sl, ti, tj);
        if (ti < mt) {
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int row = 16 * ti + lr + 4 * r, col = 16 * tj + lc;
                C[sl][r] = (row < n && col < n) ? S[(long long)row * np + col] : (row == col ? 1.0 : 0.0);
            }
        } else {
            C[sl] = dbl4{0, 0, 0, 0};
        }
    }
    if (tid < CT_MAXT) s_nz[tid] = tab[CT_TW * CT_TPW + tid];
    // b -> vb (block 0's entries are the factor wave's: it turns them into y_0)
    constexpr int TT = CT_TW * kWave;  // tile-wave threads
    for (int i = 16 + tid; i < np; i += TT) vb[i] = i < n ? b[i] : 0.0;
    __syncthreads();  // tiles loaded, block 0 factored
    for (int k = 0; k < mt; k++) {
        const int buf = k & 1;
        if (s_fail) break;
        const int kn = k + 1;
        // --- TRSM: U_kj = inv(L_kk) A_kj for the owned tiles of row-block k but (k, k+1), which
        // the factor wave solves ---
        auto trsm = [&](int sl) {
            const int tj = tIJ[sl] >> 8;
            dbl4 acc = {0, 0, 0, 0};
#pragma unroll
            for (int q = 0; q < 4; q++)
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(invT[k][4 * q + lr][lc], C[sl][q], acc, 0, 0, 0);
            C[sl] = acc;
#pragma unroll
            for (int r = 0; r < 4; r++) pan[buf][tj][lr + 4 * r][lc] = acc[r];
            // forward substitution: vb_j -= U_kj^T y_k (tile (k, j) is the only writer of
            // vb_j in this step)
            double pacc = 0;
#pragma unroll
            for (int r = 0; r < 4; r++) pacc = __builtin_fma(acc[r], vb[16 * k + lr + 4 * r], pacc);
            pacc += __shfl_xor(pacc, 16);
            pacc += __shfl_xor(pacc, 32);
            if (lr == 0) vb[16 * tj + lc] -= pacc;
        };
        auto syrk = [&](int sl) {
#pragma unroll
            for (int q = 0; q < 4; q++)
                C[sl] = __builtin_amdgcn_mfma_f64_16x16x4f64(-pan[buf][tIJ[sl] & 0xFF][4 * q + lr][lc],
                                                            pan[buf][tIJ[sl] >> 8][4 * q + lr][lc], C[sl], 0, 0, 0);
        };
        const int chain = k | kn << 8, diag = kn | kn << 8;
#pragma unroll
        for (int sl = 0; sl < CT_TPW; sl++) {
            const int ti = tIJ[sl] & 0xFF, tj = tIJ[sl] >> 8;
            if (ti == k && tj > kn) trsm(sl);
        }
        // the TRSM-phase barrier (an LDS counter: the factor wave arrives after its TRSM of
        // (k, k+1) and goes on to the factor): pan row-block k complete
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) __hip_atomic_fetch_add(&s_tile_bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        while (__hip_atomic_load(&s_tile_bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < (unsigned)((CT_TW + 1) * kn))
            __builtin_amdgcn_s_sleep(1);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#pragma unroll
        for (int sl = 0; sl < CT_TPW; sl++)  // the owner of (k, k+1) keeps U for the backward solve
            if (tIJ[sl] == chain)
#pragma unroll
                for (int r = 0; r < 4; r++) C[sl][r] = pan[buf][kn][lr + 4 * r][lc];
        // --- SYRK: A_ij -= U_ki^T U_kj for the owned tiles with k < i <= j but (k+1, k+1) (the
        // factor wave's) ---
        // (only where both U_ki and U_kj can be nonzero: the envelope of chol_tile_table)
        const unsigned nzk = (unsigned)__builtin_amdgcn_readfirstlane((int)s_nz[k]);
#pragma unroll
        for (int sl = 0; sl < CT_TPW; sl++) {
            const int i = tIJ[sl] & 0xFF, j = tIJ[sl] >> 8;
            if (i > k && i < mt && tIJ[sl] != diag && (nzk >> i & nzk >> j & 1u)) syrk(sl);
        }
        // the next step's chain tiles, now final, to the factor wave
        if (kn + 1 < mt) {
            const int nchain = kn | (kn + 1) << 8, ndiag = (kn + 1) | (kn + 1) << 8;
#pragma unroll
            for (int sl = 0; sl < CT_TPW; sl++) {
                if (tIJ[sl] == nchain)
#pragma unroll
                    for (int r = 0; r < 4; r++) cst[lr + 4 * r][lc] = C[sl][r];
                if (tIJ[sl] == ndiag)
#pragma unroll
                    for (int r = 0; r < 4; r++) dst[lr + 4 * r][lc] = C[sl][r];
            }
        }
        __syncthreads();  // block k+1 factored (invT, y_{k+1}), every SYRK of step k done
    }
    if (s_fail) {
        if (tid == 0) *fail = 1;
        return;
    }
    // --- backward: U x = y, x_k = inv(U_kk) (y_k - sum_{j>k} U_kj x_j), right-looking with
    // one barrier per block: the owner of tile (k-1, k) applies the last update of y_{k-1} and
    // then solves block k-1 itself ---
    if (mt > 0 && wave == 0) solve_block(mt - 1);
    __syncthreads();
    for (int k = mt - 1; k >= 1; k--) {
        // slots in reverse (row-major) order: the tile (k - 1, k) of the critical chain first
#pragma unroll
        for (int sl = CT_TPW - 1; sl >= 0; sl--) {
            int ti, tj;
            tile_of(sl, ti, tj);
            if (tj == k && ti < k) {
                // (U_ik x_k)[r] = sum_c U_ik[r][c] x_k[c]: row sums over the 16 lanes of a DPP row
                // (lane 15 of the row holds rows lr + 4r)
                const double xk = vb[16 * k + lc];
                double rs[4];
#pragma unroll
                for (int r = 0; r < 4; r++) rs[r] = row_sum16(C[sl][r] * xk);
                if (lc == 15)
#pragma unroll
                    for (int r = 0; r < 4; r++) vb[16 * ti + lr + 4 * r] -= rs[r];
                if (ti == k - 1) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    solve_block(k - 1);
                }
            }
        }
        __syncthreads();
    }
    for (int i = tid; i < np; i += TT) x[i] = i < n ? vb[i] : 0.0;
}

// Back-substitution, the trial state and its evaluation in one launch.  Blocks [0, npb): a
// PG-lane group per point: xl = Dinv (bl - sum_e Hpl_e^T xp[h(e)]) = Dinv bl - sum_e Z_e^T xp[h(e)]
// (Dinv symmetric; Z_e^T xp = G_e^T (Jp_e xp)), trial point B.p = A.p + xl (copy for points
// outside the system), the point part of computeScale, then the trial errors + robust chi2 of the
// point's edges with the speculative StepBundleAdjustment post-pass for both candidate states
// (cheirality + maxErrorSquare, outlier appends, inlier block partials).  Each lane forms its
// edge's trial camera pose exp(xp) * T itself (the same d_oplus the camera threads store), so the
// evaluation needs no second launch.  The remaining blocks: thread per camera, trial pose
// (VertexSE3Expmap::oplusImpl) or copy, and the camera part of computeScale.
__global__ __launch_bounds__(BA_THREADS) void update_evaluate(Problem pb, const double* __restrict__ G,
                                                              const double* __restrict__ Q,
                                                              const double* __restrict__ Hll,
                                                              const double* __restrict__ bl,
                                                              const double* __restrict__ xp, double lambda,
                                                              State A, State B, const double* __restrict__ bp,
                                                              double* __restrict__ scale_part, int npb, PointOut o,
                                                              SpecPass sp)
{
    if ((int)blockIdx.x >= npb) {
        const int i = (blockIdx.x - npb) * BA_THREADS + threadIdx.x;
        if (i >= pb.C) return;
        double q[4] = {A.q[4 * i], A.q[4 * i + 1], A.q[4 * i + 2], A.q[4 * i + 3]};
        double t[3] = {A.t[3 * i], A.t[3 * i + 1], A.t[3 * i + 2]};
        const int h = pb.camh[i];
        double sc = 0;
        if (h >= 0) {
            double u[6];
            for (int k = 0; k < 6; k++) {
                u[k] = xp[6 * h + k];
                sc += u[k] * (lambda * u[k] + bp[6 * i + k]);
            }
            d_oplus(q, t, u);
        }
        for (int k = 0; k < 4; k++) B.q[4 * i + k] = q[k];
        for (int k = 0; k < 3; k++) B.t[3 * i + k] = t[k];
        scale_part[pb.P + i] = sc;
        return;
    }
    const int gid = blockIdx.x * BA_THREADS + threadIdx.x;
    const int p = gid / PG, sub = gid % PG;
    double vs[2] = {0, 0}, vc[2] = {0, 0};
    if (p < pb.P) {  // whole groups
        double X[3] = {A.p[3 * p], A.p[3 * p + 1], A.p[3 * p + 2]};
        double sc = 0;
        const long long es = pb.ecsr;
        const int e0 = pb.pstart[p], e1 = pb.pstart[p + 1];
        // With at most PG edges (one per lane) the lane keeps its edge (index, camera, block,
        // camera update) from the first pass for the evaluation pass: no dependent reload of
        // pedges / active / ecam / camh / xp after the group reduction.
        const bool one = e1 - e0 <= PG;
        int c_e = -1, c_c = 0, c_h = -1;
        double c_u[6] = {0, 0, 0, 0, 0, 0};
        int c_pos = 0;
        if (one && e0 + sub < e1) {
            const int4 ent = pb.pe[e0 + sub];
            c_e = ent.x;
            c_c = ent.y;
            c_h = ent.z;
            c_pos = ent.w;
            if (c_h >= 0)
#pragma unroll
                for (int k = 0; k < 6; k++) c_u[k] = xp[6 * c_h + k];
            if (!pb.active[c_e]) c_e = -1;
        }
        if (pb.ptfree[p]) {
            // Hll_p and bl_p are loaded ahead of the edge pass (independent of it)
            double D[9], Di[9];
#pragma unroll
            for (int k = 0; k < 9; k++) D[k] = Hll[9 * (long long)p + k];
            const double b0 = bl[3 * p], b1 = bl[3 * p + 1], b2 = bl[3 * p + 2];
            double cl[3] = {0, 0, 0};
            auto add_edge = [&](int a2, int c, const double (&Xp)[6]) {
                double J[12];
                jac_pose_q(Q[a2], Q[es + a2], Q[2 * es + a2], pb.camk[3 * c], J);
                double u0 = 0, u1 = 0;
#pragma unroll
                for (int r = 0; r < 6; r++) {
                    u0 += J[r] * Xp[r];
                    u1 += J[6 + r] * Xp[r];
                }
#pragma unroll
                for (int k = 0; k < 3; k++) cl[k] += G[k * es + a2] * u0 + G[(3 + k) * es + a2] * u1;
            };
            if (one) {
                if (c_e >= 0 && c_h >= 0) add_edge(c_pos, c_c, c_u);
            } else {
                for (int a = e0 + sub; a < e1; a += PG) {
                    const int4 ent = pb.pe[a];
                    if (!pb.active[ent.x] || ent.z < 0) continue;
                    double Xp[6];
#pragma unroll
                    for (int r = 0; r < 6; r++) Xp[r] = xp[6 * ent.z + r];
                    add_edge(ent.w, ent.y, Xp);
                }
            }
            group_sum(cl);  // every lane of the group holds the sums
            // db_p = Dinv_p bl_p, Dinv_p = (Hll_p + lambda I)^-1 as in edge_schur
            D[0] += lambda;
            D[4] += lambda;
            D[8] += lambda;
            d_inv3(D, Di);
            for (int r = 0; r < 3; r++) {
                const double dbr = Di[3 * r] * b0 + Di[3 * r + 1] * b1 + Di[3 * r + 2] * b2;
                const double v = dbr - cl[r];
                X[r] += v;
                sc += v * (lambda * v + bl[3 * p + r]);
            }
        }
        if (sub == 0) {
            for (int k = 0; k < 3; k++) B.p[3 * p + k] = X[k];
            scale_part[p] = sc;
        }
        double chi = 0;
        for (int a = e0 + sub; a < e1; a += PG) {
            int e, c, h;
            double u[6];
            if (one) {
                e = c_e;
                if (e < 0) continue;
                c = c_c;
                h = c_h;
#pragma unroll
                for (int k = 0; k < 6; k++) u[k] = c_u[k];
            } else {
                const int4 ent = pb.pe[a];
                e = ent.x;
                if (!pb.active[e]) continue;
                c = ent.y;
                h = ent.z;
                if (h >= 0)
#pragma unroll
                    for (int k = 0; k < 6; k++) u[k] = xp[6 * h + k];
            }
            double q[4] = {A.q[4 * c], A.q[4 * c + 1], A.q[4 * c + 2], A.q[4 * c + 3]};
            double t[3] = {A.t[3 * c], A.t[3 * c + 1], A.t[3 * c + 2]};
            if (h >= 0) d_oplus(q, t, u);
            double ev[2], xc[3], rho0, rho1;
            edge_eval_at(pb, e, c, q, t, X, ev, xc, rho0, rho1);
            o.err[2 * e] = ev[0];
            o.err[2 * e + 1] = ev[1];
            chi += rho0;
            if (sp.on) {
                const double sumSquares = ev[0] * ev[0] + ev[1] * ev[1];
#pragma unroll
                for (int k = 0; k < 2; k++) {
                    const double dot = k == 0 ? cheirality_at(q, t, X) : cheirality(sp.cur, c, p);
                    if (dot <= 0 || sumSquares > sp.maxErrSq) {
                        sp.out_list[(long long)k * sp.E + atomicAdd(&sp.ctl->count[k], 1u)] = (uint32_t)e;
                    } else {
                        vs[k] += sumSquares;
                        vc[k] += 1;
                    }
                }
            }
        }
        double cv[1] = {chi};
        group_sum(cv);
        if (sub == 0) o.chi_part[p] = cv[0];
    }
    if (!sp.on) return;
    __shared__ double red[BA_THREADS / kWave][4];
    double v4[4] = {vs[0], vc[0], vs[1], vc[1]};
    block_sum<4>(v4, red);
    if (threadIdx.x < 4) sp.part[(long long)threadIdx.x * npb + blockIdx.x] = red[0][threadIdx.x];
}

// StepBundleAdjustment post-pass (BundlerLib.cpp:385-446) per active edge using the stored
// errors: an edge behind the camera or with |e|^2 > maxErrorSquare is an outlier (index appended;
// the host sorts the short list into g2o's active-edge order and drop_edges removes them).
// Read-only on the graph, so it runs speculatively with the last trial for NS candidate states
// at once (ns = 2: the trial state if accepted, the current state if rejected); list k lives at
// out_list + k E.  Block partials (sum of inlier |e|^2, inlier count) go to `part`; reduce3 adds
// them in fixed order into ctl->osum[k].
__global__ __launch_bounds__(BA_THREADS) void outlier_pass(Problem pb, State s0, State s1, int ns, int E,
                                                           const unsigned char* __restrict__ active,
                                                           const double* __restrict__ err,
                                                           double maxErrSq,
                                                           uint32_t* __restrict__ out_list,
                                                           double* __restrict__ part,  // [ns][2][gridDim.x]
                                                           LiveCtl* __restrict__ ctl)
{
    __shared__ double ssum[2][BA_THREADS / kWave], scnt[2][BA_THREADS / kWave];
    const int e = blockIdx.x * BA_THREADS + threadIdx.x;
    double vs[2] = {0, 0}, vc[2] = {0, 0};
    if (e < E && active[e]) {
        const double e0 = err[2 * e], e1 = err[2 * e + 1];
        const double sumSquares = e0 * e0 + e1 * e1;
        const int c = pb.ecam[e], p = pb.ept[e];
        for (int k = 0; k < ns; k++) {
            const State& s = k == 0 ? s0 : s1;
            // SE3Quat::inverse: q*, -(q* t); forward = q* (0,0,1)
            const double qc[4] = {-s.q[4 * c], -s.q[4 * c + 1], -s.q[4 * c + 2], s.q[4 * c + 3]};
            const double tt[3] = {s.t[3 * c], s.t[3 * c + 1], s.t[3 * c + 2]};
            double it[3], fwd[3];
            d_qrot(qc, tt, it);
            const double z[3] = {0, 0, 1};
            d_qrot(qc, z, fwd);
            const double dot = (s.p[3 * p] + it[0]) * fwd[0] + (s.p[3 * p + 1] + it[1]) * fwd[1] +
                               (s.p[3 * p + 2] + it[2]) * fwd[2];
            if (dot <= 0 || sumSquares > maxErrSq) {
                out_list[(long long)k * E + atomicAdd(&ctl->count[k], 1u)] = (uint32_t)e;
            } else {
                vs[k] = sumSquares;
                vc[k] = 1;
            }
        }
    }
    // block partials: wave sums by shuffles, then the waves in order
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    for (int k = 0; k < ns; k++) {
        double a = vs[k], b = vc[k];
        for (int o = kWave / 2; o > 0; o >>= 1) {
            a += __shfl_xor(a, o);
            b += __shfl_xor(b, o);
        }
        if (lane == 0) {
            ssum[k][w] = a;
            scnt[k][w] = b;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 0; k < ns; k++) {
            double a = 0, b = 0;
            for (int i = 0; i < BA_THREADS / kWave; i++) {
                a += ssum[k][i];
                b += scnt[k][i];
            }
            part[(2 * k) * gridDim.x + blockIdx.x] = a;
            part[(2 * k + 1) * gridDim.x + blockIdx.x] = b;
        }
    }
    // the block partials are added by reduce3 (the next launch): a last-block ticket here would
    // need an agent-scope fence per workgroup, i.e. a full L2 write-back on gfx950
}

// removeEdge for the listed observations (thread per removed edge): the edge leaves the active set
// and its point's active-edge count drops; the point leaves the system with its last edge
// (SparseOptimizer::initializeOptimization keeps only vertices with active edges).  Cameras' counts
// are kept by the host, which decides whether the block numbering must be rebuilt.  The Schur
// product lists keep the removed edges' entries: their W / G records are zero from the next
// linearisation on.
__global__ __launch_bounds__(BA_THREADS) void drop_edges(const int* __restrict__ ept,
                                                         const uint32_t* __restrict__ list, uint32_t n,
                                                         unsigned char* __restrict__ active,
                                                         unsigned char* __restrict__ removed,
                                                         int* __restrict__ ptcnt, int* __restrict__ ptfree)
{
    const uint32_t i = blockIdx.x * BA_THREADS + threadIdx.x;
    if (i >= n) return;
    const uint32_t e = list[i];
    active[e] = 0;
    removed[e] = 1;
    const int p = ept[e];
    if (atomicSub(&ptcnt[p], 1) == 1) ptfree[p] = 0;
}

// The initialisation summary into mapped host memory, completion word last (the host spins on it
// instead of a D2H copy + stream synchronisation).
__global__ __launch_bounds__(1024) void summary_out(const int* __restrict__ sum, int n, int* __restrict__ out,
                                                    unsigned* __restrict__ seq_out, unsigned seq)
{
    for (int i = threadIdx.x; i < n; i += 1024) out[i] = sum[i];
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence_system();
        *reinterpret_cast<volatile unsigned*>(seq_out) = seq;
    }
}

// Queued small host-to-device copies in one launch: the sources are in mapped host memory (the
// staging arena), read over the fabric; workgroup b copies GATHER_BLOCK_BYTES of the entry whose
// block range holds b.
constexpr int GATHER_MAX = 12;
constexpr unsigned GATHER_BLOCK_BYTES = 4096;
struct GatherList {
    const char* src[GATHER_MAX];
    char* dst[GATHER_MAX];
    unsigned bytes[GATHER_MAX];
    unsigned first[GATHER_MAX + 1];  // first workgroup of each entry
    int k;
};
__global__ __launch_bounds__(256) void gather_copy(GatherList L)
{
    int i = 0;
    while (i + 1 < L.k && blockIdx.x >= L.first[i + 1]) i++;
    const unsigned base = (blockIdx.x - L.first[i]) * GATHER_BLOCK_BYTES, n = L.bytes[i];
    const unsigned o = base + 16 * threadIdx.x;
    if (o >= n) return;
    const char* s = L.src[i] + o;
    char* d = L.dst[i] + o;
    // the arena offsets are 256-byte aligned and device buffers start aligned: 16-byte moves
    // except for an entry's tail
    if (o + 16 <= n) *reinterpret_cast<uint4*>(d) = *reinterpret_cast<const uint4*>(s);
    else
        for (unsigned j = 0; o + j < n; j++) d[j] = s[j];
}

// Zero-fill of up to 8 word ranges in one launch (instead of one memset call per buffer).
struct ClearList {
    uint32_t* p[8];
    unsigned n[8];  // 32-bit words
    int k;
};
__global__ __launch_bounds__(256) void clear_words(ClearList L)
{
    const unsigned stride = gridDim.x * 256;
    for (int r = 0; r < L.k; r++)
        for (unsigned i = blockIdx.x * 256 + threadIdx.x; i < L.n[r]; i += stride) L.p[r][i] = 0;
}

// ---- SparseOptimizer::initializeOptimization on the device ---------------------------------
// The active edge set, the vertices in the system, the point CSR (edge order) and the camera CSR
// (point order, then edge order) are built from the edge arrays already resident in HBM; the host
// reads back one summary (block count, camera counts, Schur pair counts) per initialisation.
// Summary layout (ints): INIT_HDR header words {nb, free points, active edges, a camera observes a
// point twice}, then per camera its active edge count, then the camera of every free block, then
// per block its free-point edge count, then the nbm x nbm pair counts (row stride nb).
constexpr int INIT_HDR = 8;
constexpr int INIT_LDS_CAMS = 4096;  // per-block camera histograms in LDS up to this many cameras

// Counters the chain accumulates into (per point, per camera, per-point fill cursors) are zero
// between initialisations: their single consumer clears what it read (init_scan, init_psort), so
// no clearing launch precedes the chain.

// Thread per edge: active = not removed and not (points fixed and camera fixed) (the vertices of
// an edge between two fixed vertices leave the system); active edges counted per point (one
// global atomic per distinct point of a wave) and per camera (LDS histogram per block, one global
// atomic per camera).  Also resets the edge's camera-CSR position and its camera sort key (C: an
// inactive tail entry; init_psort overwrites the active positions).
__global__ __launch_bounds__(256) void init_edges(int E, int C, int points_fixed, const int* __restrict__ ecam,
                                                  const int* __restrict__ ept, const unsigned char* __restrict__ removed,
                                                  const unsigned char* __restrict__ camflag,
                                                  unsigned char* __restrict__ active, int* __restrict__ pacc,
                                                  int* __restrict__ cacc, int* __restrict__ epos,
                                                  unsigned* __restrict__ ckey)
{
    extern __shared__ int hist[];
    const bool lds = C <= INIT_LDS_CAMS;
    if (lds)
        for (int c = threadIdx.x; c < C; c += 256) hist[c] = 0;
    __syncthreads();
    const int e = blockIdx.x * 256 + threadIdx.x;
    bool a = false;
    int p = -1;
    if (e < E) {
        const int c = ecam[e];
        p = ept[e];
        a = !removed[e] && !(points_fixed && (camflag[c] & 1));
        active[e] = a ? 1 : 0;
        epos[e] = -1;
        ckey[e] = (unsigned)C;
        if (a) {
            if (lds) atomicAdd(&hist[c], 1);
            else atomicAdd(&cacc[c], 1);
        }
    }
    // one global atomic per distinct point of the wave (a point's edges are usually adjacent:
    // BuildDataForG2O adds them point by point)
    unsigned long long todo = __ballot(a);
    while (todo) {
        const int leader = __ffsll((long long)todo) - 1;
        const int lp = __shfl(p, leader);
        const unsigned long long same = __ballot(a && p == lp);
        if ((int)(threadIdx.x & (kWave - 1)) == leader) atomicAdd(&pacc[lp], __popcll(same));
        todo &= ~same;
    }
    if (!lds) return;
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256)
        if (hist[c]) atomicAdd(&cacc[c], hist[c]);
}

// Exclusive scan of n values by one 1024-thread workgroup (load(i) / store(i, prefix)); returns the total.
template <class T, class Load, class Store>
__device__ T block_scan_1024(int n, Load load, Store store)
{
    __shared__ T ws[1024 / kWave];
    const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
    T carry = 0;
    for (int base = 0; base < n; base += 1024) {
        const int i = base + tid;
        const T v = i < n ? load(i) : T(0);
        T inc = v;
        for (int o = 1; o < kWave; o <<= 1) {
            const T t = __shfl_up(inc, o);
            if (lane >= o) inc += t;
        }
        if (lane == kWave - 1) ws[w] = inc;
        __syncthreads();
        T off = 0, tot = 0;
        for (int k = 0; k < 1024 / kWave; k++) {
            const T sw = ws[k];
            off += k < w ? sw : T(0);
            tot += sw;
        }
        if (i < n) store(i, carry + off + inc - v);
        carry += tot;
        __syncthreads();
    }
    return carry;
}

// One workgroup: point CSR offsets, the points in the system (+ their live edge counts, which
// drop_edges decrements), and how many; camera CSR offsets and counts; the free camera blocks in
// camera order (not fixed, with an active edge or an active tether).  Clears the accumulators it
// read and the per-block rhs counts init_camcsr accumulates.
__global__ __launch_bounds__(1024) void init_scan(int C, int P, int nbm, int points_fixed,
                                                  const unsigned char* __restrict__ camflag, int* __restrict__ pacc,
                                                  int* __restrict__ cacc, int* __restrict__ ptcnt,
                                                  int* __restrict__ pstart, int* __restrict__ ptfree,
                                                  int* __restrict__ cstart, int* __restrict__ camh,
                                                  int* __restrict__ camblk, int* __restrict__ sum)
{
    int* s_ccnt = sum + INIT_HDR;
    int* s_camblk = s_ccnt + C;
    int* s_rc = s_camblk + C;
    // edges per point (low word) and points in the system (high word) in one scan
    const long long pt = block_scan_1024<long long>(
        P, [&](int i) { return (long long)pacc[i] | (pacc[i] > 0 ? 1ll << 32 : 0ll); },
        [&](int i, long long x) {
            const int k = pacc[i];
            pstart[i] = (int)(x & 0xFFFFFFFFll);
            ptcnt[i] = k;
            ptfree[i] = !points_fixed && k > 0;
        });
    const int nact = (int)(pt & 0xFFFFFFFFll), nfp = points_fixed ? 0 : (int)(pt >> 32);
    block_scan_1024<int>(C, [&](int c) { return cacc[c]; },
                    [&](int c, int x) {
                        cstart[c] = x;
                        s_ccnt[c] = cacc[c];
                    });
    auto is_free = [&](int c) { return !(camflag[c] & 1) && (cacc[c] > 0 || (camflag[c] & 2)); };
    const int nb = block_scan_1024<int>(
        C, [&](int c) { return is_free(c) ? 1 : 0; },
        [&](int c, int x) {
            const bool f = is_free(c);
            camh[c] = f ? x : -1;
            if (f) {
                camblk[x] = c;
                s_camblk[x] = c;
            }
        });
    __syncthreads();  // every read of the accumulators is done
    for (int i = threadIdx.x; i < P; i += 1024) pacc[i] = 0;
    for (int c = threadIdx.x; c < C; c += 1024) cacc[c] = 0;
    for (int h = threadIdx.x; h < nbm; h += 1024) s_rc[h] = 0;
    if (threadIdx.x == 0) {
        pstart[P] = nact;
        cstart[C] = nact;
        sum[0] = nb;
        sum[1] = nfp;
        sum[2] = nact;
        sum[3] = 0;
    }
}

// Thread per active edge: its slot in its point's CSR run, one atomic per distinct point of the
// wave (lanes of one point take consecutive slots in lane order; runs split over waves may
// interleave, init_psort orders each run).
__global__ __launch_bounds__(256) void init_pfill(int E, const int* __restrict__ ept, const unsigned char* __restrict__ active,
                                                  const int* __restrict__ pstart, int* __restrict__ pcur,
                                                  int* __restrict__ pedges)
{
    const int e = blockIdx.x * 256 + threadIdx.x;
    const bool a = e < E && active[e];
    const int p = a ? ept[e] : -1;
    const int lane = threadIdx.x & (kWave - 1);
    unsigned long long todo = __ballot(a);
    while (todo) {
        const int leader = __ffsll((long long)todo) - 1;
        const int lp = __shfl(p, leader);
        const unsigned long long same = __ballot(a && p == lp);
        int base = 0;
        if (lane == leader) base = atomicAdd(&pcur[lp], __popcll(same));
        base = __shfl(base, leader);
        if (a && p == lp) pedges[pstart[lp] + base + __popcll(same & ((1ull << lane) - 1ull))] = e;
        todo &= ~same;
    }
}

// One wave per point: its CSR run in edge order — each entry's rank is the number of smaller
// entries of the run (broadcast by shuffles) — then the camera sort keys of its positions and the
// fill cursor back to zero.
constexpr int PSORT_WAVES = 4;
__global__ __launch_bounds__(PSORT_WAVES * kWave) void init_psort(int P, const int* __restrict__ pstart,
                                                                  const int* __restrict__ ecam, int* __restrict__ pcur,
                                                                  int* __restrict__ pedges, unsigned* __restrict__ ckey)
{
    const int p = blockIdx.x * PSORT_WAVES + (int)(threadIdx.x / kWave), lane = threadIdx.x & (kWave - 1);
    if (p >= P) return;
    const int b = pstart[p], k = pstart[p + 1] - b;
    if (lane == 0) pcur[p] = 0;
    if (k <= kWave) {
        const int v = lane < k ? pedges[b + lane] : INT_MAX;
        int rank = 0;
        for (int j = 0; j < k; j++) rank += __shfl(v, j) < v;
        if (lane < k) {
            pedges[b + rank] = v;
            ckey[b + rank] = (unsigned)ecam[v];
        }
        return;
    }
    // a long run (a point observed by more than 64 edges; init_pfill leaves it nearly sorted):
    // insertion sort by one lane
    if (lane != 0) return;
    for (int a = b + 1; a < b + k; a++) {
        const int v = pedges[a];
        int j = a;
        while (j > b && pedges[j - 1] > v) {
            pedges[j] = pedges[j - 1];
            j--;
        }
        pedges[j] = v;
    }
    for (int a = b; a < b + k; a++) ckey[a] = (unsigned)ecam[pedges[a]];
}

// Camera CSR from the stable sort by camera of the point-CSR order: (camera, point, edge) order.
// Flags a camera observing a point twice (two consecutive entries of one camera on one point) and
// counts each free block's edges on points in the system (its diagonal pair's rhs list).
__global__ __launch_bounds__(256) void init_camcsr(int E, int C, int nbm, const unsigned* __restrict__ ckey_sorted,
                                                   const int* __restrict__ cval, const int* __restrict__ ept,
                                                   const int* __restrict__ camh, const int* __restrict__ ptfree,
                                                   int* __restrict__ cedges, int* __restrict__ cpt,
                                                   int* __restrict__ epos, int* __restrict__ sum, int* __restrict__ rc)
{
    const int a = blockIdx.x * 256 + threadIdx.x;
    const unsigned k = a < E ? ckey_sorted[a] : (unsigned)C;
    int h = -1;
    if (k < (unsigned)C) {
        const int e = cval[a], p = ept[e];
        cedges[a] = e;
        cpt[a] = p;
        epos[e] = a;
        if (a > 0 && ckey_sorted[a - 1] == k && ept[cval[a - 1]] == p) atomicOr(&sum[3], 1);
        if (ptfree[p]) h = camh[k];
        if (h >= nbm) h = -1;  // more free blocks than the summary holds: refused by the host
    }
    // the entries are sorted by camera: one atomic per distinct block of the wave
    unsigned long long todo = __ballot(h >= 0);
    while (todo) {
        const int leader = __ffsll((long long)todo) - 1;
        const int lh = __shfl(h, leader);
        const unsigned long long same = __ballot(h == lh);
        if ((int)(threadIdx.x & (kWave - 1)) == leader) atomicAdd(&rc[lh], __popcll(same));
        todo &= ~same;
    }
}

// ---- Stable counting sort by a small key (the camera-CSR order of the point-CSR entries, and the
// Schur product lists by pair key): per 1024-entry block a key histogram (csort_count), one
// workgroup turning the histograms into every block's first output slot per key (csort_scan), then
// each block scatters its entries in order (csort_scatter): ranks inside a wave from a match of the
// key bits, across the block's waves by LDS counters taken wave after wave.  Keys < nkeys.
constexpr int CS_BLOCK = 1024;
constexpr int CS_WAVES = CS_BLOCK / kWave;
constexpr int CS_MAX_KEYS = 12288;  // per-key counters in LDS (Schur pair keys: nb^2 <= 96^2)

// A pass sorts by the digit (key >> shift) & dmask (dmask = ~0: the whole key, < nkeys); keys
// beyond CS_MAX_KEYS take several stable passes over CS_DIGIT_BITS-bit digits, least significant
// first (stable_key_sort).
constexpr int CS_DIGIT_BITS = 12;
static_assert((1 << CS_DIGIT_BITS) <= CS_MAX_KEYS, "a digit's counters fit the LDS");
template <typename KeyT>
__device__ __forceinline__ int cs_digit(KeyT k, int shift, unsigned dmask)
{
    return (int)(((unsigned long long)k >> shift) & dmask);
}

// The point CSR's entries with what the point passes read next, (edge, camera, camera block,
// camera-CSR position), in one 16-byte record per entry: a point pass's loads are then pstart ->
// record -> the edge's data, instead of pstart -> pedges -> ecam -> camh / epos.  Fixed until the
// next initialisation (removed edges keep their records; `active` says which are live).
__global__ __launch_bounds__(256) void init_pcache(int E, int P, const int* __restrict__ pstart,
                                                   const int* __restrict__ pedges, const int* __restrict__ ecam,
                                                   const int* __restrict__ camh, const int* __restrict__ epos,
                                                   int4* __restrict__ pe)
{
    const int a = blockIdx.x * 256 + threadIdx.x;
    if (a >= E || a >= pstart[P]) return;
    const int e = pedges[a], c = ecam[e];
    pe[a] = make_int4(e, c, camh[c], epos[e]);
}

template <typename KeyT>
__global__ __launch_bounds__(CS_BLOCK) void csort_count(int n, int nkeys, const KeyT* __restrict__ key,
                                                        int* __restrict__ hist, int shift, unsigned dmask)
{
    __shared__ int h[CS_MAX_KEYS];
    for (int c = threadIdx.x; c < nkeys; c += CS_BLOCK) h[c] = 0;
    __syncthreads();
    const int i = blockIdx.x * CS_BLOCK + threadIdx.x;
    if (i < n) atomicAdd(&h[cs_digit(key[i], shift, dmask)], 1);
    __syncthreads();
    int* row = hist + (size_t)blockIdx.x * nkeys;
    for (int c = threadIdx.x; c < nkeys; c += CS_BLOCK) row[c] = h[c];
}

// One workgroup: hist[b][k] (block b's count of key k) becomes block b's first output slot for k
// (keys in ascending order, blocks in order inside a key).
// Key-major exclusive offsets of the per-block key histograms (one workgroup).  G threads per key
// (a power of two, G * keys <= 1024, within one wave) each take a contiguous chunk of the blocks:
// chunk sums, a scan of them over the group's lanes, then each thread writes its chunk's offsets.
// (One thread per key walking all blocks took 35 us per call for the camera-CSR sort: 98 blocks of
// dependent-issue loads per thread.)
template <typename F>
__device__ __forceinline__ void cs_chunk_loads(const int* __restrict__ hist, int nkeys, int c, int b0, int b1, F&& f)
{
    int b = b0;
    for (; b + 4 <= b1; b += 4) {
        int v[4];
#pragma unroll
        for (int j = 0; j < 4; j++) v[j] = hist[(size_t)(b + j) * nkeys + c];
#pragma unroll
        for (int j = 0; j < 4; j++) f(b + j, v[j]);
    }
    for (; b < b1; b++) f(b, hist[(size_t)b * nkeys + c]);
}

__global__ __launch_bounds__(1024) void csort_scan(int nblocks, int nkeys, int* __restrict__ hist)
{
    __shared__ int tot[CS_MAX_KEYS];
    int G = 1;
    while (G < kWave && 2 * G * nkeys <= 1024) G *= 2;
    const int per = 1024 / G, sub = threadIdx.x % G;
    const int cs = (nblocks + G - 1) / G, b0 = min(sub * cs, nblocks), b1 = min(b0 + cs, nblocks);
    // group inclusive scan of the chunk sums (lanes of one wave: G divides 64)
    auto group_scan = [&](int v) {
        for (int o = 1; o < G; o <<= 1) {
            const int t = __shfl_up(v, o, G);
            if (sub >= o) v += t;
        }
        return v;
    };
    for (int c0 = 0; c0 < nkeys; c0 += per) {
        const int c = c0 + (int)threadIdx.x / G;
        int s = 0;
        if (c < nkeys) cs_chunk_loads(hist, nkeys, c, b0, b1, [&](int, int v) { s += v; });
        const int inc = group_scan(s);
        if (c < nkeys && sub == G - 1) tot[c] = inc;
    }
    __syncthreads();
    block_scan_1024<int>(nkeys, [&](int c) { return tot[c]; }, [&](int c, int x) { tot[c] = x; });
    __syncthreads();
    for (int c0 = 0; c0 < nkeys; c0 += per) {
        const int c = c0 + (int)threadIdx.x / G;
        int s = 0;
        if (c < nkeys) cs_chunk_loads(hist, nkeys, c, b0, b1, [&](int, int v) { s += v; });
        const int inc = group_scan(s);
        if (c < nkeys) {
            int run = tot[c] + inc - s;
            cs_chunk_loads(hist, nkeys, c, b0, b1, [&](int b, int v) {
                hist[(size_t)b * nkeys + c] = run;
                run += v;
            });
        }
    }
}

template <typename KeyT, typename ValT>
__global__ __launch_bounds__(CS_BLOCK) void csort_scatter(int n, int nkeys, int kbits, const KeyT* __restrict__ key,
                                                          const ValT* __restrict__ val, const int* __restrict__ hist,
                                                          KeyT* __restrict__ key_out, ValT* __restrict__ val_out,
                                                          int shift, unsigned dmask)
{
    __shared__ int cnt[CS_MAX_KEYS];
    const int* row = hist + (size_t)blockIdx.x * nkeys;
    for (int c = threadIdx.x; c < nkeys; c += CS_BLOCK) cnt[c] = row[c];
    const int i = blockIdx.x * CS_BLOCK + threadIdx.x;
    const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
    const bool valid = i < n;
    const KeyT kfull = valid ? key[i] : (KeyT)0;
    const int k = valid ? cs_digit(kfull, shift, dmask) : -1;
    // lanes of this wave holding the same key
    unsigned long long peers = __ballot(valid);
    for (int b = 0; b < kbits; b++) {
        const bool bit = ((k >> b) & 1) != 0;
        const unsigned long long m = __ballot(bit);
        peers &= bit ? m : ~m;
    }
    const int rank = __popcll(peers & ((1ull << lane) - 1ull));
    const int leader = valid ? __ffsll((long long)peers) - 1 : lane;
    int base = 0;
    __syncthreads();
    for (int w = 0; w < CS_WAVES; w++) {  // waves in order: the block's entries keep their order per key
        if (wave == w && valid && rank == 0) base = atomicAdd(&cnt[k], __popcll(peers));
        __syncthreads();
    }
    base = __shfl(base, leader);
    if (valid) {
        key_out[base + rank] = kfull;
        val_out[base + rank] = val[i];
    }
}

// Exclusive prefix sum of n ints by one workgroup (out may not alias in).
__global__ __launch_bounds__(1024) void scan_exclusive(int n, const int* __restrict__ in, int* __restrict__ out)
{
    block_scan_1024<int>(n, [&](int i) { return in[i]; }, [&](int i, int x) { out[i] = x; });
}

// ---- Schur product lists built on the device (SparseOptimizer::initializeOptimization + g2o's
// BlockSolver::buildStructure: which pose blocks couple through a shared point) --------------
// Per free point: its edges in free camera blocks as (block, camera-CSR position), stably sorted
// by block (insertion sort in place; a point has few edges), and the number of (x, y) products
// with block(x) <= block(y) (both orders inside one block, as the host lists had them).
__global__ __launch_bounds__(256) void schur_point_lists(int P, const int* __restrict__ pstart,
                                                         const int* __restrict__ pedges, const int* __restrict__ ecam,
                                                         const int* __restrict__ camh, const int* __restrict__ epos,
                                                         const int* __restrict__ ptfree, int2* __restrict__ plist,
                                                         int* __restrict__ pcnt, int* __restrict__ klen)
{
    const int p = blockIdx.x * 256 + threadIdx.x;
    if (p >= P) return;
    if (!ptfree[p]) {
        pcnt[p] = 0;
        klen[p] = 0;
        return;
    }
    const int b = pstart[p], end = pstart[p + 1];
    int k = 0;
    for (int a = b; a < end; a++) {
        const int e = pedges[a];
        const int h = camh[ecam[e]];
        if (h < 0) continue;
        int j = k;
        while (j > 0 && plist[b + j - 1].x > h) {
            plist[b + j] = plist[b + j - 1];
            j--;
        }
        plist[b + j] = make_int2(h, epos[e]);
        k++;
    }
    int c = 0, g = 0;
    for (int x = 0; x < k; x++) {
        if (x > 0 && plist[b + x].x != plist[b + x - 1].x) g = x;
        c += k - g;
    }
    pcnt[p] = c;
    klen[p] = k;
}

// The products of one point at its exclusive-scan offset: key = pair (h1 * nb + h2), value =
// the two camera-CSR positions; in (x, y) order, so a stable sort by key leaves every pair's
// list in point order.
__global__ __launch_bounds__(256) void schur_point_products(int P, int nb, const int* __restrict__ pstart,
                                                            const int2* __restrict__ plist, const int* __restrict__ poff,
                                                            const int* __restrict__ klen, uint16_t* __restrict__ keys,
                                                            unsigned long long* __restrict__ vals)
{
    const int p = blockIdx.x * 256 + threadIdx.x;
    if (p >= P) return;
    const int k = klen[p];
    if (k == 0) return;
    const int b = pstart[p];
    int o = poff[p], g = 0;
    for (int x = 0; x < k; x++) {
        const int2 hx = plist[b + x];
        if (x > 0 && hx.x != plist[b + x - 1].x) g = x;
        for (int y = g; y < k; y++) {
            const int2 hy = plist[b + y];
            keys[o] = (uint16_t)(hx.x * nb + hy.x);
            vals[o] = (unsigned long long)(uint32_t)hx.y | ((unsigned long long)(uint32_t)hy.y << 32);
            o++;
        }
    }
}

// First and one-past-last sorted position of every pair key (0xFFFF: unused slot).
__global__ __launch_bounds__(256) void schur_list_bounds(const uint16_t* __restrict__ keys, int n, int nk,
                                                         int* __restrict__ kb)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int k = keys[i];
    if (k == 0xFFFF) return;
    if (i == 0 || keys[i - 1] != k) kb[k] = i;
    if (i + 1 == n || keys[i + 1] != k) kb[nk + k] = i + 1;
}

__global__ __launch_bounds__(256) void schur_scatter(const uint16_t* __restrict__ keys,
                                                     const unsigned long long* __restrict__ vals, int n,
                                                     const int* __restrict__ kdst, int2* __restrict__ sentries)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int k = keys[i];
    if (k == 0xFFFF) return;
    const unsigned long long v = vals[i];
    sentries[kdst[k] + i] = make_int2((int)(uint32_t)v, (int)(uint32_t)(v >> 32));
}

// A free camera block's rhs entries (camera-CSR position, point) over its free-point edges in
// camera-CSR order: one workgroup per block, a block-wide prefix of the free flags per 256 entries.
__global__ __launch_bounds__(256) void schur_rhs(const int* __restrict__ camblk, const int* __restrict__ cstart,
                                                 const int* __restrict__ cpt, const int* __restrict__ ptfree,
                                                 const int* __restrict__ rblk, int2* __restrict__ sentries, int pad_at)
{
    // the padding entry after the last list (schur_chunks reads one past a chunk's end)
    if (blockIdx.x == 0 && threadIdx.x == 0) sentries[pad_at] = make_int2(0, 0);
    __shared__ int wsum[256 / kWave];
    const int h = blockIdx.x, c = camblk[h];
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    const int end = cstart[c + 1];
    int base = rblk[h];
    for (int a0 = cstart[c]; a0 < end; a0 += 256) {
        const int a = a0 + (int)threadIdx.x;
        const int pt = a < end ? cpt[a] : 0;
        const bool f = a < end && ptfree[pt];
        const unsigned long long m = __ballot(f);
        const int below = __popcll(m & ((1ull << lane) - 1ull));
        if (lane == 0) wsum[w] = __popcll(m);
        __syncthreads();
        int off = 0, tot = 0;
        for (int i = 0; i < 256 / kWave; i++) {
            off += i < w ? wsum[i] : 0;
            tot += wsum[i];
        }
        if (f) sentries[base + off + below] = make_int2(a, pt);
        base += tot;
        __syncthreads();
    }
}

// ---- the common case: every camera observes a point at most once ---------------------------
// Then a pair's products are its cameras' shared free points, one each: with A_h the bit set of the
// points camera block h observes (its camera-CSR run is sorted by point) and F the points in the
// system, pair (a, b)'s list in point order is the set bits of A_a & A_b & F, and the edge of point
// p in camera block h sits at camera-CSR position cstart[c_h] + (rank of p in A_h).
constexpr int SC_LDS_WORDS = 16384;  // point bit words staged in LDS (P <= 524288)

// Grid: one workgroup per possible block (the block count nb = hdr[0] is known on the device
// only) + the last one for F.
__global__ __launch_bounds__(1024) void sc_bitmaps(int P, const int* __restrict__ hdr, const int* __restrict__ camblk,
                                                   const int* __restrict__ cstart, const int* __restrict__ cpt,
                                                   const int* __restrict__ ptfree, uint32_t* __restrict__ A,
                                                   int* __restrict__ R, uint32_t* __restrict__ F)
{
    __shared__ uint32_t bm[SC_LDS_WORDS];
    __shared__ int part[1024];
    const int PW = (P + 31) / 32, tid = threadIdx.x, h = blockIdx.x;
    if (h == (int)gridDim.x - 1) {
        for (int w = tid; w < PW; w += 1024) {
            uint32_t v = 0;
            for (int j = 0; j < 32 && 32 * w + j < P; j++) v |= (ptfree[32 * w + j] ? 1u : 0u) << j;
            F[w] = v;
        }
        return;
    }
    if (h >= hdr[0]) return;
    for (int w = tid; w < PW; w += 1024) bm[w] = 0;
    __syncthreads();
    const int c = camblk[h];
    for (int a = cstart[c] + tid; a < cstart[c + 1]; a += 1024) {
        const int p = cpt[a];
        atomicOr(&bm[p >> 5], 1u << (p & 31));
    }
    __syncthreads();
    // exclusive prefix popcount per word: each thread a contiguous segment of words
    const int seg = (PW + 1023) / 1024, w0 = tid * seg, w1 = min(PW, w0 + seg);
    int sum = 0;
    for (int w = w0; w < w1; w++) sum += __popc(bm[w]);
    part[tid] = sum;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {  // inclusive scan of the thread sums
        const int v = tid >= off ? part[tid - off] : 0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    int run = part[tid] - sum;
    uint32_t* Ah = A + (size_t)h * PW;
    int* Rh = R + (size_t)h * PW;
    for (int w = w0; w < w1; w++) {
        Ah[w] = bm[w];
        Rh[w] = run;
        run += __popc(bm[w]);
    }
}

__global__ __launch_bounds__(64) void sc_pair_counts(const int* __restrict__ hdr, int PW, const uint32_t* __restrict__ A,
                                                     const uint32_t* __restrict__ F, int* __restrict__ cnt)
{
    const int a = blockIdx.x, b = blockIdx.y, nb = hdr[0];
    if (b < a || b >= nb || nb > (int)gridDim.x) return;  // more blocks than the grid: refused by the host
    const uint32_t* Aa = A + (size_t)a * PW;
    const uint32_t* Ab = A + (size_t)b * PW;
    int n = 0;
    for (int w = threadIdx.x; w < PW; w += 64) n += __popc(Aa[w] & Ab[w] & F[w]);
    for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o);
    if (threadIdx.x == 0) cnt[a * nb + b] = n;
}

// Pair (a, b)'s products (camera-CSR positions of its two edges) in point order at kbase[a nb + b].
__global__ __launch_bounds__(64) void sc_pair_fill(int nb, int PW, const uint32_t* __restrict__ A,
                                                   const int* __restrict__ R, const uint32_t* __restrict__ F,
                                                   const int* __restrict__ camblk, const int* __restrict__ cstart,
                                                   const int* __restrict__ kbase, int2* __restrict__ sentries)
{
    const int a = blockIdx.x, b = blockIdx.y, lane = threadIdx.x;
    if (b < a) return;
    int base = kbase[a * nb + b];
    if (base < 0) return;
    const uint32_t* Aa = A + (size_t)a * PW;
    const uint32_t* Ab = A + (size_t)b * PW;
    const int* Ra = R + (size_t)a * PW;
    const int* Rb = R + (size_t)b * PW;
    const int ea = cstart[camblk[a]], eb = cstart[camblk[b]];
    for (int w0 = 0; w0 < PW; w0 += 64) {
        const int w = w0 + lane;
        const uint32_t wa = w < PW ? Aa[w] : 0u, wb = w < PW ? Ab[w] : 0u;
        uint32_t m = w < PW ? wa & wb & F[w] : 0u;
        const int c = __popc(m);
        int inc = c;  // inclusive wave scan of the counts
        for (int o = 1; o < 64; o <<= 1) {
            const int v = __shfl_up(inc, o);
            if (lane >= o) inc += v;
        }
        int pos = base + inc - c;
        const int ra = w < PW ? Ra[w] : 0, rb = w < PW ? Rb[w] : 0;
        while (m) {
            const int j = __builtin_ctz(m);
            m &= m - 1u;
            const uint32_t below = (1u << j) - 1u;
            sentries[pos++] = make_int2(ea + ra + __popc(wa & below), eb + rb + __popc(wb & below));
        }
        base += __shfl(inc, 63);
    }
}

// GetPose / GetPoint's outputs of the current state written into mapped host memory after a step,
// so UpdateData after every StepBundleAdjustment (BundleAdjust.cpp:195-226) reads them without a
// D2H copy + stream sync: per camera t as float and R of the normalised quaternion as float (the
// host's arithmetic of BundlerLib.cpp:457-465, in the same order, no contraction), per point the
// position as float; the completion word is written last.
__global__ __launch_bounds__(1024) void export_state(State s, int C, int P, float* __restrict__ out,
                                                     unsigned* __restrict__ seq_out, unsigned seq)
{
    float* pos3 = out;
    float* r9 = out + 3 * C;
    float* xyz = out + 12 * C;
    for (int c = threadIdx.x; c < C; c += 1024) {
        double q[4] = {s.q[4 * c], s.q[4 * c + 1], s.q[4 * c + 2], s.q[4 * c + 3]};
        const double nn = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
        for (int k = 0; k < 4; k++) q[k] /= nn;
        const double tx = 2 * q[0], ty = 2 * q[1], tz = 2 * q[2];
        const double twx = tx * q[3], twy = ty * q[3], twz = tz * q[3];
        const double txx = tx * q[0], txy = ty * q[0], txz = tz * q[0];
        const double tyy = ty * q[1], tyz = tz * q[1], tzz = tz * q[2];
        const double R[9] = {1 - (tyy + tzz), txy - twz, txz + twy, txy + twz, 1 - (txx + tzz),
                             tyz - twx,       txz - twy, tyz + twx, 1 - (txx + tyy)};
        for (int k = 0; k < 3; k++) pos3[3 * c + k] = (float)s.t[3 * c + k];
        for (int rr = 0; rr < 3; rr++)
            for (int cc = 0; cc < 3; cc++) r9[9 * c + cc * 3 + rr] = (float)R[rr * 3 + cc];
    }
    // points: 16-byte stores of 4 floats (the mirror is written over the fabric)
    const int np = 3 * P;
    for (int i = 4 * threadIdx.x; i < np; i += 4096) {
        if (i + 3 < np && ((12 * C + i) & 3) == 0)
            *reinterpret_cast<float4*>(xyz + i) =
                make_float4((float)s.p[i], (float)s.p[i + 1], (float)s.p[i + 2], (float)s.p[i + 3]);
        else
            for (int k = 0; k < 4 && i + k < np; k++) xyz[i + k] = (float)s.p[i + k];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence_system();
        *reinterpret_cast<volatile unsigned*>(seq_out) = seq;
    }
}

}  // namespace

// ------------------------------------------------------------------------------------------
// Host: the StepOptimizer / OptimizationAlgorithmLevenberg control flow
// ------------------------------------------------------------------------------------------

// chol_tiles' slot table, ti | tj << 8 per (tile wave, slot), 0xFFFF empty, followed by one
// structural row mask per tile row (bit j of row k: tile (k, j) of U can be nonzero).  Only the
// tiles of the factor's envelope get a slot: the 6x6 blocks the Schur pairs write (every nonzero
// block of S, tether blocks included), the diagonal and the chain tiles (d-1, d), closed under
// the tile-level symbolic fill (U_ki, U_kj nonzero -> A_ij filled).  Tiles outside it are zero in
// S and stay zero in U, so their TRSMs, SYRK updates and backward products are skipped.  The
// slots go round-robin over the tile waves in row-major order; tile (0, 0) is the factor wave's
// (read from S directly).
static void chol_tile_table(int mt, const SchurPair* pairs, int npairs, std::vector<uint16_t>& tab)
{
    std::vector<uint16_t> nz(CT_MAXT, 0);
    auto mark = [&](int a, int b) {
        if (a > b) std::swap(a, b);
        if (a < mt && b < mt) nz[a] |= (uint16_t)(1u << b);
    };
    for (int d = 0; d < mt; d++) {
        mark(d, d);
        if (d > 0) mark(d - 1, d);
    }
    for (int pi = 0; pi < npairs; pi++) {
        const int r1 = 6 * pairs[pi].h1, r2 = 6 * pairs[pi].h2;
        for (int a : {r1 / 16, (r1 + 5) / 16})
            for (int b : {r2 / 16, (r2 + 5) / 16}) mark(a, b);
    }
    for (int k = 0; k < mt; k++)  // symbolic fill, in factor order
        for (int i = k + 1; i < mt; i++)
            if (nz[k] >> i & 1) nz[i] |= (uint16_t)(nz[k] & ~((1u << i) - 1u));
    tab.assign((size_t)CT_TW * CT_TPW + CT_MAXT, 0xFFFF);
    std::vector<int> cnt(CT_TW, 0);
    std::vector<std::pair<int, int>> tiles;
    for (int i = 0; i < mt; i++)
        for (int j = i; j < mt; j++)
            if (!(i == 0 && j == 0) && (nz[i] >> j & 1)) tiles.emplace_back(i, j);
    // The factor wave (wave CT_TW) shares its SIMD with the tile waves w = CT_TW (mod 4) (a
    // workgroup's waves are dealt to the SIMDs cyclically; speed only): those get the first,
    // earliest-finished tiles and few of them, so the factor's column loop meets fewer SYRK MFMAs.
    std::vector<int> light, heavy;
    for (int w = 0; w < CT_TW; w++) ((w & 3) == (CT_TW & 3) ? light : heavy).push_back(w);
    const int nheavy = (int)heavy.size() * CT_TPW;
    const int per_light = light.empty() ? 0
                                        : std::min(CT_TPW, std::max(0, ((int)tiles.size() - nheavy +
                                                                                      (int)light.size() - 1) /
                                                                                         (int)light.size()));
    size_t t = 0;
    for (int w : light)
        for (int c = 0; c < per_light && t < tiles.size(); c++, t++)
            tab[(size_t)w * CT_TPW + cnt[w]++] = (uint16_t)(tiles[t].first | tiles[t].second << 8);
    for (size_t h = 0; t < tiles.size(); t++) {
        while (cnt[heavy[h % heavy.size()]] >= CT_TPW) h++;
        const int w = heavy[h++ % heavy.size()];
        tab[(size_t)w * CT_TPW + cnt[w]++] = (uint16_t)(tiles[t].first | tiles[t].second << 8);
    }
    for (int k = 0; k < CT_MAXT; k++) tab[(size_t)CT_TW * CT_TPW + k] = k < mt ? nz[k] : 0;
}
static_assert(CT_TW * CT_TPW >= CT_MAXT * (CT_MAXT + 1) / 2 - 1, "every tile but (0, 0) has a slot");

struct BundleAdjuster {
    int device = 0;
    bool points_fixed = false;
    // host copies of the problem
    int C = 0, P = 0, E = 0;
    std::vector<double> q, t, camk, p;
    std::vector<int> fixed, ecam;  // ecam: per-camera edge bookkeeping of outlier removals
    std::vector<Tether> teth;      // distance, rotation, transform tethers (set order)
    std::vector<int> cam_tethers;  // active tethers per camera (keeps a camera in the system)
    bool dirty = true;  // full (re)initialisation needed: setters or a camera left the system
    bool useless = false, state_on_device = false, host_state_stale = false, err_initialized = false;
    int iteration = 0;
    double user_lambda = 0, lambda = 0, ni = 2, huber = 0;
    // a linearisation launched at the end of the previous step for the next one (see step())
    bool eager = false, eager_init = false;
    double eager_huber = 0, eager_lambda = 0;
    int eager_cur = -1;
    int n = 0, np = 0;  // 6 * cameras in the system, padded to a multiple of 16
    int npairs = 0, n_slots = 0, n_sblocks = 0, n_sfinish = 0;  // Schur pairs, partial slots, blocks, schur_finish pairs
    std::vector<int> camh, ptfree, cam_of_block;
    hipStream_t st = nullptr;
    // Control block read back at every host decision (one pinned copy per synchronisation):
    // doubles [0,3) linearisation chi2 / max diag, [3,6) trial, then the outlier pass's
    // OutlierCtl (sums, Cholesky failure flag, counts, ticket).
    static constexpr int CTL_DOUBLES = 16, CTL_OUTLIER = 6, CTL_SCRATCH = 12, CTL_LMNEXT = 13, CTL_SEQ = 15;
    static_assert(CTL_OUTLIER * 8 + sizeof(OutlierCtl) <= CTL_SCRATCH * 8, "control block layout");
    // The control block is host memory the kernels write directly (pinned, coherent, mapped):
    // h_ctl on the host, h_ctl_dev in kernels; a trial's results need only the stream sync.
    double* h_ctl = nullptr;
    double* h_ctl_dev = nullptr;
    size_t ctl_bytes = 0;  // the block's real size (a cached block may be larger than CTL_DOUBLES)
    OutlierCtl* d_octl() const { return reinterpret_cast<OutlierCtl*>(h_ctl_dev + CTL_OUTLIER); }
    const OutlierCtl& h_octl() const { return *reinterpret_cast<const OutlierCtl*>(h_ctl + CTL_OUTLIER); }
    LiveCtl* d_live() const { return reinterpret_cast<LiveCtl*>(d_livebuf.ptr); }
    int* d_failp() const { return &d_live()->fail; }
    mage_status read_ctl()
    {
        MAGE_HIP(hipStreamSynchronize(st));
        return MAGE_OK;
    }
    // reduce3's completion: spin on its sequence word in the host-mapped block (a blocking
    // stream sync costs ~10-20 us of wake-up per LM trial); after 2 ms fall back to the sync,
    // which also reports a failed launch
    unsigned seq_counter = 0;
    unsigned* seq_dev() const { return reinterpret_cast<unsigned*>(h_ctl_dev + CTL_SEQ); }
    mage_status wait_seq(unsigned seq)
    {
        volatile unsigned* f = reinterpret_cast<volatile unsigned*>(h_ctl + CTL_SEQ);
        const auto t0 = std::chrono::steady_clock::now();
        while (*f != seq) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) {
                MAGE_HIP(hipStreamSynchronize(st));
                MAGE_REQUIRE(*f == seq, MAGE_EDEVICE, "BA control block not updated after the stream completed");
                break;
            }
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        return MAGE_OK;
    }
    int ctl_fail() const { return h_octl().fail; }
    int cur = 0;  // which state buffer holds the current estimate
    // device buffers
    DeviceBuffer d_q[2], d_t[2], d_p[2], d_camk, d_camh, d_ptfree, d_uv, d_ecam, d_ept, d_info,
        d_pstart, d_pedges, d_pe, d_cstart, d_cedges, d_cpt, d_active, d_err, d_Hll, d_bl, d_Hpl, d_Hpp,
        d_bp, d_S, d_rhs, d_x, d_chi, d_maxd, d_scale, d_red, d_lm, d_osum, d_camblk,
        d_ptcnt, d_plist, d_pcnt, d_skeys, d_svals, d_kb, d_chist, d_kdst, d_rblk, d_sbits, d_srank, d_Z, d_campart, d_teth, d_tout, d_ptlist, d_sentries, d_spairs, d_schunks, d_spart,
        d_sfinish, d_epos, d_chi_lin, d_livebuf, d_removed, d_camflag, d_ikeys, d_ivals, d_isum, d_iacc, d_ctab, d_csort_tmp;
    bool iacc_clean = false;  // d_iacc is all zero (see initialize())
    // outlier lists of the speculative / final post-pass (2 x E entries), written by the kernels
    // straight into host memory: the host sorts and returns them after the completion wait
    MappedBuffer h_olist;
    PinnedBuffer h_kb;    // per-pair list bounds read back by build_product_lists
    MappedBuffer h_isum;  // the device initialisation's summary (init_scan etc., INIT_HDR layout)
    std::vector<int> camcnt;  // active observation edges per camera (host-side bookkeeping)
    int n_entries = 0;  // point-CSR entries (active edges at initialisation)
    int nb_free = 0;    // cameras in the reduced system
    mage_ba_stats stats{};

    static int group_grid(int items) { return (int)(((long long)items * PG + BA_THREADS - 1) / BA_THREADS); }

    Problem problem() const
    {
        Problem pb;
        pb.C = C;
        pb.P = P;
        pb.camk = d_camk.as<double>();
        pb.camh = d_camh.as<int>();
        pb.ptfree = d_ptfree.as<int>();
        pb.uv = d_uv.as<float>();
        pb.ecam = d_ecam.as<int>();
        pb.ept = d_ept.as<int>();
        pb.info = d_info.as<float>();
        pb.active = d_active.as<unsigned char>();
        pb.pstart = d_pstart.as<int>();
        pb.pedges = d_pedges.as<int>();
        pb.cstart = d_cstart.as<int>();
        pb.cedges = d_cedges.as<int>();
        pb.cpt = d_cpt.as<int>();
        pb.epos = d_epos.as<int>();
        pb.pe = d_pe.as<int4>();
        pb.ecsr = n_entries;
        pb.huber = huber;
        return pb;
    }
    State state(int i) const { return State{d_q[i].as<double>(), d_t[i].as<double>(), d_p[i].as<double>()}; }

    void release()
    {
        // an eager linearisation may still be running; only blocks of a synchronised stream are
        // idle and go to the block cache, after a failed synchronisation everything is freed
        const bool idle = !st || hipStreamSynchronize(st) == hipSuccess;
        for (auto* b : {&d_q[0], &d_q[1], &d_t[0], &d_t[1], &d_p[0], &d_p[1], &d_camk, &d_camh, &d_ptfree,
                        &d_uv, &d_ecam, &d_ept, &d_info, &d_pstart, &d_pedges, &d_pe, &d_cstart, &d_cedges, &d_cpt,
                        &d_active, &d_err, &d_Hll, &d_bl, &d_Hpl, &d_Hpp, &d_bp, &d_S, &d_rhs,
                        &d_x, &d_chi, &d_maxd, &d_scale, &d_red, &d_lm, &d_osum, &d_camblk,
                        &d_ptcnt, &d_plist, &d_pcnt, &d_skeys, &d_svals, &d_kb, &d_chist, &d_kdst, &d_rblk, &d_sbits, &d_srank, &d_Z, &d_campart, &d_teth, &d_tout, &d_ptlist, &d_sentries, &d_spairs,
                        &d_schunks, &d_spart, &d_sfinish, &d_epos, &d_chi_lin, &d_livebuf, &d_removed, &d_camflag,
                        &d_ikeys, &d_ivals, &d_isum, &d_iacc, &d_ctab, &d_csort_tmp})
            if (idle)
                b->retire();  // the stream is synchronised: the blocks are idle (common.hpp block cache)
            else
                b->release();
        if (idle) {
            h_olist.retire();
            h_state.retire();
            h_kb.retire();
            h_isum.retire();
            h_stage.retire();
            h_dma.retire();
        } else {
            h_olist.release();
            h_state.release();
            h_kb.release();
            h_isum.release();
            h_stage.release();
            h_dma.release();
        }
        iacc_clean = false;
        stage_off = dma_off = 0;
        pending.k = 0;
        if (st) {
            if (idle)
                mage::stream_retire(st);
            else
                (void)hipStreamDestroy(st);
        }
        st = nullptr;
        if (h_ctl) {
            if (idle && ctl_bytes)
                mage::pool_retire(2, h_ctl, ctl_bytes);
            else
                (void)hipHostFree(h_ctl);
        }
        h_ctl = nullptr;
        ctl_bytes = 0;
    }

    // Host-to-device copies are staged in pinned memory.  Large ones are DMA copies from a pinned
    // ring (a hipMemcpyAsync from pageable memory would be a synchronous staged copy); small ones
    // go to a device-mapped arena and are moved by one gather_copy launch (flush_uploads) instead
    // of one copy call each.  A ring / the arena restarts from its beginning only after a stream
    // synchronisation, so no pending copy sees its source change; it grows only when a single copy
    // does not fit it.
    MappedBuffer h_stage;  // small copies (read by gather_copy over the fabric)
    PinnedBuffer h_dma;    // large copies (DMA source)
    size_t stage_off = 0, dma_off = 0;
    GatherList pending{};
    static constexpr size_t GATHER_MAX_BYTES = 64 << 10;
    void flush_uploads()
    {
        if (pending.k == 0) return;
        unsigned blocks = 0;
        for (int i = 0; i < pending.k; i++) {
            pending.first[i] = blocks;
            blocks += (unsigned)((pending.bytes[i] + GATHER_BLOCK_BYTES - 1) / GATHER_BLOCK_BYTES);
        }
        pending.first[pending.k] = blocks;
        launch("ba.upload_gather", gather_copy, dim3(blocks), dim3(256), 0, st, pending);
        pending.k = 0;
    }
    // a queued (not yet launched) copy writes into [p, p + n)
    bool pending_overlaps(const void* p, size_t n) const
    {
        const char* a = static_cast<const char*>(p);
        for (int i = 0; i < pending.k; i++)
            if (pending.dst[i] < a + n && a < pending.dst[i] + pending.bytes[i]) return true;
        return false;
    }
    mage_status stage_copy(void* dst, const void* src, size_t bytes)
    {
        if (bytes == 0) return MAGE_OK;
        const size_t need = (bytes + 255) & ~(size_t)255;
        mage_status r;
        // copies stay in call order: a DMA copy goes after every queued one, and a second copy
        // into a queued destination after the first (one gather launch does not order its blocks)
        if (bytes >= GATHER_MAX_BYTES || pending_overlaps(dst, bytes)) flush_uploads();
        if (bytes >= GATHER_MAX_BYTES) {
            if (dma_off + need > h_dma.bytes) {
                MAGE_HIP(hipStreamSynchronize(st));
                dma_off = 0;
                if (need > h_dma.bytes && (r = h_dma.reserve(std::max(need, (size_t)8 << 20))) != MAGE_OK) return r;
            }
            char* h = h_dma.as<char>() + dma_off;
            std::memcpy(h, src, bytes);
            MAGE_HIP(hipMemcpyAsync(dst, h, bytes, hipMemcpyHostToDevice, st));
            dma_off += need;
            return MAGE_OK;
        }
        if (stage_off + need > h_stage.bytes) {
            flush_uploads();
            MAGE_HIP(hipStreamSynchronize(st));
            stage_off = 0;
            if (need > h_stage.bytes && (r = h_stage.reserve(std::max(need, (size_t)1 << 20))) != MAGE_OK) return r;
        }
        std::memcpy(h_stage.host<char>() + stage_off, src, bytes);
        if (pending.k == GATHER_MAX) flush_uploads();
        pending.src[pending.k] = h_stage.device<const char>() + stage_off;
        pending.dst[pending.k] = static_cast<char*>(dst);
        pending.bytes[pending.k++] = (unsigned)bytes;
        stage_off += need;
        return MAGE_OK;
    }
    template <typename T>
    mage_status upload(DeviceBuffer& b, const std::vector<T>& v)
    {
        return upload(b, v.data(), v.size());
    }
    template <typename T>
    mage_status upload(DeviceBuffer& b, const T* v, size_t n)
    {
        // a growing buffer is freed by reserve(): launch the queued copies into it first
        if (b.ptr && std::max<size_t>(n * sizeof(T), 16) > b.bytes && pending_overlaps(b.ptr, b.bytes)) flush_uploads();
        mage_status r = b.reserve(std::max<size_t>(n * sizeof(T), 16));
        if (r != MAGE_OK) return r;
        return stage_copy(b.ptr, v, n * sizeof(T));
    }

    // export_state's GetPose / GetPoint outputs of the current estimate (valid while export_seq is
    // the last sequence number launched and export_cur the current buffer)
    MappedBuffer h_state;
    unsigned export_seq = 0;
    int export_cur = -1;
    bool export_wanted = false;  // the caller read the state since the last step
    void launch_export()
    {
        if (h_state.reserve((size_t)(12 * C + 3 * P + 4) * sizeof(float)) != MAGE_OK) {
            export_cur = -1;
            return;
        }
        launch("ba.export_state", export_state, dim3(1), dim3(1024), 0, st, state(cur), C, P, h_state.device<float>(),
               seq_dev(), ++seq_counter);
        export_seq = seq_counter;
        export_cur = cur;
    }
    // the exported outputs when they are those of the current estimate (after their completion wait)
    const float* exported()
    {
        if (!state_on_device || !host_state_stale || export_cur != cur || export_seq != seq_counter) return nullptr;
        if (wait_seq(export_seq) != MAGE_OK) return nullptr;
        return h_state.host<float>();
    }

    // Pull the current estimate back to the host vectors.
    mage_status sync_host_state()
    {
        if (!state_on_device || !host_state_stale) return MAGE_OK;
        MAGE_HIP(hipMemcpyAsync(q.data(), d_q[cur].ptr, sizeof(double) * 4 * C, hipMemcpyDeviceToHost, st));
        MAGE_HIP(hipMemcpyAsync(t.data(), d_t[cur].ptr, sizeof(double) * 3 * C, hipMemcpyDeviceToHost, st));
        MAGE_HIP(hipMemcpyAsync(p.data(), d_p[cur].ptr, sizeof(double) * 3 * P, hipMemcpyDeviceToHost, st));
        MAGE_HIP(hipStreamSynchronize(st));
        host_state_stale = false;
        return MAGE_OK;
    }

    // Stable sort of n (key, value) entries by key (< nkeys) with the csort_* kernels: one pass for
    // up to CS_MAX_KEYS keys, else stable passes over CS_DIGIT_BITS-bit digits, least significant
    // first, through a scratch copy (a bundle adjustment with more cameras than the LDS counters).
    template <typename KeyT, typename ValT>
    mage_status stable_key_sort(const KeyT* kin, const ValT* vin, KeyT* kout, ValT* vout, int n, int nkeys)
    {
        if (n <= 0) return MAGE_OK;
        const int nblk = (n + CS_BLOCK - 1) / CS_BLOCK;
        mage_status r;
        int kbits = 1;
        while ((1 << kbits) < nkeys) kbits++;
        auto pass = [&](const KeyT* ki, const ValT* vi, KeyT* ko, ValT* vo, int ndig, int dbits, int shift,
                        unsigned dmask) -> mage_status {
            mage_status rr;
            if ((rr = d_chist.reserve((size_t)nblk * ndig * sizeof(int))) != MAGE_OK) return rr;
            launch("ba.sort_count", csort_count<KeyT>, dim3(nblk), dim3(CS_BLOCK), 0, st, n, ndig, ki, d_chist.as<int>(),
                   shift, dmask);
            launch("ba.sort_scan", csort_scan, dim3(1), dim3(1024), 0, st, nblk, ndig, d_chist.as<int>());
            launch("ba.sort_scatter", csort_scatter<KeyT, ValT>, dim3(nblk), dim3(CS_BLOCK), 0, st, n, ndig, dbits, ki, vi,
                   (const int*)d_chist.as<int>(), ko, vo, shift, dmask);
            return MAGE_OK;
        };
        if (nkeys <= CS_MAX_KEYS) return pass(kin, vin, kout, vout, nkeys, kbits, 0, ~0u);
        const int npass = (kbits + CS_DIGIT_BITS - 1) / CS_DIGIT_BITS;
        // two (keys, values) copies, each array starting 128-byte aligned
        const size_t kb = ((size_t)n * sizeof(KeyT) + 127) / 128 * 128, vb = ((size_t)n * sizeof(ValT) + 127) / 128 * 128;
        if ((r = d_csort_tmp.reserve(2 * (kb + vb))) != MAGE_OK) return r;
        KeyT* tk[2] = {d_csort_tmp.as<KeyT>(), nullptr};
        ValT* tv[2] = {nullptr, nullptr};
        {
            char* base = d_csort_tmp.as<char>();
            tk[0] = reinterpret_cast<KeyT*>(base);
            tv[0] = reinterpret_cast<ValT*>(base + kb);
            tk[1] = reinterpret_cast<KeyT*>(base + kb + vb);
            tv[1] = reinterpret_cast<ValT*>(base + 2 * kb + vb);
        }
        const KeyT* ki = kin;
        const ValT* vi = vin;
        for (int ps = 0; ps < npass; ps++) {
            const bool last = ps + 1 == npass;
            KeyT* ko = last ? kout : tk[ps & 1];
            ValT* vo = last ? vout : tv[ps & 1];
            if ((r = pass(ki, vi, ko, vo, 1 << CS_DIGIT_BITS, CS_DIGIT_BITS, ps * CS_DIGIT_BITS,
                          (1u << CS_DIGIT_BITS) - 1u)) != MAGE_OK)
                return r;
            ki = ko;
            vi = vo;
        }
        return MAGE_OK;
    }

    // SparseOptimizer::initializeOptimization (+ StepOptimizer::InitializeOptimization):
    // active edges, vertices in the system, CSR structures, covisible camera pairs; iteration 0.
    static size_t nprod_pad(long long n) { return (size_t)((n + 255) / 256 * 256); }
    // Builds every pair's product list on the device (schur_point_lists -> exclusive scan ->
    // schur_point_products -> stable radix sort by pair key -> schur_list_bounds) and reads back
    // each dense pair key's first sorted position and count; *nprod = the number of products.
    // Only for a camera observing a point twice (else the bit-set path of initialize()).
    mage_status build_product_lists(int nb, int ncsr, std::vector<int>& kstart, std::vector<int>& kcount,
                                    long long* nprod)
    {
        mage_status r;
        const int Pm = std::max(P, 1), nk = nb * nb;
        if ((r = d_plist.reserve((size_t)std::max(ncsr, 1) * sizeof(int2))) != MAGE_OK) return r;
        if ((r = d_pcnt.reserve((size_t)3 * Pm * sizeof(int))) != MAGE_OK) return r;
        int* pcnt = d_pcnt.as<int>();
        int* poff = pcnt + Pm;
        int* klen = pcnt + 2 * Pm;
        const unsigned gp = (unsigned)((P + 255) / 256);
        launch("ba.schur_lists", schur_point_lists, dim3(gp), dim3(256), 0, st, P, (const int*)d_pstart.as<int>(),
               (const int*)d_pedges.as<int>(), (const int*)d_ecam.as<int>(), (const int*)d_camh.as<int>(),
               (const int*)d_epos.as<int>(), (const int*)d_ptfree.as<int>(), d_plist.as<int2>(), pcnt, klen);
        launch("ba.schur_scan", scan_exclusive, dim3(1), dim3(1024), 0, st, P, (const int*)pcnt, poff);
        if ((r = h_kb.reserve((size_t)std::max(2 * nk, 2) * sizeof(int))) != MAGE_OK) return r;
        MAGE_HIP(hipMemcpyAsync(h_kb.ptr, poff + P - 1, sizeof(int), hipMemcpyDeviceToHost, st));
        MAGE_HIP(hipMemcpyAsync(h_kb.as<int>() + 1, pcnt + P - 1, sizeof(int), hipMemcpyDeviceToHost, st));
        MAGE_HIP(hipStreamSynchronize(st));
        const long long nmax = (long long)h_kb.as<int>()[0] + h_kb.as<int>()[1];
        *nprod = nmax;
        MAGE_REQUIRE(nmax < (1ll << 31), MAGE_EUNSUPPORTED, "Schur product list exceeds 2^31 entries");
        if (nmax == 0) return MAGE_OK;
        const size_t pad = nprod_pad(nmax);
        if ((r = d_skeys.reserve(2 * pad * sizeof(uint16_t))) != MAGE_OK) return r;
        if ((r = d_svals.reserve(2 * pad * sizeof(unsigned long long))) != MAGE_OK) return r;
        if ((r = d_kb.reserve((size_t)2 * nk * sizeof(int))) != MAGE_OK) return r;
        uint16_t* kin = d_skeys.as<uint16_t>();
        uint16_t* kout = kin + pad;
        unsigned long long* vin = d_svals.as<unsigned long long>();
        unsigned long long* vout = vin + pad;
        MAGE_HIP(hipMemsetAsync(d_kb.ptr, 0, (size_t)2 * nk * sizeof(int), st));
        launch("ba.schur_products", schur_point_products, dim3(gp), dim3(256), 0, st, P, nb,
               (const int*)d_pstart.as<int>(), (const int2*)d_plist.as<int2>(), (const int*)poff, (const int*)klen, kin, vin);
        if ((r = stable_key_sort(kin, vin, kout, vout, (int)nmax, nk)) != MAGE_OK) return r;
        const unsigned gn = (unsigned)((nmax + 255) / 256);
        launch("ba.schur_bounds", schur_list_bounds, dim3(gn), dim3(256), 0, st, (const uint16_t*)kout, (int)nmax, nk,
               d_kb.as<int>());
        MAGE_HIP(hipGetLastError());
        MAGE_HIP(hipMemcpyAsync(h_kb.ptr, d_kb.ptr, (size_t)2 * nk * sizeof(int), hipMemcpyDeviceToHost, st));
        MAGE_HIP(hipStreamSynchronize(st));
        const int* kb = h_kb.as<int>();
        for (int k = 0; k < nk; k++) {
            kstart[k] = kb[k];
            kcount[k] = kb[nk + k] - kb[k];
        }
        return MAGE_OK;
    }

    // MAGE_BA_TIMING=1: host phase times of initialize() on stderr (development probe)
    struct PhaseTimer {
        bool on = getenv("MAGE_BA_TIMING") != nullptr;
        std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
        void mark(const char* what)
        {
            if (!on) return;
            const auto n = std::chrono::steady_clock::now();
            fprintf(stderr, "[ba.init] %-28s %8.1f us\n", what, std::chrono::duration<double, std::micro>(n - t).count());
            t = std::chrono::steady_clock::now();  // the print is not charged to the next phase
        }
    };
    struct ScopeTimer {  // MAGE_BA_TIMING=1: one entry point's wall time on stderr
        PhaseTimer pt;
        const char* what;
        explicit ScopeTimer(const char* w) : what(w) {}
        ~ScopeTimer() { pt.mark(what); }
    };
    // initialize()'s host tables, kept between calls: reused capacity instead of fresh allocations
    // (page faults on every BuildDataForG2O window)
    struct InitTables {
        std::vector<unsigned char> camflag, mark;
        std::vector<int2> pairs;
        std::vector<int> pairidx, kcount, kstart, ptstart, ptlist, pcount, rcount, rblk, kdst, sfinish;
        std::vector<long long> pbeg, roww;
        std::vector<SchurPair> spairs;
        std::vector<SchurChunk> xcd_chunks[8], schunks;
        std::vector<uint16_t> ctab;
    } ws;
    mage_status initialize()
    {
        PhaseTimer pt;
        mage_status r = sync_host_state();
        if (r != MAGE_OK) return r;
        pt.mark("sync_host_state");
        // tethers: active unless both cameras are fixed; their cameras join the system
        cam_tethers.assign(C, 0);
        for (auto& T : teth) {
            T.active = !(fixed[T.c1] && fixed[T.c2]);
            if (T.active) {
                cam_tethers[T.c1]++;
                cam_tethers[T.c2]++;
            }
        }
        // The active edge set, the point / camera CSRs and the free blocks are built on the device
        // (init_edges, init_scan, init_pfill / init_psort, a stable radix sort by camera,
        // init_camcsr); so are the Schur pairs' product counts when no camera observes a point twice
        // (sc_bitmaps / sc_pair_counts).  One summary comes back.
        const size_t Cm = std::max(C, 1), Pm = std::max(P, 1), Em = std::max(E, 1);
        const int nbm = std::min(C, CH_PANEL_ROWS / 6);  // a larger block count is refused below
        const int PW = (P + 31) / 32;
        const size_t nsum = (size_t)INIT_HDR + 2 * (size_t)C + (size_t)nbm + (size_t)nbm * nbm;
        {
            auto& camflag = ws.camflag;
            camflag.assign(Cm, 0);
            for (int c = 0; c < C; c++) camflag[c] = (fixed[c] ? 1 : 0) | (cam_tethers[c] ? 2 : 0);
            if ((r = upload(d_camflag, camflag)) != MAGE_OK) return r;
            flush_uploads();
        }
        for (auto pr : {std::make_pair(&d_camh, (size_t)Cm * 4), std::make_pair(&d_camblk, (size_t)Cm * 4),
                        std::make_pair(&d_ptfree, (size_t)Pm * 4), std::make_pair(&d_ptcnt, (size_t)Pm * 4),
                        std::make_pair(&d_pstart, (size_t)(Pm + 1) * 4), std::make_pair(&d_cstart, (size_t)(Cm + 1) * 4),
                        std::make_pair(&d_pedges, (size_t)Em * 4), std::make_pair(&d_cedges, (size_t)Em * 4),
                        std::make_pair(&d_cpt, (size_t)Em * 4), std::make_pair(&d_epos, (size_t)Em * 4),
                        std::make_pair(&d_pe, (size_t)Em * 16),
                        std::make_pair(&d_active, (size_t)Em), std::make_pair(&d_ikeys, (size_t)Em * 8),
                        std::make_pair(&d_ivals, (size_t)Em * 4), std::make_pair(&d_isum, nsum * 4)})
            if ((r = pr.first->reserve(pr.second)) != MAGE_OK) return r;
        if ((r = h_isum.reserve(nsum * 4)) != MAGE_OK) return r;
        int* sum = d_isum.as<int>();
        int* s_ccnt = sum + INIT_HDR;
        int* s_camblk = s_ccnt + C;
        int* s_rc = s_camblk + C;
        int* s_kcnt = s_rc + nbm;
        unsigned* k0 = d_ikeys.as<unsigned>();
        unsigned* k1 = k0 + Em;
        int* v0 = d_ivals.as<int>();
        // accumulators kept zero between initialisations (cleared by their consumers): per point,
        // per camera, per-point fill cursors; cleared here only when (re)allocated or after a
        // chain that did not complete
        const size_t acc_bytes = (2 * Pm + Cm) * 4;
        if (d_iacc.bytes < acc_bytes || !iacc_clean) {
            if ((r = d_iacc.reserve(acc_bytes)) != MAGE_OK) return r;
            MAGE_HIP(hipMemsetAsync(d_iacc.ptr, 0, d_iacc.bytes, st));
        }
        iacc_clean = false;
        int* pacc = d_iacc.as<int>();
        int* cacc = pacc + Pm;
        int* pcur = cacc + Cm;
        const unsigned ge = (unsigned)((E + 255) / 256);
        if (E > 0)
            launch("ba.init_edges", init_edges, dim3(ge), dim3(256), C <= INIT_LDS_CAMS ? C * 4 : 0, st, E, C,
                   points_fixed ? 1 : 0, (const int*)d_ecam.as<int>(), (const int*)d_ept.as<int>(),
                   (const unsigned char*)d_removed.as<unsigned char>(), (const unsigned char*)d_camflag.as<unsigned char>(),
                   d_active.as<unsigned char>(), pacc, cacc, d_epos.as<int>(), k0);
        launch("ba.init_scan", init_scan, dim3(1), dim3(1024), 0, st, C, P, nbm, points_fixed ? 1 : 0,
               (const unsigned char*)d_camflag.as<unsigned char>(), pacc, cacc, d_ptcnt.as<int>(), d_pstart.as<int>(),
               d_ptfree.as<int>(), d_cstart.as<int>(), d_camh.as<int>(), d_camblk.as<int>(), sum);
        if (E > 0) {
            // point CSR in edge order (slots by atomics, each run sorted); camera CSR: that order
            // stably sorted by camera
            launch("ba.init_pfill", init_pfill, dim3(ge), dim3(256), 0, st, E, (const int*)d_ept.as<int>(),
                   (const unsigned char*)d_active.as<unsigned char>(), (const int*)d_pstart.as<int>(), pcur,
                   d_pedges.as<int>());
            if (P > 0)
                launch("ba.init_psort", init_psort, dim3((unsigned)((P + PSORT_WAVES - 1) / PSORT_WAVES)),
                       dim3(PSORT_WAVES * kWave), 0, st, P, (const int*)d_pstart.as<int>(), (const int*)d_ecam.as<int>(),
                       pcur, d_pedges.as<int>(), k0);
            if ((r = stable_key_sort((const unsigned*)k0, (const int*)d_pedges.as<int>(), k1, v0, E, C + 1)) != MAGE_OK)
                return r;
            launch("ba.init_camcsr", init_camcsr, dim3(ge), dim3(256), 0, st, E, C, nbm, (const unsigned*)k1, (const int*)v0,
                   (const int*)d_ept.as<int>(), (const int*)d_camh.as<int>(), (const int*)d_ptfree.as<int>(),
                   d_cedges.as<int>(), d_cpt.as<int>(), d_epos.as<int>(), sum, s_rc);
            launch("ba.init_pcache", init_pcache, dim3(ge), dim3(256), 0, st, E, P, (const int*)d_pstart.as<int>(),
                   (const int*)d_pedges.as<int>(), (const int*)d_ecam.as<int>(), (const int*)d_camh.as<int>(),
                   (const int*)d_epos.as<int>(), d_pe.as<int4>());
        }
        const bool bitmap_fits = PW <= SC_LDS_WORDS && nbm > 0 && P > 0;
        if (bitmap_fits) {
            if ((r = d_sbits.reserve(((size_t)nbm + 1) * PW * 4)) != MAGE_OK) return r;
            if ((r = d_srank.reserve((size_t)nbm * PW * 4)) != MAGE_OK) return r;
            uint32_t* A = d_sbits.as<uint32_t>();
            launch("ba.schur_bitmaps", sc_bitmaps, dim3(nbm + 1), dim3(1024), 0, st, P, (const int*)sum,
                   (const int*)d_camblk.as<int>(), (const int*)d_cstart.as<int>(), (const int*)d_cpt.as<int>(),
                   (const int*)d_ptfree.as<int>(), A, d_srank.as<int>(), A + (size_t)nbm * PW);
            launch("ba.schur_counts", sc_pair_counts, dim3(nbm, nbm), dim3(64), 0, st, (const int*)sum, PW,
                   (const uint32_t*)A, (const uint32_t*)(A + (size_t)nbm * PW), s_kcnt);
        }
        launch("ba.init_summary", summary_out, dim3(1), dim3(1024), 0, st, (const int*)sum, (int)nsum, h_isum.device<int>(),
               seq_dev(), ++seq_counter);
        MAGE_HIP(hipGetLastError());
        if ((r = wait_seq(seq_counter)) != MAGE_OK) return r;
        iacc_clean = true;
        pt.mark("device init + summary");
        const int* hs = h_isum.host<int>();
        const int nb = hs[0], nfp = hs[1], nact = hs[2];
        const bool dup = hs[3] != 0;  // a camera observing a point twice (its CSR run lists the point twice)
        MAGE_REQUIRE(nb <= CH_PANEL_ROWS / 6, MAGE_EUNSUPPORTED, "more than 96 free cameras in one bundle adjustment");
        camh.assign(C, -1);
        cam_of_block.assign(hs + INIT_HDR + C, hs + INIT_HDR + C + nb);
        for (int h = 0; h < nb; h++) camh[cam_of_block[h]] = h;
        camcnt.assign(hs + INIT_HDR, hs + INIT_HDR + C);
        const int* h_rc = hs + INIT_HDR + 2 * C;
        const int* h_kcnt = h_rc + nbm;
        nb_free = nb;
        n = 6 * nb;
        np = (n + 15) / 16 * 16;
        useless = (nb == 0 && nfp == 0);
        n_entries = nact;
        // The iteration's state and buffers now, so the first linearisation runs on the device while
        // the host builds the Schur tables below
        if (!state_on_device) {
            if ((r = upload(d_q[0], q)) != MAGE_OK) return r;
            if ((r = upload(d_t[0], t)) != MAGE_OK) return r;
            if ((r = upload(d_p[0], p)) != MAGE_OK) return r;
            if ((r = d_q[1].reserve(d_q[0].bytes)) != MAGE_OK) return r;
            if ((r = d_t[1].reserve(d_t[0].bytes)) != MAGE_OK) return r;
            if ((r = d_p[1].reserve(d_p[0].bytes)) != MAGE_OK) return r;
            cur = 0;
            state_on_device = true;
        }
        flush_uploads();
        {
            const size_t npm = std::max(np, 16);
            for (auto pr : {std::make_pair(&d_err, Em * 2 * 8), std::make_pair(&d_Hll, Pm * 9 * 8),
                            std::make_pair(&d_bl, Pm * 3 * 8), std::make_pair(&d_Hpl, (size_t)std::max(n_entries, 1) * EQ_N * 8),
                            std::make_pair(&d_Hpp, Cm * 36 * 8), std::make_pair(&d_bp, Cm * 6 * 8),
                            std::make_pair(&d_Z, (size_t)std::max(n_entries, 1) * EG_N * 8),
                            std::make_pair(&d_campart, Cm * CAM_CHUNKS * 27 * 8),
                            std::make_pair(&d_S, npm * npm * 8), std::make_pair(&d_rhs, npm * 8),
                            std::make_pair(&d_x, (npm + 3 * Pm + 1) * 8), std::make_pair(&d_chi, (Pm + teth.size()) * 8),
                            std::make_pair(&d_chi_lin, (Pm + teth.size()) * 8),
                            std::make_pair(&d_tout, std::max<size_t>(teth.size(), 1) * TETHER_OUT * 8),
                            std::make_pair(&d_maxd, (Pm + Cm) * 8), std::make_pair(&d_scale, (Pm + Cm) * 8),
                            std::make_pair(&d_red, (size_t)CTL_DOUBLES * 8), std::make_pair(&d_lm, sizeof(LmDev)),
                            std::make_pair(&d_osum, ((size_t)std::max<int>((int)(Em / BA_THREADS), group_grid((int)Pm)) + 2) * 4 * 8)})
                if ((r = pr.first->reserve(pr.second)) != MAGE_OK) return r;
            if ((r = d_livebuf.reserve(sizeof(LiveCtl))) != MAGE_OK) return r;
            if ((r = h_olist.reserve(Em * 2 * 4 + 16)) != MAGE_OK) return r;
            // one launch clears: the live counters, the max-diagonal / scale partials, S (chol_tiles
            // reads S without writing it and every trial rewrites the same covisible pair blocks, so
            // the zero blocks are set once here; cholesky_solve factors in place: per trial), and
            // on first use the per-edge errors
            ClearList cl{};
            auto add = [&](void* ptr, size_t bytes) {
                cl.p[cl.k] = static_cast<uint32_t*>(ptr);
                cl.n[cl.k++] = (unsigned)(bytes / 4);
            };
            static_assert(sizeof(LiveCtl) % 4 == 0, "LiveCtl is cleared as words");
            add(d_livebuf.ptr, sizeof(LiveCtl));
            add(d_maxd.ptr, (Pm + Cm) * 8);
            add(d_scale.ptr, (Pm + Cm) * 8);
            add(d_S.ptr, npm * npm * 8);
            if (!err_initialized) {
                add(d_err.ptr, Em * 2 * 8);
                err_initialized = true;
            }
            size_t words = 0;
            for (int k = 0; k < cl.k; k++) words = std::max<size_t>(words, cl.n[k]);
            launch("ba.init_clear", clear_words, dim3((unsigned)std::min<size_t>(1024, (words + 255) / 256)), dim3(256),
                   0, st, cl);
        }
        iteration = 0;
        dirty = false;
        eager = false;
        if (!useless && teth.empty()) {
            // the first call's linearisation (the one lm_solve would launch: same huber width,
            // lambda from the user or computeLambdaInit's reduction), taken up by lm_solve
            const bool init = user_lambda <= 0;
            if ((r = linearize(init ? std::numeric_limits<double>::quiet_NaN() : user_lambda, init)) != MAGE_OK) return r;
            eager = true;
            eager_init = init;
            eager_huber = huber;
            eager_lambda = init ? 0.0 : user_lambda;
            eager_cur = cur;
        }
        pt.mark("state + buffers + linearisation");
        const bool bitmaps = !dup && bitmap_fits && nb > 0 && nfp > 0;
        // covisible camera pairs (h1 <= h2) of the reduced system: every pair sharing a free point
        // (a product list), the diagonal, and the tethered pairs
        auto& pairs = ws.pairs;
        pairs.clear();
        auto& pairidx = ws.pairidx;
        pairidx.assign((size_t)std::max(nb, 1) * std::max(nb, 1), -1);
        const int nk = std::max(nb, 1) * std::max(nb, 1);  // dense pair keys h1 * nb + h2
        auto &kcount = ws.kcount, &kstart = ws.kstart;
        kcount.assign(nk, 0);
        kstart.assign(nk, 0);
        long long nprod_max = 0;  // products of the sorted (fallback) lists
        if (bitmaps) {
            for (int x = 0; x < nb; x++)
                for (int y = x; y < nb; y++) kcount[(size_t)x * nb + y] = h_kcnt[(size_t)x * nb + y];
        } else if (nb > 0 && nfp > 0) {
            if ((r = build_product_lists(nb, nact, kstart, kcount, &nprod_max)) != MAGE_OK) return r;
        }
        pt.mark("pair counts");
        if (nb > 0) {
            auto& mark = ws.mark;
            mark.assign((size_t)nb * nb, 0);
            for (int k = 0; k < nb * nb; k++) mark[k] = kcount[k] > 0;
            for (int h = 0; h < nb; h++) mark[(size_t)h * nb + h] = 1;
            for (auto& T : teth) {
                T.h1 = camh[T.c1];
                T.h2 = camh[T.c2];
                if (T.active && T.h1 >= 0 && T.h2 >= 0)
                    mark[(size_t)std::min(T.h1, T.h2) * nb + std::max(T.h1, T.h2)] = 1;
            }
            for (int x = 0; x < nb; x++)
                for (int y = x; y < nb; y++)
                    if (mark[(size_t)x * nb + y]) {
                        pairidx[(size_t)x * nb + y] = (int)pairs.size();
                        pairs.push_back(make_int2(x, y));
                    }
        }
        npairs = (int)pairs.size();
        // per pair: the tethers whose H12 lands in its block (code 2 t + transposed), set order
        auto &ptstart = ws.ptstart, &ptlist = ws.ptlist;
        ptstart.assign(npairs + 1, 0);
        ptlist.clear();
        if (!teth.empty())
            for (int pi = 0; pi < npairs; pi++) {
                for (int ti = 0; ti < (int)teth.size(); ti++) {
                    const Tether& T = teth[ti];
                    if (!T.active || T.h1 < 0 || T.h2 < 0) continue;
                    if (T.h1 == pairs[pi].x && T.h2 == pairs[pi].y) ptlist.push_back(2 * ti);
                    else if (T.h2 == pairs[pi].x && T.h1 == pairs[pi].y) ptlist.push_back(2 * ti + 1);
                }
                ptstart[pi + 1] = (int)ptlist.size();
            }
        // Schur product lists (schur_chunks): per pair the (e1, e2) products of its shared free
        // points in point order, then for a diagonal pair the rhs entries (e, p) in the camera's
        // point order (a camera's free-point edges: rcount)
        auto &pcount = ws.pcount, &rcount = ws.rcount;
        pcount.assign(npairs, 0);
        rcount.assign(npairs, 0);
        for (int pi = 0; pi < npairs; pi++) pcount[pi] = kcount[(size_t)pairs[pi].x * nb + pairs[pi].y];
        auto& rblk = ws.rblk;
        rblk.assign(std::max(nb, 1), 0);
        for (int h = 0; h < nb; h++) rcount[pairidx[(size_t)h * nb + h]] = h_rc[h];
        auto& pbeg = ws.pbeg;
        pbeg.assign(npairs + 1, 0);
        for (int pi = 0; pi < npairs; pi++) pbeg[pi + 1] = pbeg[pi] + pcount[pi] + rcount[pi];
        MAGE_REQUIRE(pbeg[npairs] < (1ll << 31), MAGE_EUNSUPPORTED, "Schur product list exceeds 2^31 entries");
        {
            // destinations: sorted product i of pair key k goes to pbeg[pair] + (i - kstart[k]);
            // camera block h's rhs entries start at pbeg[diag pair] + pcount
            auto& kdst = ws.kdst;
            kdst.assign(nk, 0);
            for (int pi = 0; pi < npairs; pi++) {
                const int k = pairs[pi].x * nb + pairs[pi].y;
                kdst[k] = (int)(pbeg[pi] - kstart[k]);
            }
            for (int h = 0; h < nb; h++) {
                const int pi = pairidx[(size_t)h * nb + h];
                rblk[h] = (int)(pbeg[pi] + pcount[pi]);
            }
            // + the padding entry after the last list (written by schur_rhs)
            if ((r = d_sentries.reserve(((size_t)pbeg[npairs] + 1) * sizeof(int2))) != MAGE_OK) return r;
            if (bitmaps)  // sc_pair_fill: a pair's first product slot (-1: no products)
                for (int k = 0; k < nk; k++) kdst[k] = kcount[k] > 0 ? kdst[k] + kstart[k] : -1;
            if ((r = upload(d_kdst, kdst)) != MAGE_OK) return r;
            if ((r = upload(d_rblk, rblk)) != MAGE_OK) return r;
            flush_uploads();
            if (bitmaps) {
                uint32_t* A = d_sbits.as<uint32_t>();
                launch("ba.schur_fill", sc_pair_fill, dim3(nb, nb), dim3(64), 0, st, nb, PW, (const uint32_t*)A,
                       (const int*)d_srank.as<int>(), (const uint32_t*)(A + (size_t)nbm * PW), (const int*)d_camblk.as<int>(),
                       (const int*)d_cstart.as<int>(), (const int*)d_kdst.as<int>(), d_sentries.as<int2>());
            }
            if (nprod_max > 0)
                launch("ba.schur_scatter", schur_scatter, dim3((unsigned)((nprod_max + 255) / 256)), dim3(256), 0, st,
                       (const uint16_t*)d_skeys.as<uint16_t>() + nprod_pad(nprod_max),
                       (const unsigned long long*)d_svals.as<unsigned long long>() + nprod_pad(nprod_max),
                       (int)nprod_max, (const int*)d_kdst.as<int>(), d_sentries.as<int2>());
            if (nb > 0)
                launch("ba.schur_rhs", schur_rhs, dim3(nb), dim3(256), 0, st, (const int*)d_camblk.as<int>(),
                       (const int*)d_cstart.as<int>(), (const int*)d_cpt.as<int>(), (const int*)d_ptfree.as<int>(),
                       (const int*)d_rblk.as<int>(), d_sentries.as<int2>(), (int)pbeg[npairs]);
            MAGE_HIP(hipGetLastError());
        }
        pt.mark("list scatter");
        // chunks; the block rows of S split into 8 contiguous groups of about equal work, one per
        // XCD (block b runs on XCD b % 8)
        auto& spairs = ws.spairs;
        spairs.assign(npairs, SchurPair{});
        auto& xcd_chunks = ws.xcd_chunks;
        for (auto& v : xcd_chunks) v.clear();
        {
            auto& roww = ws.roww;
            roww.assign(std::max(nb, 1), 0);
            for (int pi = 0; pi < npairs; pi++) roww[pairs[pi].x] += pbeg[pi + 1] - pbeg[pi] + SC_CHUNK / 4;
            long long tot = 0;
            for (long long w : roww) tot += w;
            int slot = 0, x = 0;
            long long acc_w = 0;
            int row = -1;
            for (int pi = 0; pi < npairs; pi++) {
                const int h1 = pairs[pi].x;
                if (h1 != row) {  // next row: move to the next XCD once this one has its share
                    while (x < 7 && acc_w >= (tot * (x + 1) + 7) / 8) x++;
                    row = h1;
                    acc_w += roww[h1];
                }
                const int np_ = (pcount[pi] + SC_CHUNK - 1) / SC_CHUNK, nr = (rcount[pi] + SC_CHUNK - 1) / SC_CHUNK;
                const int nch = std::max(np_ + nr, 1);
                SchurPair& sp = spairs[pi];
                sp.h1 = pairs[pi].x;
                sp.h2 = pairs[pi].y;
                sp.c1 = cam_of_block[sp.h1];
                sp.slot0 = slot;
                sp.nslots = nch;
                sp.tbeg = ptstart[pi];
                sp.tend = ptstart[pi + 1];
                sp.c2 = cam_of_block[sp.h2];
                for (int k = 0; k < nch; k++) {
                    SchurChunk ch{};
                    ch.pair = pi;
                    ch.slot = slot + k;
                    if (k < np_) {
                        ch.kind = 0;
                        ch.start = (int)(pbeg[pi] + (long long)k * SC_CHUNK);
                        ch.count = std::min(SC_CHUNK, pcount[pi] - k * SC_CHUNK);
                    } else if (k - np_ < nr) {
                        ch.kind = 1;
                        ch.start = (int)(pbeg[pi] + pcount[pi] + (long long)(k - np_) * SC_CHUNK);
                        ch.count = std::min(SC_CHUNK, rcount[pi] - (k - np_) * SC_CHUNK);
                    } else {  // nothing to sum (tether-only or empty block): Hpp / tethers only
                        ch.kind = 0;
                        ch.start = (int)pbeg[pi];
                        ch.count = 0;
                    }
                    xcd_chunks[x].push_back(ch);
                }
                slot += nch;
            }
            n_slots = slot;
        }
        size_t L = 0;
        for (auto& v : xcd_chunks) L = std::max(L, v.size());
        auto& schunks = ws.schunks;
        schunks.resize(8 * L);
        for (size_t j = 0; j < L; j++)
            for (int x = 0; x < 8; x++) {
                SchurChunk ch{};
                ch.pair = -1;
                schunks[8 * j + x] = j < xcd_chunks[x].size() ? xcd_chunks[x][j] : ch;
            }
        n_sblocks = (int)schunks.size();
        auto& sfinish = ws.sfinish;  // pairs finished by schur_finish: diagonal or more than one chunk
        sfinish.clear();
        for (int pi = 0; pi < npairs; pi++)
            if (spairs[pi].nslots > 1 || spairs[pi].h1 == spairs[pi].h2) sfinish.push_back(pi);
        n_sfinish = (int)sfinish.size();
        MAGE_REQUIRE(pbeg[npairs] < (1ll << 31), MAGE_EUNSUPPORTED, "Schur product list exceeds 2^31 entries");
        pt.mark("chunks");
        if (np <= 16 * CT_MAXT) {
            chol_tile_table(np / 16, spairs.data(), npairs, ws.ctab);
            if ((r = upload(d_ctab, ws.ctab)) != MAGE_OK) return r;
        }
        if ((r = upload(d_sfinish, sfinish)) != MAGE_OK) return r;
        if ((r = upload(d_spairs, spairs)) != MAGE_OK) return r;
        if ((r = upload(d_schunks, schunks)) != MAGE_OK) return r;
        if ((r = upload(d_ptlist, ptlist)) != MAGE_OK) return r;
        for (auto& T : teth) {
            T.h1 = camh[T.c1];
            T.h2 = camh[T.c2];
        }
        if ((r = upload(d_teth, teth)) != MAGE_OK) return r;
        pt.mark("uploads");
        flush_uploads();
        if ((r = d_spart.reserve((size_t)std::max(n_slots, 1) * 42 * 8)) != MAGE_OK) return r;
        pt.mark("buffers");
        return MAGE_OK;
    }

    // Linearise the current state (errors, Hll/bl/Hpl, Hpp/bp) and reduce chi2 / max diagonal
    // into d_red[0..2]; no host synchronisation.
    // G (edge_schur's records) is valid for this lambda (NaN: not computed)
    double g_lambda = std::numeric_limits<double>::quiet_NaN();
    int eval_blocks() const { return P > 0 ? group_grid(P) : 0; }
    PointOut point_out(double* chi) const
    {
        return PointOut{d_err.as<double>(), d_Hll.as<double>(), d_bl.as<double>(), d_Hpl.as<double>(), d_Z.as<double>(),
                        chi, d_maxd.as<double>()};
    }

    // Linearise the current state (errors, Hll / bl / per-edge records, camera partials) in one
    // launch; with a known lambda (every iteration but the first) also G, so the first trial
    // needs no edge_schur.  init_lambda: linearize_finish reduces chi2 / max diagonal
    // (computeLambdaInit) for the host right away.  No host synchronisation.
    mage_status linearize(double lam_for_g, bool init_lambda)
    {
        Problem pb = problem();
        const int npb = eval_blocks(), ncb = nb_free * CAM_CHUNKS;
        const bool with_g = std::isfinite(lam_for_g) && n_entries > 0 && !points_fixed;
        if (npb + ncb > 0)
            launch("ba.linearize", linearize_kernel, dim3(npb + ncb), dim3(BA_THREADS), 0, st, pb, state(cur),
                   point_out(d_chi_lin.as<double>()), with_g ? lam_for_g : 0.0, with_g ? 1 : 0, npb,
                   (const int*)d_camblk.as<int>(), d_campart.as<double>(), state(1 - cur), (const LmDev*)nullptr);
        g_lambda = with_g ? lam_for_g : std::numeric_limits<double>::quiet_NaN();
        const int nt = (int)teth.size();
        if (nt > 0)
            launch("ba.tether_eval", tether_eval, dim3((nt + 63) / 64), dim3(64), 0, st, (const Tether*)d_teth.as<Tether>(),
                   nt, state(cur), 1, d_chi_lin.as<double>() + P, d_tout.as<double>());
        if (init_lambda)
            launch("ba.linearize_finish", linearize_finish, dim3(1), dim3(1024), 0, st, nb_free, (const int*)d_camblk.as<int>(),
                   (const double*)d_campart.as<double>(), (const double*)d_chi_lin.as<double>(), P,
                   (const double*)d_maxd.as<double>(), (const Tether*)d_teth.as<Tether>(), nt,
                   (const double*)d_tout.as<double>(), d_Hpp.as<double>(), d_bp.as<double>(), h_ctl_dev);
        MAGE_HIP(hipGetLastError());
        return MAGE_OK;
    }

    // One trial: solve with lambda, build the trial state in the other buffer, evaluate it.
    // Reads back red[0..5] = {chi(current), -, -, chi(trial), scale, -} and the fail flag.
    // Speculative linearisation (MAGE_BA_SPEC_LIN, default on): queued behind each trial's reduce3,
    // on the state and lambda of the decision reduce3 takes on the device, so the next trial (after
    // a rejection) or the next call (after an acceptance) starts without the host round trip.
    bool spec_lin = []() {
        const char* v = std::getenv("MAGE_BA_SPEC_LIN");
        return !(v && v[0] == '0');
    }();
    bool spec_lin_queued = false;  // set by trial(): the host adopts the device's lambda
    bool last_call_removed = false;  // the previous StepBundleAdjustment removed outliers
    mage_status trial(double lam, bool* ok, double red[6], bool speculate, double cur_chi = std::numeric_limits<double>::quiet_NaN())
    {
        Problem pb = problem();
        double* xp = d_x.as<double>();
        const int npb = eval_blocks();
        if (n_entries > 0 && !points_fixed && !(g_lambda == lam)) {
            launch("ba.edge_schur", edge_schur, dim3((n_entries + BA_THREADS - 1) / BA_THREADS), dim3(BA_THREADS), 0, st,
                   pb, (const double*)d_Hll.as<double>(), (const double*)d_Hpl.as<double>(), lam, d_Z.as<double>());
            g_lambda = lam;
        }
        if (n > 0) {
            if (np > 16 * CT_MAXT) MAGE_HIP(hipMemsetAsync(d_S.ptr, 0, (size_t)np * np * 8, st));
            launch("ba.schur_pairs", schur_chunks, dim3(n_sblocks), dim3(SC_THREADS), 0, st,
                   (const SchurChunk*)d_schunks.as<SchurChunk>(), (const SchurPair*)d_spairs.as<SchurPair>(),
                   (const int2*)d_sentries.as<int2>(), (const double*)d_Z.as<double>(), (const double*)d_Hpl.as<double>(),
                   (const double*)d_camk.as<double>(), (const double*)d_bl.as<double>(), lam, np, n_entries,
                   (const int*)d_ptlist.as<int>(), (const double*)d_tout.as<double>(), d_spart.as<double>(), d_S.as<double>(),
                   d_rhs.as<double>());
            const FinishArgs fin{(const int*)d_sfinish.as<int>(), n_sfinish, (const SchurPair*)d_spairs.as<SchurPair>(),
                                 (const double*)d_spart.as<double>(), (const double*)d_campart.as<double>(),
                                 (const Tether*)d_teth.as<Tether>(), (int)teth.size(), d_Hpp.as<double>(),
                                 d_bp.as<double>(), lam, (const int*)d_ptlist.as<int>(), (const double*)d_tout.as<double>(),
                                 d_S.as<double>(), d_rhs.as<double>()};
            // (finishing these pairs inside chol_tiles' one workgroup instead measured 65 -> 138 us:
            // the ~14k entries' dependent partial loads serialise on one CU)
            if (n_sfinish > 0) launch("ba.schur_finish", schur_finish, dim3(n_sfinish), dim3(64), 0, st, fin, np);
            if (np <= 16 * CT_MAXT)
                launch("ba.cholesky_solve", chol_tiles, dim3(1), dim3(CT_THREADS), 0, st,
                       (const double*)d_S.as<double>(), np, n, (const double*)d_rhs.as<double>(), xp, d_failp(),
                       (const uint16_t*)d_ctab.as<uint16_t>());
            else
                launch("ba.cholesky_solve", cholesky_solve, dim3(1), dim3(CH_THREADS), 0, st, d_S.as<double>(), np,
                       n, (const double*)d_rhs.as<double>(), xp, d_failp());
        }
        const int ncb = (C + BA_THREADS - 1) / BA_THREADS;
        // the trial state and its evaluation with the speculative post-pass (read back with this sync)
        const bool spec = speculate && E > 0;
        SpecPass sp{state(cur), spec ? 1 : 0, outlier_max_err_sq, h_olist.device<uint32_t>(), E, d_osum.as<double>(), d_live()};
        if (npb + ncb > 0)
            launch("ba.update_evaluate", update_evaluate, dim3(npb + ncb), dim3(BA_THREADS), 0, st, pb,
                   (const double*)d_Z.as<double>(), (const double*)d_Hpl.as<double>(), (const double*)d_Hll.as<double>(),
                   (const double*)d_bl.as<double>(), (const double*)xp, lam, state(cur), state(1 - cur),
                   (const double*)d_bp.as<double>(), d_scale.as<double>(), npb, point_out(d_chi.as<double>()), sp);
        const int nt = (int)teth.size();
        if (nt > 0)
            launch("ba.tether_eval", tether_eval, dim3((nt + 63) / 64), dim3(64), 0, st, (const Tether*)d_teth.as<Tether>(),
                   nt, state(1 - cur), 0, d_chi.as<double>() + P, d_tout.as<double>());
        // (not on a call's last step when the previous call removed outliers: a removal invalidates
        // the linearisation, and the reference's schedule removes some on most calls)
        spec_lin_queued = spec_lin && !(speculate && last_call_removed) && nt == 0 && n > 0 && n_entries > 0 &&
                          !points_fixed && npb + nb_free * CAM_CHUNKS > 0;
        LmDev* lmd = spec_lin_queued ? d_lm.as<LmDev>() : nullptr;
        launch("ba.reduce", reduce3, dim3(1), dim3(1024), 0, st, (const double*)d_chi.as<double>(), P + nt,
               (const double*)d_scale.as<double>(), P + C, (const double*)d_maxd.as<double>(), 0, h_ctl_dev + 3,
               (const double*)d_chi_lin.as<double>(), P + nt, h_ctl_dev + CTL_SCRATCH,
               (const double*)d_osum.as<double>(), npb, spec ? 2 : 0, d_octl(), d_live(), seq_dev(), ++seq_counter,
               lmd, lam, (double)ni, cur, cur_chi, h_ctl_dev + CTL_LMNEXT);
        if (spec_lin_queued)
            launch("ba.linearize", linearize_kernel, dim3(npb + nb_free * CAM_CHUNKS), dim3(BA_THREADS), 0, st, pb,
                   state(0), point_out(d_chi_lin.as<double>()), 0.0, 1, npb, (const int*)d_camblk.as<int>(),
                   d_campart.as<double>(), state(1), (const LmDev*)lmd);
        MAGE_HIP(hipGetLastError());
        mage_status r = wait_seq(seq_counter);
        if (r != MAGE_OK) return r;
        for (int k = 0; k < 6; k++) red[k] = h_ctl[k];
        red[0] = h_ctl[CTL_SCRATCH];  // chi2 of the linearised (current) state
        *ok = ctl_fail() == 0;
        return MAGE_OK;
    }

    // OptimizationAlgorithmLevenberg::solve (g2o); result 1 = OK, 0 = Terminate
    mage_status lm_solve(int* result, bool speculate, int* spec_valid)
    {
        const bool init_lambda = iteration == 0 && user_lambda <= 0;
        if (iteration == 0 && !init_lambda) {
            lambda = user_lambda;
            ni = 2;
        }
        const bool reuse = eager && eager_init == init_lambda && eager_huber == huber && eager_cur == cur &&
                           (init_lambda || eager_lambda == lambda);
        eager = false;
        mage_status r = MAGE_OK;
        if (!reuse && (r = linearize(init_lambda ? std::numeric_limits<double>::quiet_NaN() : lambda, init_lambda)) != MAGE_OK)
            return r;
        double currentChi = 0;
        bool haveChi = false;
        if (init_lambda) {
            if ((r = read_ctl()) != MAGE_OK) return r;
            currentChi = h_ctl[0];
            haveChi = true;
            lambda = 1e-5 * h_ctl[2];  // computeLambdaInit, tau = 1e-5
            ni = 2;
        }
        double rho = 0;
        int qmax = 0;
        do {
            bool ok2 = true;
            double red[6];
            if ((r = trial(lambda, &ok2, red, speculate, haveChi ? currentChi : std::numeric_limits<double>::quiet_NaN())) !=
                MAGE_OK)
                return r;
            // the device's lambda for the next step when a speculative linearisation was queued (the
            // same decision from the same doubles; its pow may differ from the host's in the last bit,
            // and then the queued linearisation is not used)
            const double lam_dev = spec_lin_queued ? h_ctl[CTL_LMNEXT] : 0.0;
            *spec_valid = speculate ? 1 : -1;  // rejected: the current state's result (list 1)
            if (!haveChi) {
                currentChi = red[0];
                haveChi = true;
            }
            double tempChi = red[3];
            if (!ok2) tempChi = std::numeric_limits<double>::max();
            rho = currentChi - tempChi;
            double scale = red[4] + 1e-3;
            rho /= scale;
            stats.trials++;
            if (rho > 0 && std::isfinite(tempChi)) {
                double alpha = 1. - std::pow((2 * rho - 1), 3);
                alpha = std::min(alpha, 2. / 3.);
                double scaleFactor = std::max(1. / 3., alpha);
                lambda *= scaleFactor;
                ni = 2;
                currentChi = tempChi;
                cur = 1 - cur;  // discardTop: the trial state becomes current
                host_state_stale = true;
                *spec_valid = speculate ? 0 : -1;  // accepted (the loop ends): the trial state's list 0
            } else {
                lambda *= ni;
                ni *= 2;
                stats.rejected_trials++;  // pop: the current buffer is unchanged
            }
            if (spec_lin_queued) {
                if (lam_dev == lambda) {
                    // the queued linearisation is of this state and lambda: the next trial's G (no
                    // edge_schur) or the next call's eager linearisation
                    eager = true;
                    eager_init = false;
                    eager_huber = huber;
                    eager_lambda = lambda;
                    eager_cur = cur;
                    g_lambda = lambda;
                } else {
                    // lambda differs in the last bit: the host's (g2o's) lambda holds; the queued
                    // linearisation's G is for the other value (its H and records are still this
                    // state's, so only G is redone, by edge_schur, for the next trial)
                    eager = false;
                    g_lambda = lam_dev;
                }
            }
            qmax++;
        } while (rho < 0 && qmax < 10);
        stats.iterations++;
        stats.last_chi2 = currentChi;
        stats.lambda = lambda;
        *result = (qmax == 10 || rho == 0 || !std::isfinite(lambda)) ? 0 : 1;
        return MAGE_OK;
    }

    mage_status step_once(bool* ok, bool speculate, int* spec_valid)
    {
        mage_status r;
        if (dirty && (r = initialize()) != MAGE_OK) return r;
        if (useless) {
            *ok = false;
            return MAGE_OK;
        }
        int res = 0;
        if ((r = lm_solve(&res, speculate, spec_valid)) != MAGE_OK) return r;
        iteration++;
        *ok = res == 1;
        return MAGE_OK;
    }

    double outlier_max_err_sq = 0;
    // outlier lists and counts (live counters) and inlier (sum, count) block partials of ns states;
    // reduce3 moves them into the control block
    int outlier_blocks() const { return (E + BA_THREADS - 1) / BA_THREADS; }
    void launch_outlier_pass(State s0, State s1, int ns)
    {
        const int ge = outlier_blocks();
        launch("ba.outlier_pass", outlier_pass, dim3(ge), dim3(BA_THREADS), 0, st, problem(), s0, s1, ns, E,
                           d_active.as<unsigned char>(), d_err.as<double>(), outlier_max_err_sq,
                           h_olist.device<uint32_t>(), d_osum.as<double>(), d_live());
    }

    mage_status step(const float* hw, uint32_t nsteps, float maxErrSq, uint32_t* outliers, uint32_t cap,
                     uint32_t* nOut, float* meanSq)
    {
        mage_status r;
        MAGE_HIP(hipSetDevice(device));
        flush_uploads();  // setters' queued copies (camera intrinsics)
        PhaseTimer spt;
        float prior = -1.f;
        // The outlier pass of the final state runs speculatively with the last step's trials
        // (launched before their synchronisation): when the last trial is accepted its result is
        // the pass of the final state and the host skips one round trip.
        outlier_max_err_sq = (double)maxErrSq;
        int spec_valid = -1;  // which speculative outlier result holds for the final state (-1 none)
        for (uint32_t s = 0; s < nsteps; s++) {
            if (hw[s] != prior) {
                huber = (double)hw[s];
                prior = hw[s];
            }
            bool ok = false;
            if ((r = step_once(&ok, s + 1 == nsteps, &spec_valid)) != MAGE_OK) return r;
            if (!ok) break;
        }
        spt.mark("step: LM (incl. initialize)");
        if (dirty) {
            spec_valid = -1;
            if ((r = initialize()) != MAGE_OK) return r;
        }
        if (E == 0) {
            *nOut = 0;
            *meanSq = std::numeric_limits<float>::quiet_NaN();
            return MAGE_OK;
        }
        int k = spec_valid;
        if (k < 0) {
            launch_outlier_pass(state(cur), state(cur), 1);
            // its block partials -> ctl->osum[0] (the chi2 outputs go to a scratch slot)
            launch("ba.reduce", reduce3, dim3(1), dim3(1024), 0, st, (const double*)nullptr, 0, (const double*)nullptr, 0,
                   (const double*)nullptr, 0, h_ctl_dev + CTL_SCRATCH, (const double*)nullptr, 0,
                   h_ctl_dev + CTL_SCRATCH, (const double*)d_osum.as<double>(), outlier_blocks(), 1, d_octl(), d_live(),
                   seq_dev(), ++seq_counter, (LmDev*)nullptr, 0.0, 0.0, 0, 0.0, (double*)nullptr);
            MAGE_HIP(hipGetLastError());
            if ((r = read_ctl()) != MAGE_OK) return r;
            k = 0;
        }
        const double h[2] = {h_octl().osum[k][0], h_octl().osum[k][1]};
        const uint32_t no = h_octl().count[k];
        last_call_removed = no > 0;
        if (no > 0) {
            // the pass wrote the list into mapped host memory before the completion word
            const uint32_t* h_list = h_olist.host<uint32_t>() + (size_t)k * E;
            std::vector<uint32_t> list(h_list, h_list + no);
            launch("ba.drop_edges", drop_edges, dim3((no + BA_THREADS - 1) / BA_THREADS), dim3(BA_THREADS), 0, st,
                   (const int*)d_ept.as<int>(), (const uint32_t*)(h_olist.device<uint32_t>() + (size_t)k * E), no,
                   d_active.as<unsigned char>(), d_removed.as<unsigned char>(), d_ptcnt.as<int>(), d_ptfree.as<int>());
            std::sort(list.begin(), list.end());  // g2o active-edge order = insertion order
            for (uint32_t k = 0; k < no; k++) {
                camcnt[ecam[list[k]]]--;
                if (k < cap) outliers[k] = list[k];
            }
            // a free camera without edges changes the block numbering -> full re-initialisation
            for (int c = 0; c < C; c++)
                if (camh[c] >= 0 && camcnt[c] == 0 && cam_tethers[c] == 0) dirty = true;
            iteration = 0;  // removeEdge dirties the optimizer: next Step re-initialises (lambda init)
            eager = false;  // a speculative linearisation ran before the removal
        }
        *nOut = std::min(no, cap);
        *meanSq = (float)(h[0] / h[1]);
        spt.mark("step: outliers");
        // Eager linearisation for the caller's usual next call (BundleAdjust.cpp:311-318: the same
        // huber width, no setter in between): it runs while control is with the caller, and
        // lm_solve reuses it only when the huber width, lambda and state still match.
        // the mirror is written when the caller reads the state between steps (UpdateData after every
        // StepBundleAdjustment, BundleAdjust.cpp:400-403); a caller that stops reading stops paying for it
        if (host_state_stale && export_wanted) launch_export();
        export_wanted = false;
        // After an outlier removal the next Step starts at iteration 0 (lambda re-initialised from
        // the user lambda or computeLambdaInit): the eager linearisation is that iteration's, with
        // the reduction computeLambdaInit reads when no user lambda is set.
        const bool init_next = iteration == 0 && user_lambda <= 0;
        const double lam_next = iteration > 0 ? lambda : user_lambda;
        const bool pending = eager && eager_init == init_next && eager_huber == huber && eager_cur == cur &&
                             (init_next || eager_lambda == lam_next);  // (initialize() just launched it)
        if (!dirty && !useless && !pending) {
            const bool init = init_next;
            const double lam = lam_next;
            if ((r = linearize(init ? std::numeric_limits<double>::quiet_NaN() : lam, init)) != MAGE_OK) return r;
            eager = true;
            eager_init = init;
            eager_huber = huber;
            eager_lambda = init ? 0.0 : lam;
            eager_cur = cur;
        }
        spt.mark("step: export + eager");
        return no > cap ? MAGE_ECAPACITY : MAGE_OK;
    }
};

}  // namespace mage

struct mage_ba : mage::BundleAdjuster {};

extern "C" {

mage_status mage_ba_create(int32_t points_fixed, int device, mage_ba** out)
{
    MAGE_REQUIRE(out, MAGE_EINVAL, "null output");
    *out = nullptr;
    mage_status r = mage::bind_device(device);
    if (r != MAGE_OK) return r;
    auto* b = new mage_ba();
    b->device = device;
    b->points_fixed = points_fixed != 0;
    // a retired stream / control block of an earlier instance when there is one (MakeBundler
    // creates a BundlerLib per local-BA window; creation and hipHostFree cost ~0.1 ms each)
    size_t ctl_bytes = 0;
    b->st = mage::stream_take();
    b->h_ctl = static_cast<double*>(mage::pool_take(2, mage::BundleAdjuster::CTL_DOUBLES * sizeof(double), &ctl_bytes));
    if ((!b->st && hipStreamCreateWithFlags(&b->st, hipStreamNonBlocking) != hipSuccess) ||
        (!b->h_ctl && (ctl_bytes = mage::BundleAdjuster::CTL_DOUBLES * sizeof(double),
                       hipHostMalloc(reinterpret_cast<void**>(&b->h_ctl), ctl_bytes,
                                     hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)) ||
        (b->ctl_bytes = ctl_bytes, false) ||
        hipHostGetDevicePointer(reinterpret_cast<void**>(&b->h_ctl_dev), b->h_ctl, 0) != hipSuccess ||
        (std::memset(b->h_ctl, 0, mage::BundleAdjuster::CTL_DOUBLES * sizeof(double)), false)) {
        b->release();
        delete b;
        mage::set_error("hipStreamCreate / hipHostMalloc failed");
        return MAGE_EDEVICE;
    }
    *out = b;
    return MAGE_OK;
}

mage_status mage_ba_destroy(mage_ba* ba)
{
    if (!ba) return MAGE_OK;
    (void)hipSetDevice(ba->device);
    ba->release();
    delete ba;
    return MAGE_OK;
}

mage_status mage_ba_set_cameras(mage_ba* b, uint32_t n, const float* pos3, const float* r9, const float* intr4,
                                const uint8_t* fixed)
{
    mage::BundleAdjuster::ScopeTimer timer_("call " "set_cameras");
    MAGE_REQUIRE(b && (n == 0 || (pos3 && r9 && intr4)), MAGE_EINVAL, "null argument");
    MAGE_REQUIRE(!b->state_on_device || (int)n == b->C, MAGE_EINVAL, "cameras can only be allocated once");
    b->C = (int)n;
    b->q.assign(4 * n, 0);
    b->t.assign(3 * n, 0);
    b->camk.assign(3 * n, 0);
    b->fixed.assign(n, 0);
    for (uint32_t i = 0; i < n; i++) {
        // Eigen::Quaternionf{Map<const Matrix3f>}.normalized() in float (BundlerLib.cpp:271-273),
        // the column-major map read as m(r,c) = r9[c*3+r]
        float m[9];
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) m[r * 3 + c] = r9[9 * i + c * 3 + r];
        float qf[4];
        float tr = m[0] + m[4] + m[8];
        if (tr > 0.f) {
            float s = std::sqrt(tr + 1.0f);
            qf[3] = 0.5f * s;
            s = 0.5f / s;
            qf[0] = (m[7] - m[5]) * s;
            qf[1] = (m[2] - m[6]) * s;
            qf[2] = (m[3] - m[1]) * s;
        } else {
            int a = 0;
            if (m[4] > m[0]) a = 1;
            if (m[8] > m[a * 4]) a = 2;
            int j = (a + 1) % 3, k = (j + 1) % 3;
            float s = std::sqrt(m[a * 4] - m[j * 4] - m[k * 4] + 1.0f);
            qf[a] = 0.5f * s;
            s = 0.5f / s;
            qf[3] = (m[k * 3 + j] - m[j * 3 + k]) * s;
            qf[j] = (m[j * 3 + a] + m[a * 3 + j]) * s;
            qf[k] = (m[k * 3 + a] + m[a * 3 + k]) * s;
        }
        float nrm = std::sqrt(qf[0] * qf[0] + qf[1] * qf[1] + qf[2] * qf[2] + qf[3] * qf[3]);
        double qd[4];
        for (int k = 0; k < 4; k++) qd[k] = (double)(qf[k] / nrm);
        // SE3Quat(q, t) normalizeRotation
        if (qd[3] < 0)
            for (int k = 0; k < 4; k++) qd[k] = -qd[k];
        double dn = std::sqrt(qd[0] * qd[0] + qd[1] * qd[1] + qd[2] * qd[2] + qd[3] * qd[3]);
        for (int k = 0; k < 4; k++) b->q[4 * i + k] = qd[k] / dn;
        for (int k = 0; k < 3; k++) b->t[3 * i + k] = (double)pos3[3 * i + k];
        // CameraParameters(intrinsics[2], (intrinsics[0], intrinsics[1]), 0) (BundlerLib.cpp:266)
        b->camk[3 * i] = (double)intr4[4 * i + 2];
        b->camk[3 * i + 1] = (double)intr4[4 * i + 0];
        b->camk[3 * i + 2] = (double)intr4[4 * i + 1];
        b->fixed[i] = fixed ? (fixed[i] != 0) : 0;
    }
    b->dirty = true;
    b->state_on_device = false;
    (void)hipSetDevice(b->device);
    return b->upload(b->d_camk, b->camk);
}

mage_status mage_ba_fix_camera(mage_ba* b, uint32_t idx, int32_t fixed)
{
    MAGE_REQUIRE(b && (int)idx < b->C, MAGE_EINVAL, "bad camera index");
    b->fixed[idx] = fixed != 0;  // setFixed does not dirty the optimizer (BundlerLib.cpp:280-283)
    return MAGE_OK;
}

mage_status mage_ba_set_points(mage_ba* b, uint32_t n, const float* xyz)
{
    mage::BundleAdjuster::ScopeTimer timer_("call " "set_points");
    MAGE_REQUIRE(b && (n == 0 || xyz), MAGE_EINVAL, "null argument");
    mage_status r = b->sync_host_state();
    if (r != MAGE_OK) return r;
    b->P = (int)n;
    b->p.assign(3 * n, 0);
    for (uint32_t i = 0; i < 3 * n; i++) b->p[i] = (double)xyz[i];
    b->dirty = true;
    b->state_on_device = false;
    return MAGE_OK;
}

mage_status mage_ba_set_observations(mage_ba* b, uint32_t n, const float* uv, const uint32_t* cam,
                                     const uint32_t* pt, const float* info)
{
    mage::BundleAdjuster::ScopeTimer timer_("call " "set_observations");
    MAGE_REQUIRE(b && (n == 0 || (uv && cam && pt && info)), MAGE_EINVAL, "null argument");
    uint32_t cmax = 0, pmax = 0;
    for (uint32_t i = 0; i < n; i++) {
        cmax = std::max(cmax, cam[i]);
        pmax = std::max(pmax, pt[i]);
    }
    MAGE_REQUIRE(n == 0 || (cmax < (uint32_t)b->C && pmax < (uint32_t)b->P), MAGE_EINVAL,
                 "observation index out of range");
    b->E = (int)n;
    b->ecam.assign(cam, cam + n);
    b->dirty = true;
    (void)hipSetDevice(b->device);
    // the measurements stay float on the device (exact in the kernels' double arithmetic, as the
    // reference's Vector2d(float) measurement); the removal flags start clear
    mage_status r;
    if ((r = b->upload(b->d_uv, uv, 2 * (size_t)n)) != MAGE_OK) return r;
    if ((r = b->upload(b->d_info, info, n)) != MAGE_OK) return r;
    if ((r = b->upload(b->d_ecam, reinterpret_cast<const int*>(cam), n)) != MAGE_OK) return r;
    if ((r = b->upload(b->d_ept, reinterpret_cast<const int*>(pt), n)) != MAGE_OK) return r;
    if ((r = b->d_removed.reserve(std::max<size_t>(n, 16))) != MAGE_OK) return r;
    MAGE_HIP(hipMemsetAsync(b->d_removed.ptr, 0, n, b->st));
    return MAGE_OK;
}
mage_status mage_ba_set_lambda(mage_ba* b, float lambda)
{
    MAGE_REQUIRE(b, MAGE_EINVAL, "null handle");
    b->iteration = 0;  // StepOptimizer::SetCurrentLambda (BundlerLib.cpp:123-130)
    b->user_lambda = (double)lambda;
    b->eager = false;
    return MAGE_OK;
}

mage_status mage_ba_get_lambda(mage_ba* b, float* lambda)
{
    MAGE_REQUIRE(b && lambda, MAGE_EINVAL, "null argument");
    *lambda = (float)b->lambda;
    return MAGE_OK;
}

mage_status mage_ba_set_tethers(mage_ba* b, uint32_t kind, uint32_t n, const uint32_t* cam1, const uint32_t* cam2,
                                const float* params, const float* weight)
{
    MAGE_REQUIRE(b, MAGE_EINVAL, "null handle");
    MAGE_REQUIRE(kind <= MAGE_TETHER_TRANSFORM, MAGE_EINVAL, "unknown tether kind");
    MAGE_REQUIRE(n == 0 || (cam1 && cam2 && params && weight), MAGE_EINVAL, "null argument");
    for (uint32_t i = 0; i < n; i++) {
        MAGE_REQUIRE((int)cam1[i] < b->C && (int)cam2[i] < b->C, MAGE_EINVAL, "tether camera index out of range");
        MAGE_REQUIRE(cam1[i] != cam2[i], MAGE_EINVAL, "tether joins a camera to itself");
    }
    // Allocate*Constraints + Set*Constraint for one kind; the other kinds are kept, and the edge
    // order is distance, rotation, transform as BuildDataForG2O adds them (BundleAdjust.cpp:155-189)
    std::vector<mage::ba::Tether> nt;
    const int stride = kind == MAGE_TETHER_DISTANCE ? 1 : kind == MAGE_TETHER_ROTATION ? 4 : 7;
    for (uint32_t k = 0; k <= MAGE_TETHER_TRANSFORM; k++) {
        if (k != kind) {
            for (const auto& T : b->teth)
                if ((uint32_t)T.kind == k) nt.push_back(T);
            continue;
        }
        for (uint32_t i = 0; i < n; i++) {
            mage::ba::Tether T{};
            const float* pr = params + (size_t)stride * i;
            T.kind = (int)kind;
            T.c1 = (int)cam1[i];
            T.c2 = (int)cam2[i];
            T.h1 = T.h2 = -1;
            T.w = (double)weight[i];
            if (kind == MAGE_TETHER_DISTANCE) {
                T.dist = (double)pr[0];
            } else if (kind == MAGE_TETHER_ROTATION) {
                for (int a = 0; a < 4; a++) T.mq[a] = (double)pr[a];  // setMeasurement, not normalised
            } else {
                for (int a = 0; a < 3; a++) T.mt[a] = (double)pr[a];
                double q[4];
                for (int a = 0; a < 4; a++) q[a] = (double)pr[3 + a];
                if (q[3] < 0)  // SE3Quat(q, t): normalizeRotation
                    for (int a = 0; a < 4; a++) q[a] = -q[a];
                const double nq = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
                for (int a = 0; a < 4; a++) T.mq[a] = q[a] / nq;
            }
            nt.push_back(T);
        }
    }
    b->teth.swap(nt);
    b->dirty = true;  // addEdge dirties the StepOptimizer
    return MAGE_OK;
}

mage_status mage_ba_step(mage_ba* b, const float* huber, uint32_t nsteps, float max_error_square, uint32_t* outliers,
                         uint32_t cap, uint32_t* n_out, float* mean_sq)
{
    mage::BundleAdjuster::ScopeTimer timer_("call " "step");
    MAGE_REQUIRE(b && n_out && mean_sq && (nsteps == 0 || huber) && (cap == 0 || outliers), MAGE_EINVAL,
                 "null argument");
    for (uint32_t s = 0; s < nsteps; s++) MAGE_REQUIRE(huber[s] >= 0.f, MAGE_EINVAL, "Huber widths must be nonnegative");
    return b->step(huber, nsteps, max_error_square, outliers, cap, n_out, mean_sq);
}

mage_status mage_ba_get_poses(mage_ba* b, float* pos3, float* r9)
{
    mage::BundleAdjuster::ScopeTimer timer_("call " "get_poses");
    MAGE_REQUIRE(b && pos3 && r9, MAGE_EINVAL, "null argument");
    (void)hipSetDevice(b->device);
    b->export_wanted = true;  // GetPose / GetPoint between steps: keep the mapped mirror current
    if (const float* m = b->exported()) {
        std::memcpy(pos3, m, sizeof(float) * 3 * b->C);
        std::memcpy(r9, m + 3 * b->C, sizeof(float) * 9 * b->C);
        return MAGE_OK;
    }
    mage_status r = b->sync_host_state();
    if (r != MAGE_OK) return r;
    for (int c = 0; c < b->C; c++) {
        // GetPose (BundlerLib.cpp:457-465): t, R of the normalised quaternion, cast to float
        double q[4] = {b->q[4 * c], b->q[4 * c + 1], b->q[4 * c + 2], b->q[4 * c + 3]};
        double nn = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
        for (double& v : q) v /= nn;
        double tx = 2 * q[0], ty = 2 * q[1], tz = 2 * q[2];
        double twx = tx * q[3], twy = ty * q[3], twz = tz * q[3];
        double txx = tx * q[0], txy = ty * q[0], txz = tz * q[0];
        double tyy = ty * q[1], tyz = tz * q[1], tzz = tz * q[2];
        const double R[9] = {1 - (tyy + tzz), txy - twz, txz + twy, txy + twz, 1 - (txx + tzz),
                             tyz - twx,       txz - twy, tyz + twx, 1 - (txx + tyy)};
        for (int k = 0; k < 3; k++) pos3[3 * c + k] = (float)b->t[3 * c + k];
        for (int rr = 0; rr < 3; rr++)
            for (int cc = 0; cc < 3; cc++) r9[9 * c + cc * 3 + rr] = (float)R[rr * 3 + cc];
    }
    return MAGE_OK;
}

mage_status mage_ba_get_points(mage_ba* b, float* xyz)
{
    mage::BundleAdjuster::ScopeTimer timer_("call " "get_points");
    MAGE_REQUIRE(b && xyz, MAGE_EINVAL, "null argument");
    (void)hipSetDevice(b->device);
    b->export_wanted = true;  // GetPose / GetPoint between steps: keep the mapped mirror current
    if (const float* m = b->exported()) {
        std::memcpy(xyz, m + 12 * b->C, sizeof(float) * 3 * b->P);
        return MAGE_OK;
    }
    mage_status r = b->sync_host_state();
    if (r != MAGE_OK) return r;
    for (int i = 0; i < 3 * b->P; i++) xyz[i] = (float)b->p[i];
    return MAGE_OK;
}

mage_status mage_ba_get_state_f64(mage_ba* b, double* qt7, double* xyz)
{
    MAGE_REQUIRE(b, MAGE_EINVAL, "null handle");
    (void)hipSetDevice(b->device);
    mage_status r = b->sync_host_state();  // fp64: a D2H copy (the mapped mirror holds GetPose / GetPoint's floats)
    if (r != MAGE_OK) return r;
    if (qt7)
        for (int c = 0; c < b->C; c++) {
            for (int k = 0; k < 4; k++) qt7[7 * c + k] = b->q[4 * c + k];
            for (int k = 0; k < 3; k++) qt7[7 * c + 4 + k] = b->t[3 * c + k];
        }
    if (xyz)
        for (int i = 0; i < 3 * b->P; i++) xyz[i] = b->p[i];
    return MAGE_OK;
}

mage_status mage_ba_get_stats(mage_ba* b, mage_ba_stats* s)
{
    MAGE_REQUIRE(b && s, MAGE_EINVAL, "null argument");
    *s = b->stats;
    return MAGE_OK;
}

}  // extern "C"
