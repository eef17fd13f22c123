// ba_math.hpp — fp64 SE3Quat / Eigen / g2o primitives shared by the BA kernels (device code).
// Restates g2o se3quat.h (exp, map, normalizeRotation), Eigen Quaternion (transformVector,
// toRotationMatrix, from-matrix) and EdgeProjectXYZ2UV / RobustKernelHuber as used by BundlerLib.
#pragma once
#include <hip/hip_runtime.h>

namespace mage {
namespace ba {

// ---------------- SE3Quat / Eigen primitives (device) ----------------

__device__ __forceinline__ void d_cross(const double a[3], const double b[3], double c[3])
{
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}

// Quaternion * Vector3 (Eigen _transformVector); q = (x, y, z, w)
__device__ __forceinline__ void d_qrot(const double q[4], const double v[3], double o[3])
{
    double uv[3], uv2[3];
    d_cross(q, v, uv);
    uv[0] += uv[0];
    uv[1] += uv[1];
    uv[2] += uv[2];
    d_cross(q, uv, uv2);
    for (int i = 0; i < 3; i++) o[i] = v[i] + q[3] * uv[i] + uv2[i];
}

__device__ __forceinline__ void d_qmat(const double q[4], double r[9])
{
    double tx = 2 * q[0], ty = 2 * q[1], tz = 2 * q[2];
    double twx = tx * q[3], twy = ty * q[3], twz = tz * q[3];
    double txx = tx * q[0], txy = ty * q[0], txz = tz * q[0];
    double tyy = ty * q[1], tyz = tz * q[1], tzz = tz * q[2];
    r[0] = 1 - (tyy + tzz);
    r[1] = txy - twz;
    r[2] = txz + twy;
    r[3] = txy + twz;
    r[4] = 1 - (txx + tzz);
    r[5] = tyz - twx;
    r[6] = txz - twy;
    r[7] = tyz + twx;
    r[8] = 1 - (txx + tyy);
}

// Eigen's non-positive-trace branch for the largest diagonal element I, with constant indices
// (indexing m by a run-time i placed the matrix in scratch memory on every call: five stores per
// call, i.e. per BA edge in update_evaluate)
template <int I>
__device__ __forceinline__ void d_quat_case(const double* m, double q[4])
{
    constexpr int i = I, j = (i + 1) % 3, k = (j + 1) % 3;
    double t = sqrt(m[i * 4] - m[j * 4] - m[k * 4] + 1.0);
    q[i] = 0.5 * t;
    t = 0.5 / t;
    q[3] = (m[k * 3 + j] - m[j * 3 + k]) * t;
    q[j] = (m[j * 3 + i] + m[i * 3 + j]) * t;
    q[k] = (m[k * 3 + i] + m[i * 3 + k]) * t;
}

__device__ __forceinline__ void d_quat_from_matrix(const double* m, double q[4])
{
    double t = m[0] + m[4] + m[8];
    if (t > 0) {
        t = sqrt(t + 1.0);
        q[3] = 0.5 * t;
        t = 0.5 / t;
        q[0] = (m[7] - m[5]) * t;
        q[1] = (m[2] - m[6]) * t;
        q[2] = (m[3] - m[1]) * t;
    } else {
        int i = 0;
        if (m[4] > m[0]) i = 1;
        if (m[8] > (i == 1 ? m[4] : m[0])) i = 2;
        if (i == 0)
            d_quat_case<0>(m, q);
        else if (i == 1)
            d_quat_case<1>(m, q);
        else
            d_quat_case<2>(m, q);
    }
}

__device__ __forceinline__ void d_se3_normalize(double q[4])
{
    if (q[3] < 0)
        for (int i = 0; i < 4; i++) q[i] = -q[i];
    double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    for (int i = 0; i < 4; i++) q[i] /= n;
}

// T <- exp(u) * T  (VertexSE3Expmap::oplusImpl with SE3Quat::exp, g2o se3quat.h)
__device__ void d_oplus(double q[4], double t[3], const double u[6])
{
    const double w0 = u[0], w1 = u[1], w2 = u[2];
    const double theta = sqrt(w0 * w0 + w1 * w1 + w2 * w2);
    const double O[9] = {0, -w2, w1, w2, 0, -w0, -w1, w0, 0};
    double O2[9];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) O2[r * 3 + c] = O[r * 3] * O[c] + O[r * 3 + 1] * O[3 + c] + O[r * 3 + 2] * O[6 + c];
    double R[9], V[9];
    if (theta < 0.00001) {
        for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0 ? 1.0 : 0.0) + O[i] + O2[i];
        for (int i = 0; i < 9; i++) V[i] = R[i];
    } else {
        const double a = sin(theta) / theta, b = (1 - cos(theta)) / (theta * theta);
        const double c = (theta - sin(theta)) / (theta * theta * theta);
        for (int i = 0; i < 9; i++) {
            const double I = (i % 4 == 0 ? 1.0 : 0.0);
            R[i] = I + a * O[i] + b * O2[i];
            V[i] = I + b * O[i] + c * O2[i];
        }
    }
    double eq[4], et[3];
    d_quat_from_matrix(R, eq);
    for (int r = 0; r < 3; r++) et[r] = V[r * 3] * u[3] + V[r * 3 + 1] * u[4] + V[r * 3 + 2] * u[5];
    d_se3_normalize(eq);
    // result = e * T: t' = e.t + e.q * T.t ; q' = e.q * T.q
    double rt[3];
    d_qrot(eq, t, rt);
    double nq[4];
    nq[3] = eq[3] * q[3] - eq[0] * q[0] - eq[1] * q[1] - eq[2] * q[2];
    nq[0] = eq[3] * q[0] + eq[0] * q[3] + eq[1] * q[2] - eq[2] * q[1];
    nq[1] = eq[3] * q[1] + eq[1] * q[3] + eq[2] * q[0] - eq[0] * q[2];
    nq[2] = eq[3] * q[2] + eq[2] * q[3] + eq[0] * q[1] - eq[1] * q[0];
    d_se3_normalize(nq);
    for (int i = 0; i < 4; i++) q[i] = nq[i];
    for (int i = 0; i < 3; i++) t[i] = et[i] + rt[i];
}

__device__ __forceinline__ void d_huber(double delta, double e2, double& rho0, double& rho1)
{
    const double dsqr = delta * delta;
    if (e2 <= dsqr) {
        rho0 = e2;
        rho1 = 1.0;
    } else {
        const double sq = sqrt(e2);
        rho0 = 2 * sq * delta - dsqr;
        rho1 = delta / sq;
    }
}

// ---------------- tether edges (BundlerLib.cpp:22-88, 311-350; g2o EdgeSE3Expmap) ----------------

struct Tether {
    int kind;    // 0 EdgeScaleConstraint (distance), 1 EdgeRotationConstraint, 2 EdgeSE3Expmap
    int c1, c2;  // cameras (vertex 0, vertex 1)
    int h1, h2;  // their Hessian blocks, -1 if not in the system
    int active;  // not both cameras fixed
    double w;    // weight (kinds 0, 1: inside the error) / information scale (kind 2)
    double dist; // kind 0 measurement
    double mq[4], mt[3];  // kind 1: rotation (x, y, z, w, as given); kind 2: SE3Quat(q, t)
};

// per-tether linearisation record: H11, H22, H12 (6x6 row-major), b1, b2
constexpr int TETHER_OUT = 3 * 36 + 12;

__device__ __forceinline__ void d_qmul(const double a[4], const double b[4], double o[4])
{
    const double w = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
    const double x = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
    const double y = a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2];
    const double z = a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0];
    o[0] = x;
    o[1] = y;
    o[2] = z;
    o[3] = w;
}

// SE3Quat::inverse
__device__ __forceinline__ void d_se3_inv(const double q[4], const double t[3], double oq[4], double ot[3])
{
    oq[0] = -q[0];
    oq[1] = -q[1];
    oq[2] = -q[2];
    oq[3] = q[3];
    const double mt[3] = {-t[0], -t[1], -t[2]};
    d_qrot(oq, mt, ot);
}

// SE3Quat::operator* (normalizeRotation on the product)
__device__ __forceinline__ void d_se3_mul(const double aq[4], const double at[3], const double bq[4],
                                          const double bt[3], double oq[4], double ot[3])
{
    double rt[3];
    d_qrot(aq, bt, rt);
    for (int i = 0; i < 3; i++) ot[i] = at[i] + rt[i];
    d_qmul(aq, bq, oq);
    d_se3_normalize(oq);
}

__device__ __forceinline__ void d_skew(const double v[3], double m[9])
{
    m[0] = 0;
    m[1] = -v[2];
    m[2] = v[1];
    m[3] = v[2];
    m[4] = 0;
    m[5] = -v[0];
    m[6] = -v[1];
    m[7] = v[0];
    m[8] = 0;
}

// SE3Quat::log -> (omega, upsilon)
__device__ void d_se3_log(const double q[4], const double t[3], double res[6])
{
    double R[9];
    d_qmat(q, R);
    const double d = 0.5 * (R[0] + R[4] + R[8] - 1);
    const double dR[3] = {R[7] - R[5], R[2] - R[6], R[3] - R[1]};
    double omega[3], Om[9];
    double k;
    if (fabs(d) > 0.99999) {
        for (int i = 0; i < 3; i++) omega[i] = 0.5 * dR[i];
        k = 1.0 / 12.0;
    } else {
        const double theta = acos(d);
        const double s = theta / (2 * sqrt(1 - d * d));
        for (int i = 0; i < 3; i++) omega[i] = s * dR[i];
        k = (1 - theta / (2 * tan(theta / 2))) / (theta * theta);
    }
    d_skew(omega, Om);
    for (int r = 0; r < 3; r++) {
        double row[3];
        for (int c = 0; c < 3; c++) {
            const double o2 = Om[r * 3] * Om[c] + Om[r * 3 + 1] * Om[3 + c] + Om[r * 3 + 2] * Om[6 + c];
            row[c] = (r == c ? 1.0 : 0.0) - 0.5 * Om[r * 3 + c] + k * o2;
        }
        res[r] = omega[r];
        res[3 + r] = row[0] * t[0] + row[1] * t[1] + row[2] * t[2];
    }
}

// SE3Quat::adj (6x6 row-major), negated if neg
__device__ void d_se3_adj(const double q[4], const double t[3], bool neg, double A[36])
{
    double R[9], St[9];
    d_qmat(q, R);
    d_skew(t, St);
    const double sg = neg ? -1.0 : 1.0;
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) {
            const double sr = St[r * 3] * R[c] + St[r * 3 + 1] * R[3 + c] + St[r * 3 + 2] * R[6 + c];
            A[r * 6 + c] = sg * R[r * 3 + c];
            A[r * 6 + 3 + c] = 0.0 * sg;
            A[(3 + r) * 6 + c] = sg * sr;
            A[(3 + r) * 6 + 3 + c] = sg * R[r * 3 + c];
        }
}

// computeError of a tether for camera estimates (q1, t1), (q2, t2); returns the dimension
__device__ int d_tether_error(const Tether& T, const double q1[4], const double t1[3], const double q2[4],
                              const double t2[3], double e[6])
{
    if (T.kind == 0) {
        const double dx = t2[0] - t1[0], dy = t2[1] - t1[1], dz = t2[2] - t1[2];
        e[0] = (T.dist - sqrt(dx * dx + dy * dy + dz * dz)) * T.w;
        return 1;
    }
    if (T.kind == 1) {
        double iq[4], it[3], rq[4], rt[3];
        d_se3_inv(q1, t1, iq, it);
        d_se3_mul(iq, it, q2, t2, rq, rt);
        const double mc[4] = {-T.mq[0], -T.mq[1], -T.mq[2], T.mq[3]};
        double d[4];
        d_qmul(rq, mc, d);
        const double vn = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
        e[0] = 2.0 * atan2(vn, fabs(d[3])) * T.w;
        return 1;
    }
    double iq[4], it[3], aq[4], at[3], rq[4], rt[3];
    d_se3_inv(q2, t2, iq, it);
    d_se3_mul(iq, it, T.mq, T.mt, aq, at);
    d_se3_mul(aq, at, q1, t1, rq, rt);
    d_se3_log(rq, rt, e);
    return 6;
}

struct State {  // one copy of the optimisable state
    double* q;  // C x 4
    double* t;  // C x 3
    double* p;  // P x 3
};

struct Problem {
    int C, P;
    const double* camk;           // C x 3: f, cx, cy
    const int* camh;              // C: Hessian block index or -1
    const int* ptfree;            // P: 1 if the point is in the system
    const float* uv;              // E x 2 (the caller's float measurements)
    const int* ecam;              // E
    const int* ept;               // E
    const float* info;            // E
    const unsigned char* active;  // E: edge in the optimizer's active set
    const int* pstart;            // P+1
    const int* pedges;            // edges by point (edge order), filtered by `active`
    const int* cstart;            // C+1
    const int* cedges;            // edges by camera, sorted by point id, filtered by `active`
    const int* cpt;               // point id of each cedges entry (binary search key)
    const int* epos;              // E: position of the edge in the camera CSR (-1: not listed)
    const int4* pe;               // per point-CSR entry: (edge, camera, camera block or -1, camera-CSR
                                  // position) in one 16-byte load (init_pcache)
    int ecsr;                     // camera-CSR entries = row stride of the Hpl / Z component arrays
    double huber;
};

// computeError + chi2 + robustify for edge e of camera c with its camera pose (q, t) and point X
// given (the callers know c and X, so the edge's own loads are uv and info only)
__device__ __forceinline__ void edge_eval_at(const Problem& pb, int e, int c, const double q[4], const double t[3],
                                             const double X[3], double err[2], double xc[3], double& rho0,
                                             double& rho1)
{
    d_qrot(q, X, xc);
    xc[0] += t[0];
    xc[1] += t[1];
    xc[2] += t[2];
    const double f = pb.camk[3 * c], cx = pb.camk[3 * c + 1], cy = pb.camk[3 * c + 2];
    err[0] = pb.uv[2 * e] - (xc[0] / xc[2] * f + cx);
    err[1] = pb.uv[2 * e + 1] - (xc[1] / xc[2] * f + cy);
    const double inf = pb.info[e];
    const double chi2 = inf * (err[0] * err[0] + err[1] * err[1]);
    d_huber(pb.huber, chi2, rho0, rho1);
}

// computeError + chi2 + robustify for one edge at state s; returns rho0, writes err, xc
__device__ __forceinline__ void edge_eval(const Problem& pb, const State& s, int e, double err[2],
                                          double xc[3], double& rho0, double& rho1)
{
    const int c = pb.ecam[e], p = pb.ept[e];
    const double q[4] = {s.q[4 * c], s.q[4 * c + 1], s.q[4 * c + 2], s.q[4 * c + 3]};
    const double X[3] = {s.p[3 * p], s.p[3 * p + 1], s.p[3 * p + 2]};
    const double t[3] = {s.t[3 * c], s.t[3 * c + 1], s.t[3 * c + 2]};
    edge_eval_at(pb, e, c, q, t, X, err, xc, rho0, rho1);
}

// EdgeProjectXYZ2UV::linearizeOplus pose block (2x6, row-major).  One reciprocal of z instead of
// g2o's per-entry divisions (the Jacobians feed H and b only, compared to tolerance; the
// reprojection errors keep the exact divisions).
__device__ __forceinline__ void jac_pose(const double xc[3], double f, double Jp[12])
{
    const double x = xc[0], y = xc[1], iz = 1.0 / xc[2];
    const double xi = x * iz, yi = y * iz, fi = f * iz;
    Jp[0] = xi * yi * f;
    Jp[1] = -(1 + xi * xi) * f;
    Jp[2] = yi * f;
    Jp[3] = -fi;
    Jp[4] = 0;
    Jp[5] = xi * fi;
    Jp[6] = (1 + yi * yi) * f;
    Jp[7] = -xi * yi * f;
    Jp[8] = -xi * f;
    Jp[9] = 0;
    Jp[10] = -fi;
    Jp[11] = yi * fi;
}

// The same pose Jacobian from (x/z, y/z, f/z) and f (jac_pose's expressions): the Schur sweeps
// keep these 3 numbers per edge instead of the 6x3 Hpl.
__device__ __forceinline__ void jac_pose_q(double xi, double yi, double fi, double f, double Jp[12])
{
    Jp[0] = xi * yi * f;
    Jp[1] = -(1 + xi * xi) * f;
    Jp[2] = yi * f;
    Jp[3] = -fi;
    Jp[4] = 0;
    Jp[5] = xi * fi;
    Jp[6] = (1 + yi * yi) * f;
    Jp[7] = -xi * yi * f;
    Jp[8] = -xi * f;
    Jp[9] = 0;
    Jp[10] = -fi;
    Jp[11] = yi * fi;
}

}  // namespace ba
}  // namespace mage
