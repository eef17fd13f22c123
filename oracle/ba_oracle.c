/*
 * ba_oracle.c — CPU restatement of BundlerLib + the g2o LM / Schur semantics it relies on
 * (TEST INFRASTRUCTURE ONLY: linked by tests/, smoke() and bench.py's cpu_baseline leg).
 *
 * PARITY UNPINNED: BundlerLib wraps g2o, whose submodule is empty in the reference tree
 * (SURVEY.md §8(c)); the reference ships no BA tests or fixtures.  This file follows
 *   Dependencies/BundlerLib/Source/BundlerLib.cpp:132-471 (StepOptimizer, BundlerLib)
 * and restates the published g2o algorithms it calls (RainerKuemmerle/g2o, 2017-2020 API:
 * SE3Quat / VertexSE3Expmap / VertexSBAPointXYZ / EdgeProjectXYZ2UV / RobustKernelHuber /
 * BlockSolver_6_3 Schur / LinearSolverDense / OptimizationAlgorithmLevenberg), as written out
 * in SURVEY.md Appendix A.4.  Validated by finite-difference and convergence tests
 * (tests/test_ba_oracle.py).  The dense solve uses Cholesky (LLT) where g2o uses Eigen LDLT:
 * the Schur complement of the damped system is positive definite, so both agree to rounding.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/mage_hot.h"

typedef struct {
    double q[4]; /* x, y, z, w (Eigen coefficient order) */
    double t[3];
} se3q;

typedef struct {
    se3q pose, backup;
    double f, cx, cy;
    int fixed;
    int hidx; /* column block in the reduced system, -1 if not in it */
} cam_t;

typedef struct {
    double p[3], backup[3];
    int hidx; /* -1 if not in the system */
} pt_t;

typedef struct {
    double uv[2];
    int cam, pt;
    double info;
    int removed;
    int active;
    double err[2];
    double hpl[18]; /* 6x3 row-major, J_pose^T W J_point */
} edge_t;

/* Camera-camera constraint edges (BundlerLib.cpp:22-88, 311-350): kind 0 = EdgeScaleConstraint
 * (fixed distance), 1 = EdgeRotationConstraint, 2 = g2o EdgeSE3Expmap (relative transform). */
typedef struct {
    int kind, c1, c2;
    double w;       /* SetWeight (kinds 0, 1) or the information scale (kind 2) */
    double dist;    /* kind 0 measurement */
    se3q meas;      /* kind 1: meas.q; kind 2: SE3Quat(q, t) */
    int active;
    int dim;        /* error dimension: 1 or 6 */
    double err[6];
    double J[2][36]; /* dim x 6 row-major, per vertex */
} tether_t;

typedef struct oracle_ba {
    int points_fixed;
    int nc, np, ne, nt;
    cam_t* cams;
    pt_t* pts;
    edge_t* edges;
    tether_t* teth; /* distance, rotation, transform tethers in insertion (addEdge) order */
    double huber;
    /* optimizer state (StepOptimizer, BundlerLib.cpp:92-166) */
    int dirty, useless, iteration;
    double user_lambda, lambda, ni;
    int nfree_c, nfree_p;
    /* system */
    double *Hpp, *bp, *Hll, *bl, *x, *S, *rhs, *Dinv;
    int *pstart, *pedges; /* active edges of each point, in edge (insertion) order */
    /* stats */
    uint64_t iters, trials, rejected;
    double last_chi2;
} oracle_ba;

/* ---------------- Eigen / g2o primitives ---------------- */

static void quat_normalize(double q[4])
{
    double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    for (int i = 0; i < 4; i++) q[i] /= n;
}

/* SE3Quat::normalizeRotation: w >= 0 then normalize. */
static void se3_normalize(se3q* s)
{
    if (s->q[3] < 0)
        for (int i = 0; i < 4; i++) s->q[i] = -s->q[i];
    quat_normalize(s->q);
}

/* Eigen quaternionbase_assign_impl<Matrix3>::run (Shoemake). m row-major. */
static void quat_from_matrix(const double m[9], double q[4])
{
#define M(r, c) m[(r)*3 + (c)]
    double t = M(0, 0) + M(1, 1) + M(2, 2);
    if (t > 0) {
        t = sqrt(t + 1.0);
        q[3] = 0.5 * t;
        t = 0.5 / t;
        q[0] = (M(2, 1) - M(1, 2)) * t;
        q[1] = (M(0, 2) - M(2, 0)) * t;
        q[2] = (M(1, 0) - M(0, 1)) * t;
    } else {
        int i = 0;
        if (M(1, 1) > M(0, 0)) i = 1;
        if (M(2, 2) > M(i, i)) i = 2;
        int j = (i + 1) % 3, k = (j + 1) % 3;
        t = sqrt(M(i, i) - M(j, j) - M(k, k) + 1.0);
        q[i] = 0.5 * t;
        t = 0.5 / t;
        q[3] = (M(k, j) - M(j, k)) * t;
        q[j] = (M(j, i) + M(i, j)) * t;
        q[k] = (M(k, i) + M(i, k)) * t;
    }
#undef M
}

/* float version used by SetCameraPose: Eigen::Quaternionf{Matrix3f}.normalized() */
static void quatf_from_matrix(const float m[9], float q[4])
{
#define M(r, c) m[(r)*3 + (c)]
    float t = M(0, 0) + M(1, 1) + M(2, 2);
    if (t > 0.f) {
        t = sqrtf(t + 1.0f);
        q[3] = 0.5f * t;
        t = 0.5f / t;
        q[0] = (M(2, 1) - M(1, 2)) * t;
        q[1] = (M(0, 2) - M(2, 0)) * t;
        q[2] = (M(1, 0) - M(0, 1)) * t;
    } else {
        int i = 0;
        if (M(1, 1) > M(0, 0)) i = 1;
        if (M(2, 2) > M(i, i)) i = 2;
        int j = (i + 1) % 3, k = (j + 1) % 3;
        t = sqrtf(M(i, i) - M(j, j) - M(k, k) + 1.0f);
        q[i] = 0.5f * t;
        t = 0.5f / t;
        q[3] = (M(k, j) - M(j, k)) * t;
        q[j] = (M(j, i) + M(i, j)) * t;
        q[k] = (M(k, i) + M(i, k)) * t;
    }
#undef M
    float n = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    for (int a = 0; a < 4; a++) q[a] /= n;
}

/* QuaternionBase::toRotationMatrix, row-major output. */
static void quat_to_matrix(const double q[4], double r[9])
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

static void cross3(const double a[3], const double b[3], double c[3])
{
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}

/* Quaternion * Vector3 (Eigen _transformVector). */
static void quat_rotate(const double q[4], const double v[3], double out[3])
{
    double uv[3], uv2[3];
    cross3(q, v, uv);
    for (int i = 0; i < 3; i++) uv[i] += uv[i];
    cross3(q, uv, uv2);
    for (int i = 0; i < 3; i++) out[i] = v[i] + q[3] * uv[i] + uv2[i];
}

static void quat_mul(const double a[4], const double b[4], double o[4])
{
    double w = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
    double x = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
    double y = a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2];
    double z = a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0];
    o[0] = x;
    o[1] = y;
    o[2] = z;
    o[3] = w;
}

/* SE3Quat::map */
static void se3_map(const se3q* s, const double p[3], double out[3])
{
    quat_rotate(s->q, p, out);
    for (int i = 0; i < 3; i++) out[i] += s->t[i];
}

/* SE3Quat::exp(update), update = (omega, upsilon) */
static void se3_exp(const double u[6], se3q* out)
{
    double w[3] = {u[0], u[1], u[2]};
    double theta = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    double O[9] = {0, -w[2], w[1], w[2], 0, -w[0], -w[1], w[0], 0};
    double O2[9];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) {
            double s = 0;
            for (int k = 0; k < 3; k++) s += O[r * 3 + k] * O[k * 3 + c];
            O2[r * 3 + c] = s;
        }
    double R[9], V[9];
    if (theta < 0.00001) {
        for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0 ? 1.0 : 0.0) + O[i] + O2[i];
        memcpy(V, R, sizeof(R));
    } else {
        double a = sin(theta) / theta, b = (1 - cos(theta)) / (theta * theta);
        double c = (theta - sin(theta)) / pow(theta, 3);
        for (int i = 0; i < 9; i++) {
            double I = (i % 4 == 0 ? 1.0 : 0.0);
            R[i] = I + a * O[i] + b * O2[i];
            V[i] = I + b * O[i] + c * O2[i];
        }
    }
    quat_from_matrix(R, out->q);
    for (int r = 0; r < 3; r++) out->t[r] = V[r * 3 + 0] * u[3] + V[r * 3 + 1] * u[4] + V[r * 3 + 2] * u[5];
    se3_normalize(out);
}

/* VertexSE3Expmap::oplusImpl: estimate = exp(update) * estimate */
static void se3_oplus(se3q* s, const double u[6])
{
    se3q e, res;
    se3_exp(u, &e);
    double rt[3];
    quat_rotate(e.q, s->t, rt);
    for (int i = 0; i < 3; i++) res.t[i] = e.t[i] + rt[i];
    quat_mul(e.q, s->q, res.q);
    se3_normalize(&res);
    *s = res;
}

/* EdgeProjectXYZ2UV::computeError: e = obs - cam_map(T.map(p)) */
static void edge_error(const oracle_ba* b, const edge_t* e, double err[2], double xc[3])
{
    const cam_t* c = &b->cams[e->cam];
    se3_map(&c->pose, b->pts[e->pt].p, xc);
    double u = xc[0] / xc[2] * c->f + c->cx;
    double v = xc[1] / xc[2] * c->f + c->cy;
    err[0] = e->uv[0] - u;
    err[1] = e->uv[1] - v;
}

/* RobustKernelHuber::robustify */
static void huber(double delta, double e2, double rho[3])
{
    double dsqr = delta * delta;
    if (e2 <= dsqr) {
        rho[0] = e2;
        rho[1] = 1.;
        rho[2] = 0.;
    } else {
        double sq = sqrt(e2);
        rho[0] = 2 * sq * delta - dsqr;
        rho[1] = delta / sq;
        rho[2] = -0.5 * rho[1] / e2;
    }
}

/* ---------------- tether edges (BundlerLib.cpp:22-88; g2o EdgeSE3Expmap) ---------------- */

/* SE3Quat::inverse: r' = conj(r), t' = r' * (-t) */
static void se3_inverse(const se3q* s, se3q* o)
{
    o->q[0] = -s->q[0];
    o->q[1] = -s->q[1];
    o->q[2] = -s->q[2];
    o->q[3] = s->q[3];
    double mt[3] = {-s->t[0], -s->t[1], -s->t[2]};
    quat_rotate(o->q, mt, o->t);
}

/* SE3Quat::operator*: t = a.t + a.r * b.t, r = a.r * b.r, normalizeRotation */
static void se3_mul(const se3q* a, const se3q* b, se3q* o)
{
    se3q r;
    double rt[3];
    quat_rotate(a->q, b->t, rt);
    for (int i = 0; i < 3; i++) r.t[i] = a->t[i] + rt[i];
    quat_mul(a->q, b->q, r.q);
    se3_normalize(&r);
    *o = r;
}

static void skew3(const double v[3], double m[9])
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

static void mat3_mul(const double a[9], const double b[9], double o[9])
{
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) o[r * 3 + c] = a[r * 3] * b[c] + a[r * 3 + 1] * b[3 + c] + a[r * 3 + 2] * b[6 + c];
}

/* SE3Quat::log (g2o se3quat.h): (omega, upsilon) */
static void se3_log(const se3q* s, double res[6])
{
    double R[9];
    quat_to_matrix(s->q, R);
    double d = 0.5 * (R[0] + R[4] + R[8] - 1);
    double dR[3] = {R[7] - R[5], R[2] - R[6], R[3] - R[1]};
    double omega[3], Om[9], Om2[9], Vinv[9];
    if (fabs(d) > 0.99999) {
        for (int i = 0; i < 3; i++) omega[i] = 0.5 * dR[i];
        skew3(omega, Om);
        mat3_mul(Om, Om, Om2);
        for (int i = 0; i < 9; i++) Vinv[i] = (i % 4 == 0 ? 1.0 : 0.0) - 0.5 * Om[i] + (1. / 12.) * Om2[i];
    } else {
        double theta = acos(d);
        for (int i = 0; i < 3; i++) omega[i] = theta / (2 * sqrt(1 - d * d)) * dR[i];
        skew3(omega, Om);
        mat3_mul(Om, Om, Om2);
        double k = (1 - theta / (2 * tan(theta / 2))) / (theta * theta);
        for (int i = 0; i < 9; i++) Vinv[i] = (i % 4 == 0 ? 1.0 : 0.0) - 0.5 * Om[i] + k * Om2[i];
    }
    for (int i = 0; i < 3; i++) {
        res[i] = omega[i];
        res[3 + i] = Vinv[i * 3] * s->t[0] + Vinv[i * 3 + 1] * s->t[1] + Vinv[i * 3 + 2] * s->t[2];
    }
}

/* SE3Quat::adj: [R 0; skew(t) R, R], 6x6 row-major */
static void se3_adj(const se3q* s, double A[36])
{
    double R[9], St[9], SR[9];
    quat_to_matrix(s->q, R);
    skew3(s->t, St);
    mat3_mul(St, R, SR);
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) {
            A[r * 6 + c] = R[r * 3 + c];
            A[r * 6 + 3 + c] = 0;
            A[(3 + r) * 6 + c] = SR[r * 3 + c];
            A[(3 + r) * 6 + 3 + c] = R[r * 3 + c];
        }
}

/* computeError of one tether at the current camera estimates */
static void tether_error(const oracle_ba* b, const tether_t* t, double e[6])
{
    const se3q* T1 = &b->cams[t->c1].pose;
    const se3q* T2 = &b->cams[t->c2].pose;
    if (t->kind == 0) {
        /* EdgeScaleConstraint: (measurement - |t2 - t1|) * weight, t = SE3Quat translation */
        double dt[3] = {T2->t[0] - T1->t[0], T2->t[1] - T1->t[1], T2->t[2] - T1->t[2]};
        e[0] = (t->dist - sqrt(dt[0] * dt[0] + dt[1] * dt[1] + dt[2] * dt[2])) * t->w;
    } else if (t->kind == 1) {
        /* EdgeRotationConstraint: (T1^-1 T2).rotation().angularDistance(measurement) * weight;
         * Eigen 3.3 angularDistance: d = this * other.conjugate(), 2 atan2(|d.vec|, |d.w|) */
        se3q i1, rel;
        se3_inverse(T1, &i1);
        se3_mul(&i1, T2, &rel);
        double mc[4] = {-t->meas.q[0], -t->meas.q[1], -t->meas.q[2], t->meas.q[3]};
        double d[4];
        quat_mul(rel.q, mc, d);
        double vn = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
        e[0] = 2.0 * atan2(vn, fabs(d[3])) * t->w;
    } else {
        /* EdgeSE3Expmap::computeError: (T2^-1 * C * T1).log() */
        se3q i2, a, r;
        se3_inverse(T2, &i2);
        se3_mul(&i2, &t->meas, &a);
        se3_mul(&a, T1, &r);
        se3_log(&r, e);
    }
}

/* linearizeOplus: BaseMultiEdge numeric differences (delta 1e-9, central) for kinds 0 / 1,
 * EdgeSE3Expmap's analytic adjoints for kind 2.  Only vertices in the system get a Jacobian. */
static void tether_jacobians(oracle_ba* b, tether_t* t)
{
    const int cams[2] = {t->c1, t->c2};
    if (t->kind == 2) {
        const se3q* Ti = &b->cams[t->c1].pose;
        const se3q* Tj = &b->cams[t->c2].pose;
        se3q invTij, invTj, invTi, invTj_Tij, invTi_invTij;
        se3_inverse(&t->meas, &invTij);
        se3_inverse(Tj, &invTj);
        se3_inverse(Ti, &invTi);
        se3_mul(&invTj, &t->meas, &invTj_Tij);
        se3_mul(&invTi, &invTij, &invTi_invTij);
        se3_adj(&invTj_Tij, t->J[0]);
        se3_adj(&invTi_invTij, t->J[1]);
        for (int k = 0; k < 36; k++) t->J[1][k] = -t->J[1][k];
        return;
    }
    const double delta = 1e-9, scalar = 1 / (2 * delta);
    for (int v = 0; v < 2; v++) {
        cam_t* c = &b->cams[cams[v]];
        if (c->hidx < 0) continue;
        for (int dd = 0; dd < 6; dd++) {
            double add[6] = {0, 0, 0, 0, 0, 0}, ep[6], em[6];
            se3q keep = c->pose;
            add[dd] = delta;
            se3_oplus(&c->pose, add);
            tether_error(b, t, ep);
            c->pose = keep;
            add[dd] = -delta;
            se3_oplus(&c->pose, add);
            tether_error(b, t, em);
            c->pose = keep;
            for (int r = 0; r < t->dim; r++) t->J[v][r * 6 + dd] = scalar * (ep[r] - em[r]);
        }
    }
}

/* information scale: Identity (kinds 0, 1; the weight is inside the error), weight * I6 (kind 2) */
static double tether_omega(const tether_t* t) { return t->kind == 2 ? t->w : 1.0; }

static double tether_chi2(const tether_t* t)
{
    double s = 0;
    for (int r = 0; r < t->dim; r++) s += t->err[r] * t->err[r];
    return tether_omega(t) * s;
}

/* H12 (6x6 row-major) = J1^T Omega J2 of an active tether with both cameras in the system */
static void tether_h12(const tether_t* t, double H[36])
{
    const double om = tether_omega(t);
    for (int r = 0; r < 6; r++)
        for (int c = 0; c < 6; c++) {
            double s = 0;
            for (int m = 0; m < t->dim; m++) s += t->J[0][m * 6 + r] * t->J[1][m * 6 + c];
            H[r * 6 + c] = s * om;
        }
}

void oracle_ba_set_tethers(oracle_ba* b, int kind, int n, const uint32_t* cam1, const uint32_t* cam2,
                           const float* params, const float* weight)
{
    /* keep the other kinds, replace this one; order distance, rotation, transform */
    int keep = 0;
    tether_t* nt = (tether_t*)calloc((size_t)(b->nt + n) + 1, sizeof(tether_t));
    for (int k = 0; k <= 2; k++) {
        if (k == kind) {
            const int stride = kind == 0 ? 1 : kind == 1 ? 4 : 7;
            for (int i = 0; i < n; i++) {
                tether_t* t = &nt[keep++];
                const float* pr = params + (size_t)stride * i;
                t->kind = kind;
                t->c1 = (int)cam1[i];
                t->c2 = (int)cam2[i];
                t->w = (double)weight[i];
                t->dim = kind == 2 ? 6 : 1;
                if (kind == 0) {
                    t->dist = (double)pr[0];
                } else if (kind == 1) {
                    /* setMeasurement(Quaternionf.cast<double>()), not normalised */
                    for (int a = 0; a < 4; a++) t->meas.q[a] = (double)pr[a];
                } else {
                    /* SE3Quat(q.cast<double>(), t.cast<double>()) normalises the rotation */
                    for (int a = 0; a < 3; a++) t->meas.t[a] = (double)pr[a];
                    for (int a = 0; a < 4; a++) t->meas.q[a] = (double)pr[3 + a];
                    se3_normalize(&t->meas);
                }
            }
        } else {
            for (int i = 0; i < b->nt; i++)
                if (b->teth[i].kind == k) nt[keep++] = b->teth[i];
        }
    }
    free(b->teth);
    b->teth = nt;
    b->nt = keep;
    b->dirty = 1;
}

/* ---------------- optimizer ---------------- */

oracle_ba* oracle_ba_create(int points_fixed)
{
    oracle_ba* b = (oracle_ba*)calloc(1, sizeof(oracle_ba));
    b->points_fixed = points_fixed;
    b->dirty = 1;
    b->user_lambda = 0;
    b->lambda = 0;
    b->ni = 2;
    return b;
}

static void free_system(oracle_ba* b)
{
    free(b->Hpp);
    free(b->bp);
    free(b->Hll);
    free(b->bl);
    free(b->x);
    free(b->S);
    free(b->rhs);
    free(b->Dinv);
    free(b->pstart);
    free(b->pedges);
    b->Hpp = b->bp = b->Hll = b->bl = b->x = b->S = b->rhs = b->Dinv = NULL;
    b->pstart = b->pedges = NULL;
}

void oracle_ba_destroy(oracle_ba* b)
{
    if (!b) return;
    free_system(b);
    free(b->cams);
    free(b->pts);
    free(b->edges);
    free(b->teth);
    free(b);
}

void oracle_ba_set_cameras(oracle_ba* b, int n, const float* pos3, const float* r9,
                           const float* intr4, const uint8_t* fixed)
{
    free(b->cams);
    b->nc = n;
    b->cams = (cam_t*)calloc((size_t)n, sizeof(cam_t));
    for (int i = 0; i < n; i++) {
        /* Eigen::Map<const Matrix3f> is column-major: m(r,c) = r9[c*3+r] */
        float m[9], qf[4];
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) m[r * 3 + c] = r9[9 * i + c * 3 + r];
        quatf_from_matrix(m, qf);
        cam_t* c = &b->cams[i];
        for (int k = 0; k < 4; k++) c->pose.q[k] = (double)qf[k];
        for (int k = 0; k < 3; k++) c->pose.t[k] = (double)pos3[3 * i + k];
        se3_normalize(&c->pose); /* SE3Quat(q, t) ctor normalizes */
        /* CameraParameters(intrinsics[2], Vector2(intrinsics[0], intrinsics[1]), 0) :266 */
        c->f = (double)intr4[4 * i + 2];
        c->cx = (double)intr4[4 * i + 0];
        c->cy = (double)intr4[4 * i + 1];
        c->fixed = fixed ? fixed[i] != 0 : 0;
    }
    b->dirty = 1;
}

void oracle_ba_fix_camera(oracle_ba* b, int idx, int fixed)
{
    b->cams[idx].fixed = fixed != 0;
    /* setFixed does not dirty the StepOptimizer (BundlerLib.cpp:280-283) */
}

void oracle_ba_set_points(oracle_ba* b, int n, const float* xyz)
{
    free(b->pts);
    b->np = n;
    b->pts = (pt_t*)calloc((size_t)n, sizeof(pt_t));
    for (int i = 0; i < n; i++)
        for (int k = 0; k < 3; k++) b->pts[i].p[k] = (double)xyz[3 * i + k];
    b->dirty = 1;
}

void oracle_ba_set_observations(oracle_ba* b, int n, const float* uv, const uint32_t* cam,
                                const uint32_t* pt, const float* info)
{
    free(b->edges);
    b->ne = n;
    b->edges = (edge_t*)calloc((size_t)n, sizeof(edge_t));
    for (int i = 0; i < n; i++) {
        edge_t* e = &b->edges[i];
        e->uv[0] = (double)uv[2 * i];
        e->uv[1] = (double)uv[2 * i + 1];
        e->cam = (int)cam[i];
        e->pt = (int)pt[i];
        e->info = (double)info[i];
    }
    b->dirty = 1;
}

void oracle_ba_set_lambda(oracle_ba* b, float lambda)
{
    b->iteration = 0; /* StepOptimizer::SetCurrentLambda :123-130 */
    b->user_lambda = (double)lambda;
}

float oracle_ba_get_lambda(const oracle_ba* b) { return (float)b->lambda; }

/* SparseOptimizer::initializeOptimization + buildIndexMapping (BundlerLib.cpp:156-166):
 * an edge is active unless removed or all its vertices are fixed; a vertex is in the system
 * if it is not fixed and has an active edge.  Poses are indexed in id order. */
static void initialize(oracle_ba* b)
{
    int* camHas = (int*)calloc((size_t)b->nc, sizeof(int));
    int* ptHas = (int*)calloc((size_t)b->np, sizeof(int));
    for (int i = 0; i < b->ne; i++) {
        edge_t* e = &b->edges[i];
        int camFixed = b->cams[e->cam].fixed, ptFixed = b->points_fixed;
        e->active = !e->removed && !(camFixed && ptFixed);
        if (e->active) {
            camHas[e->cam] = 1;
            ptHas[e->pt] = 1;
        }
    }
    /* a tether is active unless both cameras are fixed (edges with all vertices fixed are not
     * active); its cameras then belong to the system even without observations */
    for (int i = 0; i < b->nt; i++) {
        tether_t* t = &b->teth[i];
        t->active = !(b->cams[t->c1].fixed && b->cams[t->c2].fixed);
        if (t->active) {
            camHas[t->c1] = 1;
            camHas[t->c2] = 1;
        }
    }
    b->nfree_c = 0;
    for (int c = 0; c < b->nc; c++)
        b->cams[c].hidx = (!b->cams[c].fixed && camHas[c]) ? b->nfree_c++ : -1;
    b->nfree_p = 0;
    /* points: ids decrease with index (BundlerLib.cpp:209-217) so the Hessian order is
     * descending point index */
    for (int p = b->np - 1; p >= 0; p--)
        b->pts[p].hidx = (!b->points_fixed && ptHas[p]) ? b->nfree_p++ : -1;
    free(camHas);
    free(ptHas);
    b->useless = (b->nfree_c + b->nfree_p) == 0;
    free_system(b);
    int n = 6 * b->nfree_c;
    b->Hpp = (double*)calloc((size_t)b->nc * 36 + 1, sizeof(double));
    b->bp = (double*)calloc((size_t)b->nc * 6 + 1, sizeof(double));
    b->Hll = (double*)calloc((size_t)b->np * 9 + 1, sizeof(double));
    b->bl = (double*)calloc((size_t)b->np * 3 + 1, sizeof(double));
    b->Dinv = (double*)calloc((size_t)b->np * 9 + 1, sizeof(double));
    b->x = (double*)calloc((size_t)n + 3 * (size_t)b->np + 1, sizeof(double));
    b->S = (double*)calloc((size_t)n * n + 1, sizeof(double));
    b->rhs = (double*)calloc((size_t)n + 1, sizeof(double));
    b->pstart = (int*)calloc((size_t)b->np + 1, sizeof(int));
    b->pedges = (int*)calloc((size_t)b->ne + 1, sizeof(int));
    for (int i = 0; i < b->ne; i++)
        if (b->edges[i].active) b->pstart[b->edges[i].pt + 1]++;
    for (int p = 0; p < b->np; p++) b->pstart[p + 1] += b->pstart[p];
    {
        int* fill = (int*)malloc(sizeof(int) * ((size_t)b->np + 1));
        memcpy(fill, b->pstart, sizeof(int) * ((size_t)b->np + 1));
        for (int i = 0; i < b->ne; i++)
            if (b->edges[i].active) b->pedges[fill[b->edges[i].pt]++] = i;
        free(fill);
    }
    b->iteration = 0;
    b->dirty = 0;
}

/* computeActiveErrors + activeRobustChi2 */
static double compute_errors(oracle_ba* b)
{
    double chi = 0;
    for (int i = 0; i < b->ne; i++) {
        edge_t* e = &b->edges[i];
        if (!e->active) continue;
        double xc[3], rho[3];
        edge_error(b, e, e->err, xc);
        double chi2 = e->info * (e->err[0] * e->err[0] + e->err[1] * e->err[1]);
        huber(b->huber, chi2, rho);
        chi += rho[0];
    }
    /* tethers follow the observations in addEdge (internal id) order; no robust kernel */
    for (int i = 0; i < b->nt; i++) {
        tether_t* t = &b->teth[i];
        if (!t->active) continue;
        tether_error(b, t, t->err);
        chi += tether_chi2(t);
    }
    return chi;
}

/* EdgeProjectXYZ2UV::linearizeOplus: Jpt (2x3) and Jpose (2x6), row-major. */
static void edge_jacobians(const oracle_ba* b, const edge_t* e, double Jpt[6], double Jp[12])
{
    const cam_t* c = &b->cams[e->cam];
    double xc[3];
    se3_map(&c->pose, b->pts[e->pt].p, xc);
    double x = xc[0], y = xc[1], z = xc[2], z2 = z * z, f = c->f;
    double R[9];
    quat_to_matrix(c->pose.q, R);
    double tmp[6] = {f, 0, -x / z * f, 0, f, -y / z * f};
    for (int r = 0; r < 2; r++)
        for (int k = 0; k < 3; k++) {
            double s = 0;
            for (int m = 0; m < 3; m++) s += tmp[r * 3 + m] * R[m * 3 + k];
            Jpt[r * 3 + k] = -1. / z * s;
        }
    Jp[0] = x * y / z2 * f;
    Jp[1] = -(1 + (x * x / z2)) * f;
    Jp[2] = y / z * f;
    Jp[3] = -1. / z * f;
    Jp[4] = 0;
    Jp[5] = x / z2 * f;
    Jp[6] = (1 + y * y / z2) * f;
    Jp[7] = -x * y / z2 * f;
    Jp[8] = -x / z * f;
    Jp[9] = 0;
    Jp[10] = -1. / z * f;
    Jp[11] = y / z2 * f;
}

/* BlockSolver::buildSystem with BaseBinaryEdge::constructQuadraticForm (robust, first order). */
static void build_system(oracle_ba* b)
{
    memset(b->Hpp, 0, sizeof(double) * b->nc * 36);
    memset(b->bp, 0, sizeof(double) * b->nc * 6);
    memset(b->Hll, 0, sizeof(double) * b->np * 9);
    memset(b->bl, 0, sizeof(double) * b->np * 3);
    for (int i = 0; i < b->ne; i++) {
        edge_t* e = &b->edges[i];
        if (!e->active) continue;
        int ptFree = b->pts[e->pt].hidx >= 0, camFree = b->cams[e->cam].hidx >= 0;
        if (!ptFree && !camFree) continue;
        double Jpt[6], Jp[12], rho[3];
        edge_jacobians(b, e, Jpt, Jp);
        double chi2 = e->info * (e->err[0] * e->err[0] + e->err[1] * e->err[1]);
        huber(b->huber, chi2, rho);
        double w = rho[1] * e->info;            /* weightedOmega = rho' * info * I */
        double or0 = -e->info * e->err[0] * rho[1]; /* omega_r = -Omega e, *= rho' */
        double or1 = -e->info * e->err[1] * rho[1];
        if (ptFree) {
            double* H = &b->Hll[9 * e->pt];
            double* g = &b->bl[3 * e->pt];
            for (int r = 0; r < 3; r++) {
                g[r] += Jpt[r] * or0 + Jpt[3 + r] * or1;
                for (int c = 0; c < 3; c++) H[r * 3 + c] += (Jpt[r] * Jpt[c] + Jpt[3 + r] * Jpt[3 + c]) * w;
            }
            if (camFree)
                for (int r = 0; r < 6; r++)
                    for (int c = 0; c < 3; c++)
                        e->hpl[r * 3 + c] = (Jp[r] * Jpt[c] + Jp[6 + r] * Jpt[3 + c]) * w;
        }
        if (camFree) {
            double* H = &b->Hpp[36 * e->cam];
            double* g = &b->bp[6 * e->cam];
            for (int r = 0; r < 6; r++) {
                g[r] += Jp[r] * or0 + Jp[6 + r] * or1;
                for (int c = 0; c < 6; c++) H[r * 6 + c] += (Jp[r] * Jp[c] + Jp[6 + r] * Jp[6 + c]) * w;
            }
        }
    }
    /* tethers: BaseMultiEdge / BaseBinaryEdge::constructQuadraticForm without a robust kernel:
     * H_vv += J_v^T Omega J_v, b_v += J_v^T (-Omega e); the H_12 block enters S in solve_system */
    for (int i = 0; i < b->nt; i++) {
        tether_t* t = &b->teth[i];
        if (!t->active) continue;
        tether_jacobians(b, t);
        const double om = tether_omega(t);
        const int cams[2] = {t->c1, t->c2};
        for (int v = 0; v < 2; v++) {
            if (b->cams[cams[v]].hidx < 0) continue;
            double* H = &b->Hpp[36 * cams[v]];
            double* g = &b->bp[6 * cams[v]];
            const double* J = t->J[v];
            for (int r = 0; r < 6; r++) {
                double s = 0;
                for (int m = 0; m < t->dim; m++) s += J[m * 6 + r] * (-om * t->err[m]);
                g[r] += s;
                for (int c = 0; c < 6; c++) {
                    double h = 0;
                    for (int m = 0; m < t->dim; m++) h += J[m * 6 + r] * J[m * 6 + c];
                    H[r * 6 + c] += h * om;
                }
            }
        }
    }
}

/* computeLambdaInit: tau * max |H_ii| over vertices in the system (tau = 1e-5). */
static double lambda_init(const oracle_ba* b)
{
    if (b->user_lambda > 0) return b->user_lambda;
    double m = 0;
    for (int c = 0; c < b->nc; c++)
        if (b->cams[c].hidx >= 0)
            for (int j = 0; j < 6; j++) m = fmax(fabs(b->Hpp[36 * c + j * 7]), m);
    for (int p = 0; p < b->np; p++)
        if (b->pts[p].hidx >= 0)
            for (int j = 0; j < 3; j++) m = fmax(fabs(b->Hll[9 * p + j * 4]), m);
    return 1e-5 * m;
}

/* Eigen Matrix3d::inverse (cofactors / determinant). */
static void inv3(const double m[9], double o[9])
{
    double c0 = m[4] * m[8] - m[5] * m[7];
    double c1 = m[5] * m[6] - m[3] * m[8];
    double c2 = m[3] * m[7] - m[4] * m[6];
    double det = m[0] * c0 + m[1] * c1 + m[2] * c2;
    double id = 1.0 / det;
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

/* BlockSolver::setLambda + solve (Schur) + LinearSolverDense; x = [xp (6 per free cam), xl
 * (3 per point, by point index)].  Returns 0 if the reduced system is not positive definite. */
static int solve_system(oracle_ba* b, double lambda)
{
    int nf = b->nfree_c, n = 6 * nf;
    double* S = b->S;
    memset(S, 0, sizeof(double) * n * n);
    for (int c = 0; c < b->nc; c++) {
        int h = b->cams[c].hidx;
        if (h < 0) continue;
        for (int r = 0; r < 6; r++) {
            for (int k = 0; k < 6; k++) S[(6 * h + r) * n + 6 * h + k] = b->Hpp[36 * c + r * 6 + k];
            S[(6 * h + r) * n + 6 * h + r] += lambda;
            b->rhs[6 * h + r] = b->bp[6 * c + r];
        }
    }
    for (int i = 0; i < b->nt; i++) {
        const tether_t* t = &b->teth[i];
        const int h1 = b->cams[t->c1].hidx, h2 = b->cams[t->c2].hidx;
        if (!t->active || h1 < 0 || h2 < 0) continue;
        double H[36];
        tether_h12(t, H);
        for (int r = 0; r < 6; r++)
            for (int c = 0; c < 6; c++) {
                S[(6 * h1 + r) * n + 6 * h2 + c] += H[r * 6 + c];
                S[(6 * h2 + c) * n + 6 * h1 + r] += H[r * 6 + c];
            }
    }
    /* landmarks in Hessian order (descending index); Hpl columns per landmark by pose row */
    for (int p = b->np - 1; p >= 0; p--) {
        if (b->pts[p].hidx < 0) continue;
        double D[9];
        memcpy(D, &b->Hll[9 * p], sizeof(D));
        for (int j = 0; j < 3; j++) D[j * 4] += lambda;
        double* Di = &b->Dinv[9 * p];
        inv3(D, Di);
        double db[3];
        for (int r = 0; r < 3; r++) db[r] = Di[r * 3] * b->bl[3 * p] + Di[r * 3 + 1] * b->bl[3 * p + 1] + Di[r * 3 + 2] * b->bl[3 * p + 2];
        for (int a = b->pstart[p]; a < b->pstart[p + 1]; a++) {
            edge_t* e1 = &b->edges[b->pedges[a]];
            if (b->cams[e1->cam].hidx < 0) continue;
            int h1 = b->cams[e1->cam].hidx;
            double BDinv[18];
            for (int r = 0; r < 6; r++)
                for (int c = 0; c < 3; c++)
                    BDinv[r * 3 + c] = e1->hpl[r * 3] * Di[c] + e1->hpl[r * 3 + 1] * Di[3 + c] + e1->hpl[r * 3 + 2] * Di[6 + c];
            for (int r = 0; r < 6; r++)
                b->rhs[6 * h1 + r] -= e1->hpl[r * 3] * db[0] + e1->hpl[r * 3 + 1] * db[1] + e1->hpl[r * 3 + 2] * db[2];
            for (int bb = b->pstart[p]; bb < b->pstart[p + 1]; bb++) {
                edge_t* e2 = &b->edges[b->pedges[bb]];
                if (b->cams[e2->cam].hidx < h1) continue;
                int h2 = b->cams[e2->cam].hidx;
                for (int r = 0; r < 6; r++)
                    for (int c = 0; c < 6; c++) {
                        double s = BDinv[r * 3] * e2->hpl[c * 3] + BDinv[r * 3 + 1] * e2->hpl[c * 3 + 1] + BDinv[r * 3 + 2] * e2->hpl[c * 3 + 2];
                        S[(6 * h1 + r) * n + 6 * h2 + c] -= s;
                        if (h1 != h2) S[(6 * h2 + c) * n + 6 * h1 + r] -= s;
                    }
            }
        }
    }
    /* dense Cholesky S = L L^T (lower, in place) */
    for (int j = 0; j < n; j++) {
        double d = S[j * n + j];
        for (int k = 0; k < j; k++) d -= S[j * n + k] * S[j * n + k];
        if (!(d > 0)) return 0;
        d = sqrt(d);
        S[j * n + j] = d;
        for (int i = j + 1; i < n; i++) {
            double s = S[i * n + j];
            for (int k = 0; k < j; k++) s -= S[i * n + k] * S[j * n + k];
            S[i * n + j] = s / d;
        }
    }
    double* xp = b->x;
    for (int i = 0; i < n; i++) {
        double s = b->rhs[i];
        for (int k = 0; k < i; k++) s -= S[i * n + k] * xp[k];
        xp[i] = s / S[i * n + i];
    }
    for (int i = n - 1; i >= 0; i--) {
        double s = xp[i];
        for (int k = i + 1; k < n; k++) s -= S[k * n + i] * xp[k];
        xp[i] = s / S[i * n + i];
    }
    /* landmarks: xl = Dinv (bl - Hpl^T xp) */
    double* xl = b->x + n;
    for (int p = 0; p < b->np; p++) {
        if (b->pts[p].hidx < 0) continue;
        double cl[3] = {b->bl[3 * p], b->bl[3 * p + 1], b->bl[3 * p + 2]};
        for (int a = b->pstart[p]; a < b->pstart[p + 1]; a++) {
            edge_t* e = &b->edges[b->pedges[a]];
            if (b->cams[e->cam].hidx < 0) continue;
            int h = b->cams[e->cam].hidx;
            for (int c = 0; c < 3; c++)
                for (int r = 0; r < 6; r++) cl[c] -= e->hpl[r * 3 + c] * xp[6 * h + r];
        }
        const double* Di = &b->Dinv[9 * p];
        for (int r = 0; r < 3; r++) xl[3 * p + r] = Di[r * 3] * cl[0] + Di[r * 3 + 1] * cl[1] + Di[r * 3 + 2] * cl[2];
    }
    return 1;
}

static void push_state(oracle_ba* b)
{
    for (int c = 0; c < b->nc; c++) b->cams[c].backup = b->cams[c].pose;
    for (int p = 0; p < b->np; p++) memcpy(b->pts[p].backup, b->pts[p].p, sizeof(double) * 3);
}

static void pop_state(oracle_ba* b)
{
    for (int c = 0; c < b->nc; c++) b->cams[c].pose = b->cams[c].backup;
    for (int p = 0; p < b->np; p++) memcpy(b->pts[p].p, b->pts[p].backup, sizeof(double) * 3);
}

static void apply_update(oracle_ba* b)
{
    int n = 6 * b->nfree_c;
    for (int c = 0; c < b->nc; c++)
        if (b->cams[c].hidx >= 0) se3_oplus(&b->cams[c].pose, &b->x[6 * b->cams[c].hidx]);
    for (int p = 0; p < b->np; p++)
        if (b->pts[p].hidx >= 0)
            for (int k = 0; k < 3; k++) b->pts[p].p[k] += b->x[n + 3 * p + k];
}

/* computeScale: sum_j x_j (lambda x_j + b_j) */
static double compute_scale(const oracle_ba* b, double lambda)
{
    int n = 6 * b->nfree_c;
    double s = 0;
    for (int c = 0; c < b->nc; c++) {
        int h = b->cams[c].hidx;
        if (h < 0) continue;
        for (int r = 0; r < 6; r++) s += b->x[6 * h + r] * (lambda * b->x[6 * h + r] + b->bp[6 * c + r]);
    }
    for (int p = b->np - 1; p >= 0; p--) {
        if (b->pts[p].hidx < 0) continue;
        for (int r = 0; r < 3; r++) s += b->x[n + 3 * p + r] * (lambda * b->x[n + 3 * p + r] + b->bl[3 * p + r]);
    }
    return s;
}

/* OptimizationAlgorithmLevenberg::solve(iteration).  Returns 1 = OK, 0 = Terminate. */
static int lm_solve(oracle_ba* b)
{
    double currentChi = compute_errors(b);
    double tempChi = currentChi;
    build_system(b);
    if (b->iteration == 0) {
        b->lambda = lambda_init(b);
        b->ni = 2;
    }
    double rho = 0;
    int qmax = 0;
    do {
        push_state(b);
        int ok2 = solve_system(b, b->lambda);
        apply_update(b);
        tempChi = compute_errors(b);
        if (!ok2) tempChi = 1.7976931348623157e308;
        rho = currentChi - tempChi;
        double scale = compute_scale(b, b->lambda);
        scale += 1e-3;
        rho /= scale;
        b->trials++;
        if (rho > 0 && isfinite(tempChi)) {
            double alpha = 1. - pow((2 * rho - 1), 3);
            alpha = fmin(alpha, 2. / 3.);
            double scaleFactor = fmax(1. / 3., alpha);
            b->lambda *= scaleFactor;
            b->ni = 2;
            currentChi = tempChi;
        } else {
            b->lambda *= b->ni;
            b->ni *= 2;
            pop_state(b);
            b->rejected++;
        }
        qmax++;
    } while (rho < 0 && qmax < 10);
    b->last_chi2 = currentChi;
    b->iters++;
    if (qmax == 10 || rho == 0 || !isfinite(b->lambda)) return 0;
    return 1;
}

/* StepOptimizer::Step (BundlerLib.cpp:132-149) */
static int step_once(oracle_ba* b)
{
    if (b->dirty) initialize(b);
    if (b->useless) return 0;
    int r = lm_solve(b);
    b->iteration++;
    return r;
}

/* BundlerLib::StepBundleAdjustment (BundlerLib.cpp:364-447) */
int oracle_ba_step(oracle_ba* b, const float* huberw, int nsteps, float maxErrorSquare,
                   uint32_t* outliers, uint32_t cap, uint32_t* n_out, float* mean_sq)
{
    float prior = -1.f;
    for (int s = 0; s < nsteps; s++) {
        if (huberw[s] != prior) {
            b->huber = (double)huberw[s];
            prior = huberw[s];
        }
        if (!step_once(b)) break;
    }
    if (b->dirty) initialize(b); /* no Step ran on a fresh graph: activeEdges still empty */
    int count = 0;
    double error = 0;
    uint32_t no = 0;
    for (int i = 0; i < b->ne; i++) {
        edge_t* e = &b->edges[i];
        if (!e->active) continue;
        double sumSquares = e->err[0] * e->err[0] + e->err[1] * e->err[1];
        /* cheirality: (world point - camera centre) . forward, via SE3Quat::inverse */
        const se3q* T = &b->cams[e->cam].pose;
        double qc[4] = {-T->q[0], -T->q[1], -T->q[2], T->q[3]};
        double it[3], fwd[3];
        quat_rotate(qc, T->t, it);
        double trans[3] = {-it[0], -it[1], -it[2]};
        double z[3] = {0, 0, 1};
        quat_rotate(qc, z, fwd);
        const double* P = b->pts[e->pt].p;
        double dot = (P[0] - trans[0]) * fwd[0] + (P[1] - trans[1]) * fwd[1] + (P[2] - trans[2]) * fwd[2];
        if (dot <= 0 || sumSquares > (double)maxErrorSquare) {
            e->removed = 1;
            b->dirty = 1;
            if (no < cap) outliers[no] = (uint32_t)i;
            no++;
        } else {
            error += sumSquares;
            count++;
        }
    }
    *n_out = no;
    *mean_sq = (float)(error / count);
    return MAGE_OK;
}

void oracle_ba_get_poses(const oracle_ba* b, float* pos3, float* r9)
{
    for (int c = 0; c < b->nc; c++) {
        const se3q* s = &b->cams[c].pose;
        double q[4];
        memcpy(q, s->q, sizeof(q));
        quat_normalize(q);
        double R[9];
        quat_to_matrix(q, R);
        for (int k = 0; k < 3; k++) pos3[3 * c + k] = (float)s->t[k];
        for (int r = 0; r < 3; r++)
            for (int cc = 0; cc < 3; cc++) r9[9 * c + cc * 3 + r] = (float)R[r * 3 + cc];
    }
}

void oracle_ba_get_points(const oracle_ba* b, float* xyz)
{
    for (int p = 0; p < b->np; p++)
        for (int k = 0; k < 3; k++) xyz[3 * p + k] = (float)b->pts[p].p[k];
}

void oracle_ba_get_stats(const oracle_ba* b, uint64_t* iters, uint64_t* trials,
                         uint64_t* rejected, double* last_chi2, double* lambda)
{
    *iters = b->iters;
    *trials = b->trials;
    *rejected = b->rejected;
    *last_chi2 = b->last_chi2;
    *lambda = b->lambda;
}

/* Double-precision accessors used by the parity tests (poses as q,t; points). */
void oracle_ba_get_state(const oracle_ba* b, double* qt7, double* xyz)
{
    for (int c = 0; c < b->nc; c++) {
        memcpy(qt7 + 7 * c, b->cams[c].pose.q, 4 * sizeof(double));
        memcpy(qt7 + 7 * c + 4, b->cams[c].pose.t, 3 * sizeof(double));
    }
    for (int p = 0; p < b->np; p++) memcpy(xyz + 3 * p, b->pts[p].p, 3 * sizeof(double));
}

/* Residual/Jacobian of one observation at the current state, for finite-difference tests. */
void oracle_ba_edge_linearization(oracle_ba* b, int i, double err[2], double Jpt[6], double Jp[12])
{
    double xc[3];
    edge_error(b, &b->edges[i], err, xc);
    edge_jacobians(b, &b->edges[i], Jpt, Jp);
}

/* Apply a 6-dof update to camera c (exp map), for finite-difference tests. */
void oracle_ba_perturb_camera(oracle_ba* b, int c, const double u[6]) { se3_oplus(&b->cams[c].pose, u); }
void oracle_ba_perturb_point(oracle_ba* b, int p, const double u[3])
{
    for (int k = 0; k < 3; k++) b->pts[p].p[k] += u[k];
}

/* Error and Jacobians of tether i at the current state (indices after set order), for tests.
 * Returns the error dimension, or 0 if the tether is inactive / out of range. */
int oracle_ba_tether_linearization(oracle_ba* b, int i, double err[6], double J1[36], double J2[36])
{
    if (b->dirty) initialize(b);
    if (i < 0 || i >= b->nt || !b->teth[i].active) return 0;
    tether_t* t = &b->teth[i];
    tether_error(b, t, t->err);
    tether_jacobians(b, t);
    memcpy(err, t->err, sizeof(t->err));
    memcpy(J1, t->J[0], sizeof(t->J[0]));
    memcpy(J2, t->J[1], sizeof(t->J[1]));
    return t->dim;
}

/* TrackLocalMap::OptimizeCameraPose (TrackLocalMap.cpp:421-501) for a batch of independent
 * problems, each through a fresh BundlerLib with ArePointsFixed: one free camera, observation i
 * of problem k on point i, nsteps x huber, then the StepBundleAdjustment post-pass.  Outputs as
 * mage_ba_pose_batch (outlier flags per observation). */
void oracle_ba_pose_batch(uint32_t problems, const float* pos3, const float* r9, const float* intr4,
                          const uint32_t* obs_start, const float* points3, const float* uv, const float* info,
                          uint32_t nsteps, float huber, float max_error_square, float* pos3_out, float* r9_out,
                          double* qt7_out, uint8_t* outlier, float* mean_sq, uint32_t* stats)
{
    for (uint32_t k = 0; k < problems; k++) {
        const uint32_t e0 = obs_start[k], n = obs_start[k + 1] - e0;
        oracle_ba* b = oracle_ba_create(1);
        const uint8_t nofix = 0;
        oracle_ba_set_cameras(b, 1, pos3 + 3 * k, r9 + 9 * k, intr4 + 4 * k, &nofix);
        oracle_ba_set_points(b, (int)n, points3 + 3 * (size_t)e0);
        uint32_t* cam = (uint32_t*)calloc((size_t)n + 1, sizeof(uint32_t));
        uint32_t* pt = (uint32_t*)calloc((size_t)n + 1, sizeof(uint32_t));
        for (uint32_t i = 0; i < n; i++) pt[i] = i;
        oracle_ba_set_observations(b, (int)n, uv + 2 * (size_t)e0, cam, pt, info + e0);
        float* hw = (float*)malloc(sizeof(float) * ((size_t)nsteps + 1));
        for (uint32_t s = 0; s < nsteps; s++) hw[s] = huber;
        uint32_t* outl = (uint32_t*)calloc((size_t)n + 1, sizeof(uint32_t));
        uint32_t no = 0;
        oracle_ba_step(b, hw, (int)nsteps, max_error_square, outl, n, &no, &mean_sq[k]);
        for (uint32_t i = 0; i < n; i++) outlier[e0 + i] = 0;
        for (uint32_t i = 0; i < no && i < n; i++) outlier[e0 + outl[i]] = 1;
        oracle_ba_get_poses(b, pos3_out + 3 * k, r9_out + 9 * k);
        if (qt7_out) {
            memcpy(qt7_out + 7 * k, b->cams[0].pose.q, 4 * sizeof(double));
            memcpy(qt7_out + 7 * k + 4, b->cams[0].pose.t, 3 * sizeof(double));
        }
        if (stats) {
            stats[2 * k] = (uint32_t)b->iters;
            stats[2 * k + 1] = (uint32_t)b->trials;
        }
        free(cam);
        free(pt);
        free(hw);
        free(outl);
        oracle_ba_destroy(b);
    }
}
