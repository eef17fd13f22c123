// track.hip — the C4 tracking loop device-resident: the same specification as csrc/track.cpp
// (PoseEstimator::TryEstimatePoseFromKeyframe, PoseEstimator.cpp:439-607; TrackLocalMap's two
// OptimizeCameraPose passes, TrackLocalMap.cpp:37-140; NewKeyFrameDecision.cpp:196) with every
// per-frame decision taken on the device, so the host enqueues the whole sequence and
// synchronises once.  Per frame, in one stream:
//   trk_project     prediction (constant velocity on SE3, fp64) + ProjectUndistorted of the
//                   keyframe's map points (f32), ordered compaction of the points in front
//   radius x 3      RadiusMatch at SearchRadius / WiderSearchRadius (position overrides) /
//                   ExtraWiderSearchRadius (keypoint positions); pass k+1 gets a zero query
//                   count unless pass k ran and was weak (trk_weak), which the kernels skip
//   trk_gather      the last pass's matches -> pose-BA observations, "lost" when too few
//   pose BA 1       mage_ba_pose_batch_device (3 steps, Huber 4, 6^2)
//   trk_filter      ordered compaction of pass 1's inliers
//   pose BA 2       (4 steps, Huber 0.9, 4.5^2)
//   trk_finish      the frame's pose / counts, keyframe decision, new keyframe's map points
// Every expression matches track.cpp (same order, f32 projection, fp64 poses, no contraction:
// the library is built with -ffp-contract=off), so the two loops give identical results.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstring>
#include <vector>

#include "common.hpp"
#include "depth_noise.hpp"

namespace mage {
namespace {

constexpr int TT = 1024;  // threads of the per-frame control kernels
// RadiusMatch band-index ring of mage_track_sequence_device: chunks of BAND_CHUNK frames, two
// chunks resident (the host runs at most a few frames ahead of the device)
constexpr uint32_t BAND_CHUNK = 16, BAND_SLOTS = 2 * BAND_CHUNK;

struct DPose {
    double R[9];  // world -> camera, row-major
    double t[3];
};

__device__ void d_mv(const double* R, const double* v, double* out)
{
    for (int i = 0; i < 3; i++) out[i] = (R[3 * i] * v[0] + R[3 * i + 1] * v[1]) + R[3 * i + 2] * v[2];
}

__device__ DPose d_inverse(const DPose& p)
{
    DPose q;
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) q.R[3 * r + c] = p.R[3 * c + r];
    double m[3];
    d_mv(q.R, p.t, m);
    for (int i = 0; i < 3; i++) q.t[i] = -m[i];
    return q;
}

__device__ DPose d_mul(const DPose& a, const DPose& b)
{
    DPose o;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            o.R[3 * i + j] = (a.R[3 * i] * b.R[j] + a.R[3 * i + 1] * b.R[3 + j]) + a.R[3 * i + 2] * b.R[6 + j];
    double m[3];
    d_mv(a.R, b.t, m);
    for (int i = 0; i < 3; i++) o.t[i] = m[i] + a.t[i];
    return o;
}

__device__ DPose load_pose(const double* p)
{
    DPose q;
    for (int i = 0; i < 9; i++) q.R[i] = p[i];
    for (int i = 0; i < 3; i++) q.t[i] = p[9 + i];
    return q;
}

__device__ void store_pose(double* p, const DPose& q)
{
    for (int i = 0; i < 9; i++) p[i] = q.R[i];
    for (int i = 0; i < 3; i++) p[9 + i] = q.t[i];
}

// Exclusive position of this thread's item among the block's items with pr set, in thread order;
// *total = their count.  wsum: 16 words of LDS.
__device__ uint32_t block_prefix(bool pr, uint32_t* wsum, uint32_t* total)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t b = __ballot(pr);
    const uint32_t before = __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
    if (lane == 0) wsum[wave] = (uint32_t)__builtin_popcountll(b);
    __syncthreads();
    uint32_t woff = 0, tot = 0;
    for (int w = 0; w < TT / 64; w++) {
        if (w < wave) woff += wsum[w];
        tot += wsum[w];
    }
    __syncthreads();
    *total = tot;
    return woff + before;
}

constexpr int NKMAX = 8;  // keyframes of the local map

struct Ctl {              // per-call control words (device)
    uint32_t exec[3];     // radius pass k ran
    uint32_t ns;          // queries (keyframe points in front of the predicted camera)
    uint32_t lost;
    uint32_t kf_first;    // keyframe ring: oldest slot, slots in use (ascending keyframe id)
    uint32_t kf_count;
    uint32_t kf_n[NKMAX]; // keyframe feature counts per slot
    uint32_t lm_nq;       // local-map queries of the frame
    uint32_t kf_id[NKMAX];  // frame index of the keyframe in each slot
    uint32_t kf_an[NKMAX];  // associations per slot (the keyframe frame's pass-2 inliers)
    uint32_t halt;        // local BA pending: every frame kernel is a no-op until the host clears it
};

struct TrackBufs {
    Ctl* ctl;
    double* pred;          // 12
    // keyframe ring (NKMAX slots of cap entries; the reference keyframe is the newest slot)
    mage_keypoint* kf_kp;
    uint8_t* kf_desc;
    float* kf_pts;
    float* kf_mvd;   // mean viewing directions (3 per point)
    float* kf_dmin;
    float* kf_dmax;
    double* kf_pose;      // 12 per slot (R row-major, t)
    // mapping side (local BA): per point its refinement count and own-observation flag, per slot
    // the associations (owner keyframe id, point index, keypoint x, y bits) and their flags
    uint32_t* kf_ref;
    uint8_t* kf_own;
    int4* kf_assoc;
    uint8_t* kf_aalive;
    int2* src1;           // pose-BA observation sources (owner keyframe id, point index)
    int2* src2;
    float* info1;         // per observation: MapPointRefinementConfidence of the point
    float* info2;
    int2* lm_qsrc;
    float* lm_qinfo;
    uint32_t* prog;       // mapped host words {frame done, frame that requested a local BA}
    // local-map search
    uint32_t* lm_mask;    // unassociated keypoints (bit words)
    uint8_t* lm_visited;  // reference-keyframe points associated as pass-1 inliers
    int32_t* lm_hide;     // reference-keyframe points of pass-1 outliers: their keypoint
    float* lm_qpos;
    int32_t* lm_qoct;
    int32_t* lm_qhide;
    uint8_t* lm_qdesc;
    float* lm_qpt;        // the queries' map point positions
    int32_t* lm_res;
    uint32_t* lm_status;
    void* lm_scratch;
    // queries
    mage_keypoint* qkp;
    uint8_t* qdesc;
    float* qpos;
    uint32_t* sel;
    uint32_t* nq;          // 3: query count of each radius pass
    mage_dmatch* m;        // 3 x cap
    uint32_t* mn;          // 3
    // pose BA
    float* pos3;
    float* r9;
    float* intr4;
    uint32_t* os1;         // 2
    uint32_t* os2;         // 2
    float* pts1;
    float* uv1;
    float* pts2;
    float* uv2;
    float* pos3_o1;
    float* r9_o1;
    float* pos3_o2;
    float* r9_o2;
    uint8_t* out1;
    uint8_t* out2;
    float* msq;
};

struct TrackConst {
    float fx, fy, cx, cy;  // (float)K
    double K[4];
    double plane_z;
    mage_track_settings s;
    uint32_t cap;          // keypoints per frame slot
    uint32_t nk;           // keyframe ring slots (max(local_map_keyframes, 1))
    uint32_t qcap;         // local-map queries per frame (nk x cap)
    uint32_t acap;         // associations per keyframe slot (cap + qcap)
    float fmax[8], fmin[8];  // ComputeDMax / ComputeDMin factors per octave (powf on the host)
    float log2s;           // log2(scale factor)
};

__device__ float dot3f(const float* a, const float* b) { return ((0.f + a[0] * b[0]) + a[1] * b[1]) + a[2] * b[2]; }

// MapPointRefinementConfidence (Map/MappingMath.h:42-49): 1 - 1 / powf(1.5 + count, 2); the square
// of 1.5 + count is exact in float, so x * x is powf's result
__host__ __device__ inline float refinement_confidence(uint32_t count)
{
    const float x = 1.5f + (float)count;
    return 1.f - 1.f / (x * x);
}

// Pose::GetWorldSpacePosition of the float view matrix (see track.cpp world_position)
__device__ void world_position(const double* R, const double* t, float C[3])
{
    for (int i = 0; i < 3; i++) {
        float s = 0.f;
        for (int k = 0; k < 3; k++) s = s + (float)R[3 * k + i] * -(float)t[k];
        C[i] = s + 0.f;
    }
}

// Keyframe slot <- frame features (kp, desc, n) with map points back-projected at pose P onto the
// plane and their MapPoint::UpdateMeanViewDirectionAndDistances attributes (track.cpp
// map_point_attributes).
__device__ void make_keyframe(const TrackBufs& b, const TrackConst& c, uint32_t slot, const mage_keypoint* fk,
                              const uint8_t* fd, uint32_t nf, const DPose& P, uint32_t fid)
{
    const double fx = c.K[0], fy = c.K[1], cx = c.K[2], cy = c.K[3];
    const double* R = P.R;
    double C[3];
    for (int j = 0; j < 3; j++) C[j] = -((R[j] * P.t[0] + R[3 + j] * P.t[1]) + R[6 + j] * P.t[2]);
    float Cf[3];
    world_position(P.R, P.t, Cf);
    const size_t o = (size_t)slot * c.cap;
    if (threadIdx.x < 12) b.kf_pose[12 * slot + threadIdx.x] = threadIdx.x < 9 ? P.R[threadIdx.x] : P.t[threadIdx.x - 9];
    for (uint32_t i = threadIdx.x; i < nf; i += TT) {
        b.kf_ref[o + i] = 0;
        b.kf_own[o + i] = 1;
        b.kf_kp[o + i] = fk[i];
        const uint4* s = reinterpret_cast<const uint4*>(fd + 32ull * i);
        uint4* d = reinterpret_cast<uint4*>(b.kf_desc + 32ull * (o + i));
        d[0] = s[0];
        d[1] = s[1];
        const double u = ((double)fk[i].x - cx) / fx, v = ((double)fk[i].y - cy) / fy;
        double dd[3];
        for (int j = 0; j < 3; j++) dd[j] = (u * R[j] + v * R[3 + j]) + R[6 + j];
        double lam = (c.plane_z - C[2]) / dd[2];
        if (c.s.map_point_depth_noise != 0.f) lam = lam * depth_noise_factor(fid, i, c.s.map_point_depth_noise);
        float Pp[3];
        for (int j = 0; j < 3; j++) Pp[j] = (float)(C[j] + lam * dd[j]);
        for (int j = 0; j < 3; j++) b.kf_pts[3 * (o + i) + j] = Pp[j];
        float vv[3] = {Pp[0] - Cf[0], Pp[1] - Cf[1], Pp[2] - Cf[2]};
        const float d1 = sqrtf(dot3f(vv, vv));
        if (d1 != 0) {
            const float inv = 1.f / d1;
            for (int j = 0; j < 3; j++) vv[j] = vv[j] * inv;
        }
        const float d2 = sqrtf(dot3f(vv, vv));
        if (d2 != 0) {
            const float inv = 1.f / d2;
            for (int j = 0; j < 3; j++) vv[j] = vv[j] * inv;
        }
        for (int j = 0; j < 3; j++) b.kf_mvd[3 * (o + i) + j] = vv[j];
        const float dl[3] = {Cf[0] - Pp[0], Cf[1] - Pp[1], Cf[2] - Pp[2]};
        const float dist = sqrtf((dl[0] * dl[0] + dl[1] * dl[1]) + dl[2] * dl[2]);
        const int oc = min(max(fk[i].octave, 0), 7);
        b.kf_dmin[o + i] = dist * c.fmin[oc];
        b.kf_dmax[o + i] = dist * c.fmax[oc];
    }
}

__device__ __forceinline__ uint32_t ref_slot(const Ctl* ctl, const TrackConst& c)
{
    return (ctl->kf_first + ctl->kf_count - 1) % c.nk;
}

// Frame 0: its keyframe at the first pose (already in poses[0]).
// A frame's keypoint count, clamped to the frame slot (`cap` keypoints): a larger count would copy
// the next frame's (or unallocated) entries into the keyframe buffers, which hold `cap`; the
// overflow is reported through status bit 1 (MAGE_ECAPACITY on return).
__device__ uint32_t frame_count(const TrackConst& c, const uint32_t* nf, uint32_t* status)
{
    const uint32_t n = *nf;
    if (n > c.cap) {
        if (threadIdx.x == 0) atomicOr(status, 2u);
        return c.cap;
    }
    return n;
}

__global__ __launch_bounds__(TT) void trk_init(TrackBufs b, TrackConst c, const mage_keypoint* fk, const uint8_t* fd,
                                               const uint32_t* nf, double* poses, uint32_t* matches,
                                               uint32_t* inliers, uint8_t* keyframe, uint32_t* status)
{
    const uint32_t n = frame_count(c, nf, status);
    make_keyframe(b, c, 0, fk, fd, n, load_pose(poses), 0u);
    if (threadIdx.x == 0) {
        b.ctl->kf_first = 0;
        b.ctl->kf_count = 1;
        b.ctl->kf_n[0] = n;
        b.ctl->kf_id[0] = 0;
        b.ctl->kf_an[0] = 0;
        b.ctl->halt = 0;
        matches[0] = inliers[0] = n;
        keyframe[0] = 1;
        b.intr4[0] = c.cx;  // BundlerLib's {cx, cy, fx, fy}
        b.intr4[1] = c.cy;
        b.intr4[2] = c.fx;
        b.intr4[3] = c.fy;
    }
}

__device__ void project_frame(const TrackBufs& b, const TrackConst& c, int f, const double* poses)
{
    __shared__ float R32[9], t32[3];
    __shared__ uint32_t wsum[TT / 64];
    if (b.ctl->halt) {  // a local BA is pending: this frame runs again after it (zero counts downstream)
        if (threadIdx.x == 0) {
            b.ctl->ns = 0;
            for (int k = 0; k < 3; k++) b.ctl->exec[k] = b.nq[k] = 0;
        }
        return;
    }
    if (threadIdx.x == 0) {
        const DPose p1 = load_pose(poses + 12ll * (f - 1));
        const DPose pred = f < 2 ? p1 : d_mul(d_mul(p1, d_inverse(load_pose(poses + 12ll * (f - 2)))), p1);
        store_pose(b.pred, pred);
        for (int i = 0; i < 9; i++) R32[i] = (float)pred.R[i];
        for (int i = 0; i < 3; i++) t32[i] = (float)pred.t[i];
    }
    __syncthreads();
    const uint32_t slot = ref_slot(b.ctl, c), nk = b.ctl->kf_n[slot];
    const size_t o = (size_t)slot * c.cap;
    uint32_t base = 0;
    for (uint32_t c0 = 0; c0 < nk; c0 += TT) {
        const uint32_t i = c0 + threadIdx.x;
        bool front = false;
        float u = 0.f, v = 0.f;
        if (i < nk) {
            const float X = b.kf_pts[3 * (o + i)], Y = b.kf_pts[3 * (o + i) + 1], Z = b.kf_pts[3 * (o + i) + 2];
            float xc[3];
            for (int r = 0; r < 3; r++) xc[r] = ((R32[3 * r] * X + R32[3 * r + 1] * Y) + R32[3 * r + 2] * Z) + t32[r];
            front = xc[2] > 0.f;
            u = (xc[0] / xc[2]) * c.fx + c.cx;
            v = (xc[1] / xc[2]) * c.fy + c.cy;
        }
        uint32_t tot;
        const uint32_t pos = base + block_prefix(front, wsum, &tot);
        if (front) {
            b.qkp[pos] = b.kf_kp[o + i];
            const uint4* s = reinterpret_cast<const uint4*>(b.kf_desc + 32ull * (o + i));
            uint4* d = reinterpret_cast<uint4*>(b.qdesc + 32ull * pos);
            d[0] = s[0];
            d[1] = s[1];
            b.qpos[2 * pos] = u;
            b.qpos[2 * pos + 1] = v;
            b.sel[pos] = i;
        }
        base += tot;
    }
    if (threadIdx.x == 0) {
        b.ctl->ns = base;
        b.ctl->exec[0] = 1;
        b.ctl->exec[1] = b.ctl->exec[2] = 0;
        b.nq[0] = base;
        b.nq[1] = b.nq[2] = 0;
    }
}

// Pass k + 1 runs when pass k ran and its result is weak (too few matches or ratio).
__global__ void trk_weak(TrackBufs b, TrackConst c, int k)
{
    if (threadIdx.x != 0) return;
    const uint32_t ns = b.ctl->ns, n = b.mn[k];
    const bool weak = n < c.s.min_matches || (double)n / (double)max(ns, 1u) < c.s.small_match_ratio;
    const uint32_t run = b.ctl->exec[k] && weak;
    b.ctl->exec[k + 1] = run;
    b.nq[k + 1] = run ? ns : 0u;
}

__global__ __launch_bounds__(TT) void trk_gather(TrackBufs b, TrackConst c, const mage_keypoint* fk, int f,
                                                 uint32_t* matches)
{
    if (b.ctl->halt) {
        if (threadIdx.x == 0) {
            b.ctl->lost = 1;
            b.os1[0] = b.os1[1] = 0;
        }
        return;
    }
    const int fin = b.ctl->exec[2] ? 2 : (b.ctl->exec[1] ? 1 : 0);
    const uint32_t n = b.mn[fin];
    const bool lost = n < c.s.min_matches;
    const mage_dmatch* m = b.m + (size_t)fin * c.cap;
    if (!lost) {
        const uint32_t slot = ref_slot(b.ctl, c);
        const size_t o = (size_t)slot * c.cap;
        const int kid = (int)b.ctl->kf_id[slot];
        for (uint32_t k = threadIdx.x; k < n; k += TT) {
            const uint32_t q = b.sel[m[k].query_idx], t = (uint32_t)m[k].train_idx;
            for (int j = 0; j < 3; j++) b.pts1[3 * k + j] = b.kf_pts[3 * (o + q) + j];
            b.uv1[2 * k] = fk[t].x;
            b.uv1[2 * k + 1] = fk[t].y;
            b.info1[k] = refinement_confidence(b.kf_ref[o + q]);  // TrackLocalMap.cpp:473-475
            b.src1[k] = make_int2(kid, (int)q);
        }
    }
    if (threadIdx.x == 0) {
        matches[f] = n;
        b.ctl->lost = lost;
        b.os1[0] = 0;
        b.os1[1] = lost ? 0u : n;
        for (int i = 0; i < 3; i++) b.pos3[i] = (float)b.pred[9 + i];
        for (int r = 0; r < 3; r++)
            for (int cc = 0; cc < 3; cc++) b.r9[3 * cc + r] = (float)b.pred[3 * r + cc];  // column-major
    }
}

// Pass-1 inliers -> the pose-BA 2 observations (ordered compaction); with the local map on, the
// frame's associations after TrackLocalMap unassociates the outliers (:116-147): the unassociated
// keypoint mask, the reference points associated as inliers (visited) and each outlier point's
// keypoint (hidden from its own local-map search).
__device__ void filter_frame(const TrackBufs& b, const TrackConst& c, const uint32_t* nf_ptr)
{
    __shared__ uint32_t wsum[TT / 64];
    const uint32_t n = b.os1[1];
    uint32_t base = 0;
    for (uint32_t c0 = 0; c0 < n; c0 += TT) {
        const uint32_t k = c0 + threadIdx.x;
        const bool keep = k < n && !b.out1[k];
        uint32_t tot;
        const uint32_t pos = base + block_prefix(keep, wsum, &tot);
        if (keep) {
            for (int j = 0; j < 3; j++) b.pts2[3 * pos + j] = b.pts1[3 * k + j];
            b.uv2[2 * pos] = b.uv1[2 * k];
            b.uv2[2 * pos + 1] = b.uv1[2 * k + 1];
            b.info2[pos] = b.info1[k];
            b.src2[pos] = b.src1[k];
        }
        base += tot;
    }
    if (threadIdx.x == 0) {
        b.os2[0] = 0;
        b.os2[1] = base;
    }
    if (c.s.local_map_keyframes == 0 || b.ctl->lost) return;
    // the unassociated-keypoint mask is built in LDS (2000 atomics on ~63 global words serialised
    // at the L2) and written out once
    __shared__ uint32_t smask[4096 / 32];
    const uint32_t nf = min(min(*nf_ptr, c.cap), 4096u);
    const uint32_t nk = b.ctl->kf_n[ref_slot(b.ctl, c)];
    for (uint32_t w = threadIdx.x; w < (nf + 31) / 32; w += TT)
        smask[w] = (32 * w + 32 <= nf) ? 0xFFFFFFFFu : ((1u << (nf - 32 * w)) - 1u);
    for (uint32_t i = threadIdx.x; i < nk; i += TT) {
        b.lm_visited[i] = 0;
        b.lm_hide[i] = -1;
    }
    __syncthreads();
    const int fin = b.ctl->exec[2] ? 2 : (b.ctl->exec[1] ? 1 : 0);
    const mage_dmatch* m = b.m + (size_t)fin * c.cap;
    for (uint32_t k = threadIdx.x; k < n; k += TT) {
        const uint32_t q = b.sel[m[k].query_idx], t = (uint32_t)m[k].train_idx;
        if (!b.out1[k]) {
            if (t < nf) atomicAnd(&smask[t >> 5], ~(1u << (t & 31)));
            b.lm_visited[q] = 1;
        } else {
            b.lm_hide[q] = (int32_t)t;
        }
    }
    __syncthreads();
    for (uint32_t w = threadIdx.x; w < (nf + 31) / 32; w += TT) b.lm_mask[w] = smask[w];
}

// TrackLocalMap.cpp:149-223: the local map's unvisited points, keyframe by keyframe in ascending id,
// through ProjectMapPointIntoCurrentFrame / IsGoodCandidate / ComputeOctave with the pass-1 pose
// (tracking.py local_map_queries, track.cpp): ordered compaction of the candidates into queries.
// No pass-1 inlier left (mapPoints.empty(), :149-150) is a lost frame.
__device__ void lm_project_frame(const TrackBufs& b, const TrackConst& c)
{
    __shared__ uint32_t wsum[TT / 64];
    const bool off = c.s.local_map_keyframes == 0 || b.ctl->lost;
    if (off || b.os2[1] == 0) {
        if (threadIdx.x == 0) {
            if (!off) b.ctl->lost = 1;
            b.ctl->lm_nq = 0;
        }
        return;
    }
    float R[9], t[3], C[3];
    for (int r = 0; r < 3; r++)
        for (int cc = 0; cc < 3; cc++) R[3 * r + cc] = b.r9_o1[3 * cc + r];
    for (int i = 0; i < 3; i++) t[i] = b.pos3_o1[i];
    for (int i = 0; i < 3; i++) {
        float sum = 0.f;
        for (int k = 0; k < 3; k++) sum = sum + R[3 * k + i] * -t[k];
        C[i] = sum + 0.f;
    }
    const float fw[3] = {R[6], R[7], R[8]};
    const float border = c.s.image_border, W = (float)c.s.width, H = (float)c.s.height;
    const uint32_t first = b.ctl->kf_first, count = b.ctl->kf_count;
    uint32_t base = 0;
    for (uint32_t si = 0; si < count; si++) {
        const uint32_t slot = (first + si) % c.nk, n = b.ctl->kf_n[slot];
        const bool is_ref = si + 1 == count;
        const size_t o = (size_t)slot * c.cap;
        for (uint32_t c0 = 0; c0 < n; c0 += TT) {
            const uint32_t i = c0 + threadIdx.x;
            bool ok = i < n && !(is_ref && b.lm_visited[i]);
            float px = 0.f, py = 0.f;
            int oc = 0;
            if (ok) {
                const float* P = b.kf_pts + 3 * (o + i);
                float cs[3];
                for (int r = 0; r < 3; r++)
                    cs[r] = (((0.f + R[3 * r] * P[0]) + R[3 * r + 1] * P[1]) + R[3 * r + 2] * P[2]) + t[r] * 1.f;
                const float depth = cs[2], div = depth != 0 ? depth : 1.f;
                px = (cs[0] / div) * c.fx + c.cx;
                py = (cs[1] / div) * c.fy + c.cy;
                ok = !(depth < 0) && border <= px && border <= py && px < W - border && py < H - border;
                ok = ok && !(dot3f(b.kf_mvd + 3 * (o + i), fw) < c.s.min_view_cos);
                const float dl[3] = {P[0] - C[0], P[1] - C[1], P[2] - C[2]};
                const float d2 = (dl[0] * dl[0] + dl[1] * dl[1]) + dl[2] * dl[2];
                const float dmin = b.kf_dmin[o + i], dmax = b.kf_dmax[o + i];
                ok = ok && !(d2 < dmin * dmin || dmax * dmax < d2);
                if (ok) {
                    const float rr = sqrtf(d2) / dmin;
                    oc = (int)roundf((float)log2((double)rr) / c.log2s - 0.5f);
                    ok = oc >= 0 && oc <= (int)c.s.num_levels;
                }
            }
            uint32_t tot;
            const uint32_t pos = base + block_prefix(ok, wsum, &tot);
            if (ok && pos < c.qcap) {
                b.lm_qpos[2 * pos] = px;
                b.lm_qpos[2 * pos + 1] = py;
                b.lm_qoct[pos] = oc;
                b.lm_qhide[pos] = is_ref ? b.lm_hide[i] : -1;
                const uint4* sd = reinterpret_cast<const uint4*>(b.kf_desc + 32ull * (o + i));
                uint4* dd = reinterpret_cast<uint4*>(b.lm_qdesc + 32ull * pos);
                dd[0] = sd[0];
                dd[1] = sd[1];
                for (int j = 0; j < 3; j++) b.lm_qpt[3 * pos + j] = b.kf_pts[3 * (o + i) + j];
                b.lm_qsrc[pos] = make_int2((int)b.ctl->kf_id[slot], (int)i);
                b.lm_qinfo[pos] = refinement_confidence(b.kf_ref[o + i]);
            }
            base += tot;
        }
    }
    if (threadIdx.x == 0) b.ctl->lm_nq = min(base, c.qcap);
}

// The local map's new associations appended to the pass-2 observations in query order.
__global__ __launch_bounds__(TT) void trk_lm_assemble(TrackBufs b, const mage_keypoint* fk)
{
    __shared__ uint32_t wsum[TT / 64];
    const uint32_t nq = b.ctl->lm_nq;
    if (b.ctl->lost || nq == 0) return;
    const uint32_t base0 = b.os2[1];
    uint32_t base = base0;
    for (uint32_t c0 = 0; c0 < nq; c0 += TT) {
        const uint32_t q = c0 + threadIdx.x;
        const int r = q < nq ? b.lm_res[q] : -1;
        uint32_t tot;
        const uint32_t pos = base + block_prefix(r >= 0, wsum, &tot);
        if (r >= 0) {
            for (int j = 0; j < 3; j++) b.pts2[3 * pos + j] = b.lm_qpt[3 * q + j];
            b.uv2[2 * pos] = fk[r].x;
            b.uv2[2 * pos + 1] = fk[r].y;
            b.info2[pos] = b.lm_qinfo[q];
            b.src2[pos] = b.lm_qsrc[q];
        }
        base += tot;
    }
    if (threadIdx.x == 0) b.os2[1] = base;
}

__device__ void finish_frame(const TrackBufs& b, const TrackConst& c, int f, const mage_keypoint* fk,
                             const uint8_t* fd, const uint32_t* nf, double* poses, uint32_t* inliers,
                             uint8_t* keyframe, uint32_t* status)
{
    __shared__ uint32_t wsum[TT / 64];
    __shared__ int s_kf;
    __shared__ uint32_t s_slot;
    __shared__ double sP[12];
    if (b.ctl->halt) return;  // re-run after the pending local BA
    bool lost = b.ctl->lost != 0;
    uint32_t n_in = 0;
    if (!lost) {
        const uint32_t n2 = b.os2[1];
        for (uint32_t c0 = 0; c0 < n2; c0 += TT) {
            const uint32_t k = c0 + threadIdx.x;
            uint32_t tot;
            (void)block_prefix(k < n2 && !b.out2[k], wsum, &tot);
            n_in += tot;
        }
        // TrackLocalMap.cpp:309-314: too few associations after the second pass
        if (c.s.local_map_keyframes > 0 && n_in < c.s.min_tracked) lost = true;
    }
    if (threadIdx.x == 0) {
        DPose P;
        if (lost) {
            P = load_pose(b.pred);
        } else {
            for (int r = 0; r < 3; r++)
                for (int cc = 0; cc < 3; cc++) P.R[3 * r + cc] = (double)b.r9_o2[3 * cc + r];
            for (int i = 0; i < 3; i++) P.t[i] = (double)b.pos3_o2[i];
        }
        store_pose(poses + 12ll * f, P);
        store_pose(sP, P);
        inliers[f] = lost ? 0u : n_in;
        const uint32_t nk = b.ctl->kf_n[ref_slot(b.ctl, c)];
        s_kf = !lost && (double)n_in < c.s.keyframe_ratio * (double)nk + (double)c.s.keyframe_min;
        keyframe[f] = (uint8_t)s_kf;
        if (s_kf) {  // the keyframe ring: a free slot, or the oldest keyframe's
            if (b.ctl->kf_count < c.nk) {
                s_slot = (b.ctl->kf_first + b.ctl->kf_count) % c.nk;
                b.ctl->kf_count++;
            } else {
                s_slot = b.ctl->kf_first;
                b.ctl->kf_first = (b.ctl->kf_first + 1) % c.nk;
            }
        }
    }
    __syncthreads();
    if (s_kf) {
        const uint32_t n = frame_count(c, nf, status);
        make_keyframe(b, c, s_slot, fk, fd, n, load_pose(sP), f);
        // its associations: the pass-2 inliers in observation order (ordered compaction)
        const uint32_t n2 = b.os2[1];
        int4* as = b.kf_assoc + (size_t)s_slot * c.acap;
        uint8_t* aa = b.kf_aalive + (size_t)s_slot * c.acap;
        uint32_t base = 0;
        for (uint32_t c0 = 0; c0 < n2; c0 += TT) {
            const uint32_t k = c0 + threadIdx.x;
            const bool in = k < n2 && !b.out2[k];
            uint32_t tot;
            const uint32_t pos = base + block_prefix(in, wsum, &tot);
            if (in && pos < c.acap) {
                as[pos] = make_int4(b.src2[k].x, b.src2[k].y, __float_as_int(b.uv2[2 * k]), __float_as_int(b.uv2[2 * k + 1]));
                aa[pos] = 1;
            }
            base += tot;
        }
        if (threadIdx.x == 0) {
            b.ctl->kf_n[s_slot] = n;
            b.ctl->kf_id[s_slot] = (uint32_t)f;
            b.ctl->kf_an[s_slot] = min(base, c.acap);
            // a window needs two keyframes: halt the queued frames until the host ran the local BA
            if (c.s.local_ba && b.ctl->kf_count >= 2) b.ctl->halt = 1;
        }
    }
    if (b.prog && threadIdx.x == 0) {  // progress for the host (local BA): request word, then frame
        if (s_kf && c.s.local_ba && b.ctl->kf_count >= 2) *reinterpret_cast<volatile uint32_t*>(b.prog + 1) = (uint32_t)f;
        __threadfence_system();
        *reinterpret_cast<volatile uint32_t*>(b.prog) = (uint32_t)f;
    }
}

// The per-frame control kernels, and two fused pairs that save a dependent launch each per frame
// (the parts are separated by a workgroup barrier: what one part writes to global memory the next
// reads in the same workgroup).
__global__ __launch_bounds__(TT) void trk_project(TrackBufs b, TrackConst c, int f, const double* poses)
{
    project_frame(b, c, f, poses);
}

__global__ __launch_bounds__(TT) void trk_filter(TrackBufs b, TrackConst c, const uint32_t* nf_ptr)
{
    filter_frame(b, c, nf_ptr);
}

// trk_filter + trk_lm_project (the local map's candidate queries of the frame)
__global__ __launch_bounds__(TT) void trk_filter_lm(TrackBufs b, TrackConst c, const uint32_t* nf_ptr)
{
    filter_frame(b, c, nf_ptr);
    __syncthreads();
    lm_project_frame(b, c);
}

// trk_finish of frame f + trk_project of frame f + 1 (its prediction needs f's pose and ring)
__global__ __launch_bounds__(TT) void trk_finish_project(TrackBufs b, TrackConst c, int f, const mage_keypoint* fk,
                                                         const uint8_t* fd, const uint32_t* nf, double* poses,
                                                         uint32_t* inliers, uint8_t* keyframe, uint32_t* status,
                                                         int project_next)
{
    finish_frame(b, c, f, fk, fd, nf, poses, inliers, keyframe, status);
    if (!project_next) return;
    __syncthreads();
    project_frame(b, c, f + 1, poses);
}

}  // namespace
}  // namespace mage

namespace mage {
namespace {

// ---- Local BA of the device loop (host side, between frames: MappingWorker's BundleAdjustTask) ----
// The same window / schedule / write-back as tracking.py build_ba_window + apply_ba_window, over the
// keyframe ring copied from the device; BundlerLib through the C-ABI (one instance per call of the
// loop, the lambda persisted across windows as MappingWorker does).
// MAGE_TRACK_PROFILE=1 in the environment: per-window phase times of the local BA on stderr
// (development; tools/track_kernels.py)
struct PhaseClock {
    bool on = false;
    std::chrono::steady_clock::time_point t;
    char line[512];
    int len = 0;
    void start()
    {
        if (!on) return;
        t = std::chrono::steady_clock::now();
        len = 0;
    }
    void mark(const char* name)
    {
        if (!on) return;
        const auto n = std::chrono::steady_clock::now();
        len += snprintf(line + len, sizeof(line) - len, " %s %.3f", name,
                        std::chrono::duration<double, std::milli>(n - t).count());
        t = n;
    }
    void flush()
    {
        if (on) fprintf(stderr, "local BA window ms:%s\n", line);
    }
};

// Page-locked host array (the ring's host copy): DMA copies in both directions, queued with
// hipMemcpyAsync on the loop's stream instead of one synchronous pageable copy per field.
template <class T>
struct Pinned {
    T* p = nullptr;
    size_t n = 0;
    Pinned() = default;
    Pinned(const Pinned&) = delete;
    Pinned& operator=(const Pinned&) = delete;
    ~Pinned()
    {
        if (p) (void)hipHostFree(p);
    }
    bool resize(size_t m)
    {
        if (m <= n) return true;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
        if (hipHostMalloc(reinterpret_cast<void**>(&p), std::max<size_t>(m, 1) * sizeof(T), hipHostMallocDefault) != hipSuccess)
            return false;
        n = m;
        return true;
    }
    T& operator[](size_t i) { return p[i]; }
    const T& operator[](size_t i) const { return p[i]; }
    T* data() { return p; }
};

struct HostRing {
    uint32_t first = 0, count = 0, nk = 0, cap = 0, acap = 0;
    uint32_t n[NKMAX], id[NKMAX], an[NKMAX];
    // a page-locked byte-for-byte mirror of the device ring's fields (one DMA copy each way per
    // window); the arrays below point into it at the device layout's offsets
    Pinned<uint8_t> mirror;
    double* pose = nullptr;       // 12 per slot
    mage_keypoint* kp = nullptr;  // cap per slot
    float *pts = nullptr, *mvd = nullptr, *dmin = nullptr, *dmax = nullptr;
    uint32_t* ref = nullptr;
    uint8_t *own = nullptr, *aalive = nullptr;
    int4* assoc = nullptr;
    Pinned<uint32_t> zero;  // the halt word's clear value
};

struct LocalBA {  // MappingWorker's CurrentLambda and CosVisThreashold, persisted across the windows
    bool have_lambda = false;
    float lambda = 0.f;
    bool have_theta = false;
    uint32_t theta = 0;
};

struct BundlerHandle {  // a fresh BundlerLib per window (BundleAdjust.cpp MakeBundler)
    mage_ba* ba = nullptr;
    ~BundlerHandle()
    {
        if (ba) mage_ba_destroy(ba);
    }
};

void host_world_position(const double* R, const double* t, float C[3])
{
    for (int i = 0; i < 3; i++) {
        float sum = 0.f;
        for (int k = 0; k < 3; k++) sum = sum + (float)R[3 * k + i] * -(float)t[k];
        C[i] = sum + 0.f;
    }
}

float host_dot3(const float* a, const float* b) { return ((0.f + a[0] * b[0]) + a[1] * b[1]) + a[2] * b[2]; }

float bits_float(int v)
{
    float f;
    std::memcpy(&f, &v, 4);
    return f;
}

// tracking.point_attributes for point i of a slot
void host_point_attributes(HostRing& R, uint32_t slot, uint32_t i, const TrackConst& c)
{
    const size_t o = (size_t)slot * R.cap + i;
    float C[3];
    host_world_position(&R.pose[12 * slot], &R.pose[12 * slot + 9], C);
    const float* P = &R.pts[3 * o];
    float v[3] = {P[0] - C[0], P[1] - C[1], P[2] - C[2]};
    const float d = sqrtf(host_dot3(v, v));
    if (d != 0) {
        const float inv = 1.f / d;
        for (float& x : v) x = x * inv;
    }
    const float d2 = sqrtf(host_dot3(v, v));
    if (d2 != 0) {
        const float inv = 1.f / d2;
        for (float& x : v) x = x * inv;
    }
    for (int j = 0; j < 3; j++) R.mvd[3 * o + j] = v[j];
    const float dl[3] = {C[0] - P[0], C[1] - P[1], C[2] - P[2]};
    const float dist = sqrtf((dl[0] * dl[0] + dl[1] * dl[1]) + dl[2] * dl[2]);
    const int oc = std::min(std::max(R.kp[o].octave, 0), 7);
    R.dmin[o] = dist * c.fmin[oc];
    R.dmax[o] = dist * c.fmax[oc];
}

// One local BA on the ring (on the host copy); returns the outlier count (UINT32_MAX: no window).
mage_status host_local_ba(HostRing& R, const TrackConst& c, LocalBA& L, int device, uint32_t* n_out,
                          std::vector<uint8_t>& slot_changed, PhaseClock& prof)
{
    *n_out = 0xFFFFFFFFu;
    const uint32_t nr = R.count;
    if (nr < 2) return MAGE_OK;
    uint32_t slot_of[NKMAX];
    for (uint32_t r = 0; r < nr; r++) slot_of[r] = (R.first + r) % R.nk;
    auto pos_of = [&](int id) -> int {
        for (uint32_t r = 0; r < nr; r++)
            if ((int)R.id[slot_of[r]] == id) return (int)r;
        return -1;
    };
    struct Obs {
        uint32_t cam, owner, idx;
        float u, v;
        uint32_t kind, src;  // 0: own (point index), 1: association (entry)
    };
    std::vector<Obs> obs;
    obs.reserve((size_t)nr * R.cap * 2);
    for (uint32_t r = 0; r < nr; r++) {
        const uint32_t sl = slot_of[r];
        const size_t o = (size_t)sl * R.cap;
        for (uint32_t i = 0; i < R.n[sl]; i++)
            if (R.own[o + i]) obs.push_back({r, r, i, R.kp[o + i].x, R.kp[o + i].y, 0, i});
        const size_t ao = (size_t)sl * R.acap;
        for (uint32_t a = 0; a < R.an[sl]; a++) {
            const int4 e = R.assoc[ao + a];
            const int ow = pos_of(e.x);
            if (R.aalive[ao + a] && ow >= 0)
                obs.push_back({r, (uint32_t)ow, (uint32_t)e.y, bits_float(e.z), bits_float(e.w), 1, a});
        }
    }
    // the window's points, ascending (owner, index): a dense (ring position, index) map instead of
    // a sorted key list (the window build runs between frames, on the loop's critical path)
    std::vector<int32_t> pmap((size_t)nr * R.cap, -1);
    uint32_t freemask = 0;
    if (c.s.ba_free_keyframes > 0) {
        // the newest ba_free_keyframes free, the oldest fixed (at least one); the points they observe
        const uint32_t nfix = nr > c.s.ba_free_keyframes ? nr - c.s.ba_free_keyframes : 1u;
        for (uint32_t r = nfix; r < nr; r++) freemask |= 1u << r;
        for (const Obs& ob : obs)
            if (ob.cam >= nfix) pmap[(size_t)ob.owner * R.cap + ob.idx] = 0;
    } else {
        // GetMapPointsAndDistantKeyframes (ThreadSafeMap.cpp:888-957; tracking.py covisible_window):
        // per point the mask of ring keyframes observing it; the covisibility weight of keyframe r
        // to the newest one is the count of points both observe (CovisibilityGraph.cpp:131-170)
        std::vector<uint8_t> seen((size_t)nr * R.cap, 0);
        for (const Obs& ob : obs) seen[(size_t)ob.owner * R.cap + ob.idx] |= (uint8_t)(1u << ob.cam);
        const uint32_t last = nr - 1;
        uint32_t weight[NKMAX] = {};
        for (uint8_t m : seen)
            if (m >> last & 1u)
                for (uint32_t r = 0; r < last; r++) weight[r] += m >> r & 1u;
        uint32_t theta = L.have_theta ? L.theta : c.s.covis_min_threshold, kc = 0;
        for (uint32_t step = 0; step <= c.s.covis_max_steps; step++) {
            kc = 1u << last;
            for (uint32_t r = 0; r < last; r++)
                if (weight[r] >= theta) kc |= 1u << r;
            size_t n_assoc = 0;
            for (const Obs& ob : obs) n_assoc += (seen[(size_t)ob.owner * R.cap + ob.idx] & kc) != 0;
            if (n_assoc > c.s.ba_upper_connections) {
                theta += c.s.covis_ba_step;
                continue;
            }
            if (n_assoc < c.s.ba_lower_connections && theta > c.s.covis_min_threshold) {
                theta -= c.s.covis_ba_step;
                continue;
            }
            break;
        }
        L.theta = theta;
        L.have_theta = true;
        for (size_t q = 0; q < seen.size(); q++)
            if (seen[q] & kc) pmap[q] = 0;
        for (uint32_t r = 0; r < nr; r++)  // the map's first keyframe stays fixed (ThreadSafeMap.cpp:89)
            if ((kc >> r & 1u) && R.id[slot_of[r]] != 0) freemask |= 1u << r;
    }
    std::vector<uint64_t> keys;
    for (uint32_t r = 0; r < nr; r++)
        for (uint32_t i = 0; i < R.cap; i++)
            if (pmap[(size_t)r * R.cap + i] == 0) {
                pmap[(size_t)r * R.cap + i] = (int32_t)keys.size();
                keys.push_back((uint64_t)r << 32 | i);
            }
    std::vector<Obs> kept;
    std::vector<uint32_t> cam, pt;
    std::vector<float> uv, info;
    kept.reserve(obs.size());
    cam.reserve(obs.size());
    pt.reserve(obs.size());
    uv.reserve(2 * obs.size());
    for (const Obs& ob : obs) {
        const int32_t p = pmap[(size_t)ob.owner * R.cap + ob.idx];
        if (p < 0) continue;
        kept.push_back(ob);
        cam.push_back(ob.cam);
        pt.push_back((uint32_t)p);
        uv.push_back(ob.u);
        uv.push_back(ob.v);
    }
    if (kept.empty() || freemask == 0) return MAGE_OK;
    const uint32_t P = (uint32_t)keys.size(), E = (uint32_t)kept.size();
    std::vector<float> xyz(3ull * P);
    std::vector<uint32_t> pref(P);
    for (uint32_t q = 0; q < P; q++) {
        const uint32_t sl = slot_of[keys[q] >> 32], i = (uint32_t)(keys[q] & 0xFFFFFFFFu);
        const size_t o = (size_t)sl * R.cap + i;
        for (int j = 0; j < 3; j++) xyz[3 * q + j] = R.pts[3 * o + j];
        pref[q] = R.ref[o];
    }
    for (uint32_t e = 0; e < E; e++) info.push_back(refinement_confidence(pref[pt[e]]));
    // cameras: view-space t, Eigen column-major R, {cx, cy, fx, fy}; the oldest fixed
    std::vector<float> pos3(3 * nr), r9(9 * nr), intr(4 * nr);
    std::vector<uint8_t> fixed(nr, 0);
    for (uint32_t r = 0; r < nr; r++) fixed[r] = (freemask >> r & 1u) ? 0 : 1;
    for (uint32_t r = 0; r < nr; r++) {
        const double* ps = &R.pose[12 * slot_of[r]];
        for (int i = 0; i < 3; i++) pos3[3 * r + i] = (float)ps[9 + i];
        for (int rr = 0; rr < 3; rr++)
            for (int cc = 0; cc < 3; cc++) r9[9 * r + 3 * cc + rr] = (float)ps[3 * rr + cc];
        intr[4 * r] = (float)c.K[2];
        intr[4 * r + 1] = (float)c.K[3];
        intr[4 * r + 2] = (float)c.K[0];
        intr[4 * r + 3] = (float)c.K[1];
    }
    // NumStepsPerRun / Huber width by the connectivity ratio (MappingWorker.cpp:254-263)
    const uint32_t ratio = c.s.ba_upper_connections / E;
    uint32_t steps = c.s.ba_steps_per_run;
    float huber = c.s.ba_huber;
    if (ratio > 0) {
        steps = steps * (uint32_t)((float)ratio * c.s.ba_low_connectivity_scale);
        huber = huber * powf(c.s.ba_huber_scale, (float)ratio);
    }
    const std::vector<float> hw(std::max(steps, 1u), huber);
    mage_status st;
    prof.mark("window");
    BundlerHandle H;
    if ((st = mage_ba_create(0, device, &H.ba)) != MAGE_OK) return st;
    prof.mark("create");
    if (L.have_lambda && (st = mage_ba_set_lambda(H.ba, L.lambda)) != MAGE_OK) return st;
    if ((st = mage_ba_set_cameras(H.ba, nr, pos3.data(), r9.data(), intr.data(), fixed.data())) != MAGE_OK ||
        (st = mage_ba_set_points(H.ba, P, xyz.data())) != MAGE_OK ||
        (st = mage_ba_set_observations(H.ba, E, uv.data(), cam.data(), pt.data(), info.data())) != MAGE_OK)
        return st;
    prof.mark("setters");
    std::vector<uint32_t> outl(E);
    uint32_t nout = 0;
    float ms = 0.f;
    if ((st = mage_ba_step(H.ba, hw.data(), (uint32_t)hw.size(), c.s.ba_max_outlier_error, outl.data(), E, &nout, &ms)) !=
        MAGE_OK)
        return st;
    prof.mark("step");
    std::vector<float> pos_o(3 * nr), r9_o(9 * nr), xyz_o(3ull * P);
    float lam = 0.f;
    if ((st = mage_ba_get_poses(H.ba, pos_o.data(), r9_o.data())) != MAGE_OK ||
        (st = mage_ba_get_points(H.ba, xyz_o.data())) != MAGE_OK || (st = mage_ba_get_lambda(H.ba, &lam)) != MAGE_OK)
        return st;
    L.have_lambda = true;
    L.lambda = std::max(lam, c.s.min_lambda);
    // AdjustPosesAndMapPoints: outlier associations, free poses, points (+ refinement), attributes
    for (uint32_t k = 0; k < std::min(nout, E); k++) {
        const Obs& ob = kept[outl[k]];
        const uint32_t sl = slot_of[ob.cam];
        if (ob.kind == 0)
            R.own[(size_t)sl * R.cap + ob.src] = 0;
        else
            R.aalive[(size_t)sl * R.acap + ob.src] = 0;
        slot_changed[sl] = 1;
    }
    for (uint32_t r = 0; r < nr; r++) {
        if (!(freemask >> r & 1u)) continue;
        double* ps = &R.pose[12 * slot_of[r]];
        for (int rr = 0; rr < 3; rr++)
            for (int cc = 0; cc < 3; cc++) ps[3 * rr + cc] = (double)r9_o[9 * r + 3 * cc + rr];
        for (int i = 0; i < 3; i++) ps[9 + i] = (double)pos_o[3 * r + i];
        slot_changed[slot_of[r]] = 1;
    }
    for (uint32_t q = 0; q < P; q++) {
        const uint32_t sl = slot_of[keys[q] >> 32], i = (uint32_t)(keys[q] & 0xFFFFFFFFu);
        const size_t o = (size_t)sl * R.cap + i;
        for (int j = 0; j < 3; j++) R.pts[3 * o + j] = xyz_o[3 * q + j];
        R.ref[o] += 1;
        slot_changed[sl] = 1;
    }
    for (uint32_t q = 0; q < P; q++)
        host_point_attributes(R, slot_of[keys[q] >> 32], (uint32_t)(keys[q] & 0xFFFFFFFFu), c);
    prof.mark("get + apply");
    *n_out = nout;
    return MAGE_OK;
}

}  // namespace
}  // namespace mage

extern "C" mage_status mage_track_sequence_device(const mage_keypoint* d_kp, const uint8_t* d_desc, uint32_t pitch,
                                                  const uint32_t* d_n, uint32_t frames, const double K[4],
                                                  const double first_pose[12], double plane_z,
                                                  const mage_track_settings* s, double* poses, uint32_t* matches,
                                                  uint32_t* inliers, uint8_t* keyframe, uint32_t* ba_outliers,
                                                  mage_stream stream)
{
    using namespace mage;
    MAGE_REQUIRE(K && first_pose && s && poses && matches && inliers && keyframe, MAGE_EINVAL, "null argument");
    if (frames == 0) return MAGE_OK;
    MAGE_REQUIRE(d_kp && d_desc && d_n, MAGE_EINVAL, "null features");
    MAGE_REQUIRE(pitch > 0 && pitch <= 4096, MAGE_EINVAL, "frame pitch must be in [1, 4096] keypoints");
    hipStream_t st = (hipStream_t)stream;
    MAGE_REQUIRE(s->local_map_keyframes <= (uint32_t)NKMAX, MAGE_EINVAL, "local_map_keyframes must be <= 8");
    // the observations' information is MapPointRefinementConfidence of each point's refinement
    // count (TrackLocalMap.cpp:473-475); the setting only names its count-0 value
    MAGE_REQUIRE(s->refinement_info == refinement_confidence(0), MAGE_EINVAL,
                 "refinement_info must be MapPointRefinementConfidence(0) = 1 - 1/1.5^2");
    const size_t cap = pitch;
    const uint32_t NK = std::max(s->local_map_keyframes, 1u);
    const size_t qcap = s->local_map_keyframes > 0 ? (size_t)NK * cap : 0;  // local-map queries
    const size_t c2 = cap + qcap;                                           // pose-BA 2 observations
    const size_t acap = c2;                                                 // associations per keyframe
    // one device allocation for the per-call scratch and outputs
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off = al(off + bytes);
        return o;
    };
    const size_t o_ctl = take(sizeof(Ctl)), o_pred = take(12 * 8), o_kfkp = take(28 * cap * NK),
                 o_kfd = take(32 * cap * NK), o_kfp = take(12 * cap * NK), o_kfv = take(12 * cap * NK),
                 o_kfdn = take(4 * cap * NK), o_kfdx = take(4 * cap * NK), o_kfps = take(96 * NK),
                 o_kfr = take(4 * cap * NK), o_kfo = take(cap * NK), o_kfa = take(16 * acap * NK), o_kfaa = take(acap * NK),
                 o_s1 = take(8 * cap), o_s2 = take(8 * c2), o_i1 = take(4 * cap), o_lqs = take(8 * qcap),
                 o_lqi = take(4 * qcap), o_qkp = take(28 * cap), o_qd = take(32 * cap),
                 o_qp = take(8 * cap), o_sel = take(4 * cap), o_nq = take(16), o_m = take(3 * 16 * cap), o_mn = take(16),
                 o_rs = take(4 * cap), o_rst = take(4), o_pos = take(12), o_r9 = take(36), o_in = take(16),
                 o_os1 = take(8), o_os2 = take(8), o_p1 = take(12 * cap), o_u1 = take(8 * cap), o_p2 = take(12 * c2),
                 o_u2 = take(8 * c2), o_inf = take(4 * c2), o_po1 = take(12), o_ro1 = take(36), o_po2 = take(12),
                 o_ro2 = take(36), o_out1 = take(cap), o_out2 = take(c2), o_msq = take(8),
                 o_lmm = take(4 * 4096 / 32), o_lmv = take(cap), o_lmh = take(4 * cap), o_lqp = take(8 * qcap),
                 o_lqo = take(4 * qcap), o_lqh = take(4 * qcap), o_lqd = take(32 * qcap), o_lqt = take(12 * qcap),
                 o_lres = take(4 * qcap), o_lst = take(4), o_lscr = take(local_map_scratch_bytes((uint32_t)qcap)),
                 o_poses = take(96ull * frames), o_mt = take(4ull * frames), o_il = take(4ull * frames),
                 o_kf = take(frames), o_bk = take(8ull * pitch * BAND_SLOTS), o_bxy = take(8ull * pitch * BAND_SLOTS),
                 o_bd = take(32ull * pitch * BAND_SLOTS);
    DeviceBuffer buf;
    mage_status r = buf.reserve(off);
    if (r != MAGE_OK) return r;
    char* d = buf.as<char>();
    TrackBufs b{};
    b.ctl = reinterpret_cast<Ctl*>(d + o_ctl);
    b.pred = reinterpret_cast<double*>(d + o_pred);
    b.kf_kp = reinterpret_cast<mage_keypoint*>(d + o_kfkp);
    b.kf_desc = reinterpret_cast<uint8_t*>(d + o_kfd);
    b.kf_pts = reinterpret_cast<float*>(d + o_kfp);
    b.kf_mvd = reinterpret_cast<float*>(d + o_kfv);
    b.kf_dmin = reinterpret_cast<float*>(d + o_kfdn);
    b.kf_dmax = reinterpret_cast<float*>(d + o_kfdx);
    b.kf_pose = reinterpret_cast<double*>(d + o_kfps);
    b.kf_ref = reinterpret_cast<uint32_t*>(d + o_kfr);
    b.kf_own = reinterpret_cast<uint8_t*>(d + o_kfo);
    b.kf_assoc = reinterpret_cast<int4*>(d + o_kfa);
    b.kf_aalive = reinterpret_cast<uint8_t*>(d + o_kfaa);
    b.src1 = reinterpret_cast<int2*>(d + o_s1);
    b.src2 = reinterpret_cast<int2*>(d + o_s2);
    b.info1 = reinterpret_cast<float*>(d + o_i1);
    b.lm_qsrc = reinterpret_cast<int2*>(d + o_lqs);
    b.lm_qinfo = reinterpret_cast<float*>(d + o_lqi);
    b.lm_mask = reinterpret_cast<uint32_t*>(d + o_lmm);
    b.lm_visited = reinterpret_cast<uint8_t*>(d + o_lmv);
    b.lm_hide = reinterpret_cast<int32_t*>(d + o_lmh);
    b.lm_qpos = reinterpret_cast<float*>(d + o_lqp);
    b.lm_qoct = reinterpret_cast<int32_t*>(d + o_lqo);
    b.lm_qhide = reinterpret_cast<int32_t*>(d + o_lqh);
    b.lm_qdesc = reinterpret_cast<uint8_t*>(d + o_lqd);
    b.lm_qpt = reinterpret_cast<float*>(d + o_lqt);
    b.lm_res = reinterpret_cast<int32_t*>(d + o_lres);
    b.lm_status = reinterpret_cast<uint32_t*>(d + o_lst);
    b.lm_scratch = d + o_lscr;
    b.qkp = reinterpret_cast<mage_keypoint*>(d + o_qkp);
    b.qdesc = reinterpret_cast<uint8_t*>(d + o_qd);
    b.qpos = reinterpret_cast<float*>(d + o_qp);
    b.sel = reinterpret_cast<uint32_t*>(d + o_sel);
    b.nq = reinterpret_cast<uint32_t*>(d + o_nq);
    b.m = reinterpret_cast<mage_dmatch*>(d + o_m);
    b.mn = reinterpret_cast<uint32_t*>(d + o_mn);
    b.pos3 = reinterpret_cast<float*>(d + o_pos);
    b.r9 = reinterpret_cast<float*>(d + o_r9);
    b.intr4 = reinterpret_cast<float*>(d + o_in);
    b.os1 = reinterpret_cast<uint32_t*>(d + o_os1);
    b.os2 = reinterpret_cast<uint32_t*>(d + o_os2);
    b.pts1 = reinterpret_cast<float*>(d + o_p1);
    b.uv1 = reinterpret_cast<float*>(d + o_u1);
    b.pts2 = reinterpret_cast<float*>(d + o_p2);
    b.uv2 = reinterpret_cast<float*>(d + o_u2);
    b.info2 = reinterpret_cast<float*>(d + o_inf);
    b.pos3_o1 = reinterpret_cast<float*>(d + o_po1);
    b.r9_o1 = reinterpret_cast<float*>(d + o_ro1);
    b.pos3_o2 = reinterpret_cast<float*>(d + o_po2);
    b.r9_o2 = reinterpret_cast<float*>(d + o_ro2);
    b.out1 = reinterpret_cast<uint8_t*>(d + o_out1);
    b.out2 = reinterpret_cast<uint8_t*>(d + o_out2);
    b.msq = reinterpret_cast<float*>(d + o_msq);
    int32_t* rscratch = reinterpret_cast<int32_t*>(d + o_rs);
    uint32_t* rstatus = reinterpret_cast<uint32_t*>(d + o_rst);
    double* dposes = reinterpret_cast<double*>(d + o_poses);
    uint32_t* dmt = reinterpret_cast<uint32_t*>(d + o_mt);
    uint32_t* dil = reinterpret_cast<uint32_t*>(d + o_il);
    uint8_t* dkf = reinterpret_cast<uint8_t*>(d + o_kf);
    // RadiusMatch band indices (each frame is matched up to 3 times, so its index is built once):
    // a ring of BAND_SLOTS frames, built BAND_CHUNK frames at a time by the enqueue of a chunk's
    // first frame — the loop runs at most DEPTH frames ahead, so a chunk's slots are free again
    // when the chunk two ahead is built, and device memory does not grow with the sequence
    unsigned long long* bkeys = reinterpret_cast<unsigned long long*>(d + o_bk);
    float* bxy = reinterpret_cast<float*>(d + o_bxy);
    uint32_t* bdesc = reinterpret_cast<uint32_t*>(d + o_bd);

    TrackConst c{};
    c.fx = (float)K[0];
    c.fy = (float)K[1];
    c.cx = (float)K[2];
    c.cy = (float)K[3];
    for (int i = 0; i < 4; i++) c.K[i] = K[i];
    c.plane_z = plane_z;
    c.s = *s;
    c.cap = pitch;
    c.nk = NK;
    c.qcap = (uint32_t)qcap;
    c.acap = (uint32_t)acap;
    for (int o = 0; o < 8; o++) {
        c.fmax[o] = powf(s->scale_factor, (float)s->num_levels - ((float)o + 0.5f));
        c.fmin[o] = powf(s->scale_factor, 0.f - ((float)o + 0.5f));
    }
    c.log2s = (float)std::log2((double)s->scale_factor);
    const float e1 = (float)(s->initial_max_error * s->initial_max_error);
    const float e2 = (float)(s->final_max_error * s->final_max_error);

    auto fail = [&](mage_status st2) {
        (void)hipStreamSynchronize(st);
        buf.release();
        return st2;
    };
    if (hipMemsetAsync(d, 0, off, st) != hipSuccess ||
        hipMemcpyAsync(dposes, first_pose, 96, hipMemcpyHostToDevice, st) != hipSuccess)
        return fail(MAGE_EDEVICE);
    hipLaunchKernelGGL(trk_init, dim3(1), dim3(TT), 0, st, b, c, d_kp, d_desc, d_n, dposes, dmt, dil, dkf, rstatus);
    const float radius[3] = {s->search_radius, s->wider_search_radius, s->extra_wider_search_radius};
    // project: frame f's prediction is its own launch (first frame, first frame after a local BA);
    // otherwise the previous frame's trk_finish_project made it
    auto enqueue = [&](uint32_t f, bool project) -> mage_status {
        const mage_keypoint* fk = d_kp + (size_t)f * pitch;
        const uint8_t* fd = d_desc + 32ull * f * pitch;
        const uint32_t* nf = d_n + f;
        const size_t slot = (size_t)(f % BAND_SLOTS);
        mage_status rr;
        if (f == 1 || f % BAND_CHUNK == 0) {  // build the band indices of frames [f, next chunk)
            const uint32_t end = std::min(frames, (f / BAND_CHUNK + 1) * BAND_CHUNK);
            if ((rr = radius_band_index_launch(fk, fd, nf, (int64_t)pitch, end - f, bkeys + slot * pitch,
                                               bxy + 2 * slot * pitch, bdesc + 8 * slot * pitch, st)) != MAGE_OK)
                return rr;
        }
        if (project) launch("track.project", trk_project, dim3(1), dim3(TT), 0, st, b, c, (int)f, (const double*)dposes);
        for (int k = 0; k < 3; k++) {
            // passes 0 and 1 end with the fallback decision for the next (trk_weak's, in the pass's
            // last workgroup: one dependent launch less per pass)
            const RadiusFollow follow{&b.ctl->ns, b.ctl->exec, b.nq + k + 1, k, s->min_matches, s->small_match_ratio};
            rr = radius_match_indexed(b.qkp, k < 2 ? b.qpos : nullptr, b.qdesc, (int64_t)pitch, b.nq + k, fk, fd,
                                      (int64_t)pitch, nf, bkeys + slot * pitch, bxy + 2 * slot * pitch,
                                      bdesc + 8 * slot * pitch, 1, radius[k], s->max_hamming, s->min_hamming_difference,
                                      rscratch, b.m + (size_t)k * pitch, pitch, b.mn + k, rstatus, st,
                                      k < 2 ? &follow : nullptr);
            if (rr != MAGE_OK) return rr;
        }
        launch("track.gather", trk_gather, dim3(1), dim3(TT), 0, st, b, c, fk, (int)f, dmt);
        rr = mage_ba_pose_batch_device(1, b.pos3, b.r9, b.intr4, b.os1, b.pts1, b.uv1, b.info1, s->initial_steps,
                                       s->initial_huber, e1, b.pos3_o1, b.r9_o1, nullptr, b.out1, b.msq, nullptr,
                                       stream);
        if (rr != MAGE_OK) return rr;
        if (s->local_map_keyframes > 0) {
            launch("track.filter_lm", trk_filter_lm, dim3(1), dim3(TT), 0, st, b, c, nf);
            LocalMapArgs la{};
            la.qpos = b.lm_qpos;
            la.qoct = b.lm_qoct;
            la.qhide = b.lm_qhide;
            la.qdesc = b.lm_qdesc;
            la.nq = &b.ctl->lm_nq;
            la.q_cap = (uint32_t)qcap;
            la.tkp = fk;
            la.tdesc = fd;
            la.nt = nf;
            la.mask_words = b.lm_mask;
            la.radius = s->match_search_radius;
            la.max_dist = s->local_max_hamming;
            la.min_diff = s->local_min_hamming_difference;
            la.result = b.lm_res;
            la.status = b.lm_status;
            la.keys = bkeys + slot * pitch;
            if ((rr = local_map_match_launch(la, b.lm_scratch, st)) != MAGE_OK) return rr;
            launch("track.lm_assemble", trk_lm_assemble, dim3(1), dim3(TT), 0, st, b, fk);
        } else {
            launch("track.filter", trk_filter, dim3(1), dim3(TT), 0, st, b, c, nf);
        }
        rr = mage_ba_pose_batch_device(1, b.pos3_o1, b.r9_o1, b.intr4, b.os2, b.pts2, b.uv2, b.info2, s->final_steps,
                                       s->final_huber, e2, b.pos3_o2, b.r9_o2, nullptr, b.out2, b.msq + 1, nullptr,
                                       stream);
        if (rr != MAGE_OK) return rr;
        launch("track.finish", trk_finish_project, dim3(1), dim3(TT), 0, st, b, c, (int)f, fk, fd, nf, dposes, dil,
               dkf, rstatus, (int)(f + 1 < frames));
        return MAGE_OK;
    };
    if (ba_outliers)
        for (uint32_t f = 0; f < frames; f++) ba_outliers[f] = 0xFFFFFFFFu;
    if (!s->local_ba) {
        for (uint32_t f = 1; f < frames; f++)
            if ((r = enqueue(f, f == 1)) != MAGE_OK) return fail(r);
    } else {
        // Local BA after every new keyframe (MappingWorker; tracking.py local_bundle_adjust).  The
        // host stays up to two frames ahead; trk_finish of a keyframe frame sets ctl->halt (the
        // queued frames become no-ops) and reports it in mapped memory: the host drains the stream,
        // runs the BA on its copy of the keyframe ring, writes the ring back, clears the halt and
        // enqueues the following frames again.
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess) return fail(MAGE_EDEVICE);
        MappedBuffer prog;
        if ((r = prog.reserve(64)) != MAGE_OK) return fail(r);
        volatile uint32_t* hp = prog.host<volatile uint32_t>();
        hp[0] = 0;
        hp[1] = 0;
        b.prog = prog.device<uint32_t>();
        HostRing R;
        R.nk = NK;
        R.cap = (uint32_t)cap;
        R.acap = (uint32_t)acap;
        LocalBA L;
        PhaseClock prof;
        {
            const char* e = getenv("MAGE_TRACK_PROFILE");
            prof.on = e && *e == '1';
        }
        std::vector<uint8_t> changed(NK);
        uint32_t next = 1;
        bool need_project = true;  // the next enqueued frame makes its own prediction
        constexpr uint32_t DEPTH = 2;
        for (uint32_t f = 1; f < frames; f++) {
            while (next < frames && next <= f + DEPTH) {
                if ((r = enqueue(next, need_project)) != MAGE_OK) return fail(r);
                need_project = false;
                next++;
            }
            const auto t0 = std::chrono::steady_clock::now();
            while (hp[0] < f) {  // frame f done (trk_finish writes its index last)
                if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(50)) {
                    if (hipStreamSynchronize(st) != hipSuccess) return fail(MAGE_EDEVICE);
                    if (hp[0] < f) return fail(MAGE_EDEVICE);
                }
            }
            std::atomic_thread_fence(std::memory_order_acquire);
            if (hp[1] != f) continue;
            // a local BA: the halted frames drain, the ring comes to the host
            prof.start();
            if (hipStreamSynchronize(st) != hipSuccess) return fail(MAGE_EDEVICE);
            prof.mark("drain");
            Ctl hc;
            if (hipMemcpy(&hc, b.ctl, sizeof(Ctl), hipMemcpyDeviceToHost) != hipSuccess) return fail(MAGE_EDEVICE);
            R.first = hc.kf_first;
            R.count = hc.kf_count;
            for (uint32_t k = 0; k < NK; k++) {
                R.n[k] = hc.kf_n[k];
                R.id[k] = hc.kf_id[k];
                R.an[k] = hc.kf_an[k];
            }
            // the ring's fields are consecutive in the device block from kf_kp to kf_aalive
            const size_t mbytes = o_kfaa + acap * NK - o_kfkp;
            if (!R.mirror.resize(mbytes) || !R.zero.resize(1)) return fail(MAGE_ENOMEM);
            uint8_t* hm = R.mirror.data();
            R.kp = reinterpret_cast<mage_keypoint*>(hm + (o_kfkp - o_kfkp));
            R.pts = reinterpret_cast<float*>(hm + (o_kfp - o_kfkp));
            R.mvd = reinterpret_cast<float*>(hm + (o_kfv - o_kfkp));
            R.dmin = reinterpret_cast<float*>(hm + (o_kfdn - o_kfkp));
            R.dmax = reinterpret_cast<float*>(hm + (o_kfdx - o_kfkp));
            R.pose = reinterpret_cast<double*>(hm + (o_kfps - o_kfkp));
            R.ref = reinterpret_cast<uint32_t*>(hm + (o_kfr - o_kfkp));
            R.own = hm + (o_kfo - o_kfkp);
            R.assoc = reinterpret_cast<int4*>(hm + (o_kfa - o_kfkp));
            R.aalive = hm + (o_kfaa - o_kfkp);
            R.zero[0] = 0;
            if (hipMemcpyAsync(hm, d + o_kfkp, mbytes, hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess)
                return fail(MAGE_EDEVICE);
            prof.mark("ring D2H");
            std::fill(changed.begin(), changed.end(), 0);
            uint32_t nout = 0;
            if ((r = host_local_ba(R, c, L, dev, &nout, changed, prof)) != MAGE_OK) return fail(r);
            if (ba_outliers) ba_outliers[f] = nout;
            // write back the changed slots, the frame's pose (= its keyframe's) and clear the halt:
            // queued on the stream ahead of the next frames (the ring's host copy is not touched
            // again before the next window's drain)
            bool any = false;
            for (uint32_t k = 0; k < NK; k++) any = any || changed[k];
            // one copy of the mirror from the points on (kf_pts .. kf_aalive: every field the window
            // changes; the unchanged slots and the associations go back as they came)
            if (any && hipMemcpyAsync(d + o_kfp, R.mirror.data() + (o_kfp - o_kfkp), o_kfaa + acap * NK - o_kfp,
                                      hipMemcpyHostToDevice, st) != hipSuccess)
                return fail(MAGE_EDEVICE);
            const uint32_t newest = (R.first + R.count - 1) % NK;
            if (hipMemcpyAsync(dposes + 12ull * f, &R.pose[12 * newest], 96, hipMemcpyHostToDevice, st) != hipSuccess ||
                hipMemcpyAsync(&b.ctl->halt, R.zero.data(), 4, hipMemcpyHostToDevice, st) != hipSuccess)
                return fail(MAGE_EDEVICE);
            prof.mark("write-back");
            prof.flush();
            next = f + 1;
            need_project = true;
        }
        // the last window's write-back reads the pinned ring: done before the ring is freed
        if (hipStreamSynchronize(st) != hipSuccess) return fail(MAGE_EDEVICE);
    }
    if (hipGetLastError() != hipSuccess) return fail(MAGE_EDEVICE);
    uint32_t rst = 0, lst = 0;
    if (hipMemcpyAsync(poses, dposes, 96ull * frames, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(matches, dmt, 4ull * frames, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(inliers, dil, 4ull * frames, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(keyframe, dkf, frames, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(&rst, rstatus, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(&lst, b.lm_status, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return fail(MAGE_EDEVICE);
    buf.release();
    MAGE_REQUIRE(!(rst & 1u), MAGE_ECAPACITY, "a frame has more than 4096 keypoints");
    MAGE_REQUIRE(!(rst & 2u), MAGE_ECAPACITY, "a frame's keypoint count exceeds the frame pitch");
    MAGE_REQUIRE(lst == 0, MAGE_ECAPACITY, "local-map search: a frame has more than 4096 keypoints");
    return MAGE_OK;
}
