// mage.hpp — header-only C++ facades over the C-ABI (include/mage_hot.h) with the reference's
// class shapes, so MAGE-SLAM's L3 callers (ImageAnalyzer, MapInitialization, BundleAdjust,
// TrackLocalMap) can switch by swapping the type they hold.  No OpenCV / Eigen / g2o types:
// keypoints are cv::KeyPoint-layout records, descriptors 32-byte rows, matrices plain floats
// in the reference's layouts (Eigen column-major rotations).  Errors throw like the reference:
// MAGE_EINVAL -> std::invalid_argument (CV_Assert), everything else -> mage::hot::Error.
#pragma once

#include <algorithm>
#include <array>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "../mage_hot.h"

namespace mage {
namespace hot {

struct Error : std::runtime_error {
    mage_status status;
    Error(mage_status s, const std::string& m) : std::runtime_error(m), status(s) {}
};

inline void check(mage_status s)
{
    if (s == MAGE_OK) return;
    std::string msg = mage_last_error();
    if (s == MAGE_EINVAL) throw std::invalid_argument(msg);
    throw Error(s, msg);
}

using KeyPoint = mage_keypoint;
using DMatch = mage_dmatch;
using Descriptor = std::array<uint8_t, 32>;  // ORBDescriptor (ORBDescriptor.h:14-133)

// OrbDetector (Core/MAGESLAM/Source/Image/OpenCVModified.h:64-173).
class OrbDetector {
public:
    OrbDetector(unsigned gaussianKernelSize, unsigned nfeatures, float scaleFactor, unsigned nlevels,
                unsigned patchSize, unsigned fastThreshold, bool useOrientation, float featureFactorANMS,
                float featureStrengthANMS, int strongResponseANMS, float minRobustFactor,
                float maxRobustFactor, int numCellsX, int numCellsY, int device = 0)
        : m_settings{gaussianKernelSize, nfeatures, scaleFactor, nlevels, patchSize, fastThreshold,
                     useOrientation ? 1 : 0, featureFactorANMS, featureStrengthANMS, strongResponseANMS,
                     minRobustFactor, maxRobustFactor, numCellsX, numCellsY}
    {
        check(mage_orb_create(&m_settings, device, &m_handle));
    }
    ~OrbDetector() { mage_orb_destroy(m_handle); }
    OrbDetector(const OrbDetector&) = delete;
    OrbDetector& operator=(const OrbDetector&) = delete;

    // DetectAndCompute(thread_memory, ImageData&, const cv::Mat&): the ImageData becomes the two
    // output vectors; `capacity` is ImageData's maxFeatures (defaults to nfeatures).
    void DetectAndCompute(const uint8_t* gray, int width, int height, int stride,
                          std::vector<KeyPoint>& keypoints, std::vector<Descriptor>& descriptors,
                          uint32_t capacity = 0)
    {
        const uint32_t cap = capacity ? capacity : m_settings.nfeatures;
        keypoints.resize(cap);
        descriptors.resize(cap);
        uint32_t n = 0;
        check(mage_orb_detect_and_compute(m_handle, gray, width, height, stride, keypoints.data(),
                                          descriptors.empty() ? nullptr : descriptors.front().data(), cap, &n));
        keypoints.resize(n);
        descriptors.resize(n);
    }

    mage_orb* handle() const { return m_handle; }

private:
    mage_orb_settings m_settings;
    mage_orb* m_handle = nullptr;
};

// GetDescriptorDistance (Core/MAGESLAM/Source/Tracking/FeatureMatcher.cpp:453-504).
inline int GetDescriptorDistance(const Descriptor& a, const Descriptor& b)
{
    return mage_hamming_distance(a.data(), b.data());
}

// Match (FeatureMatcher.cpp:61-190) with descriptor rows and boolean masks instead of
// AnalyzedImage; returns the match count and fills goodMatches (ascending A index).
inline unsigned Match(const std::vector<Descriptor>& a, const std::vector<Descriptor>& b,
                      const std::vector<bool>& maskA, const std::vector<bool>& maskB, int maxHammingDist,
                      int minHammingDifference, std::vector<DMatch>& goodMatches)
{
    std::vector<uint8_t> ma(maskA.begin(), maskA.end()), mb(maskB.begin(), maskB.end());
    goodMatches.resize(a.size());
    uint32_t n = 0;
    check(mage_hamming_match(a.empty() ? nullptr : a.front().data(), (uint32_t)a.size(), ma.empty() ? nullptr : ma.data(),
                             b.empty() ? nullptr : b.front().data(), (uint32_t)b.size(), mb.empty() ? nullptr : mb.data(),
                             maxHammingDist, minHammingDifference, goodMatches.data(), (uint32_t)goodMatches.size(), &n));
    goodMatches.resize(n);
    return n;
}

// RadiusMatch (FeatureMatcher.cpp:294-378): the target KeypointSpatialIndex is built on the device
// from targetKeypoints, so callers pass the keypoints instead of the index.  Optional position
// overrides and masks (nullptr = none).  Clears and fills goodMatches (query order).
inline unsigned RadiusMatch(const std::vector<KeyPoint>& queryKeypoints, const std::vector<float>* queryPositionOverrides,
                            const std::vector<bool>* queryKeypointsMask, const std::vector<Descriptor>& queryDescriptors,
                            const std::vector<KeyPoint>& targetKeypoints, const std::vector<bool>* targetKeypointsMask,
                            const std::vector<Descriptor>& targetDescriptors, float radius, int maxHammingDist,
                            int minHammingDifference, std::vector<DMatch>& goodMatches)
{
    std::vector<uint8_t> qm, tm;
    if (queryKeypointsMask) qm.assign(queryKeypointsMask->begin(), queryKeypointsMask->end());
    if (targetKeypointsMask) tm.assign(targetKeypointsMask->begin(), targetKeypointsMask->end());
    goodMatches.resize(queryKeypoints.size());
    uint32_t n = 0;
    check(mage_radius_match(queryKeypoints.data(), queryPositionOverrides ? queryPositionOverrides->data() : nullptr,
                            queryKeypointsMask ? qm.data() : nullptr,
                            queryDescriptors.empty() ? nullptr : queryDescriptors.front().data(), (uint32_t)queryKeypoints.size(),
                            targetKeypoints.data(), targetKeypointsMask ? tm.data() : nullptr,
                            targetDescriptors.empty() ? nullptr : targetDescriptors.front().data(),
                            (uint32_t)targetKeypoints.size(), radius, maxHammingDist, minHammingDifference,
                            goodMatches.data(), (uint32_t)goodMatches.size(), &n));
    goodMatches.resize(n);
    return n;
}

// TrackLocalMap's per-map-point matching loop (TrackLocalMap.cpp:175-256): projected map points in
// order (positions x, y interleaved; octaves; descriptors; the keypoint to hide for a
// pose-estimation outlier point, -1 otherwise) against a frame's keypoints; unassociatedMask is
// updated like the reference's (a match takes its keypoint).  Returns the keypoint per point or -1.
inline std::vector<int32_t> LocalMapMatch(const std::vector<float>& positions, const std::vector<int32_t>& octaves,
                                          const std::vector<Descriptor>& descriptors, const std::vector<int32_t>& hidden,
                                          const std::vector<KeyPoint>& targetKeypoints,
                                          const std::vector<Descriptor>& targetDescriptors,
                                          std::vector<bool>& unassociatedMask, float radius, int maxHammingDist,
                                          int minHammingDifference, int device = 0)
{
    const uint32_t n = (uint32_t)octaves.size();
    std::vector<uint8_t> mask(unassociatedMask.begin(), unassociatedMask.end());
    std::vector<int32_t> result(n, -1);
    check(mage_local_map_match(positions.data(), octaves.data(), descriptors.empty() ? nullptr : descriptors.front().data(),
                               hidden.empty() ? nullptr : hidden.data(), n, targetKeypoints.data(),
                               targetDescriptors.empty() ? nullptr : targetDescriptors.front().data(),
                               (uint32_t)targetKeypoints.size(), mask.data(), radius, maxHammingDist,
                               minHammingDifference, result.data(), device));
    for (size_t t = 0; t < mask.size(); t++) unassociatedMask[t] = mask[t] != 0;
    return result;
}

// OnlineBow vocabulary tree on the device (OnlineBow.cpp:289-311 FindLeafNode; nodes as CreateTree
// builds them: node i's descriptor, children in childrenIDs order, root 0).
class OnlineBowTree {
public:
    OnlineBowTree(const std::vector<Descriptor>& nodes, const std::vector<uint32_t>& childStart,
                  const std::vector<uint32_t>& children, int device = 0)
    {
        check(mage_bow_create(nodes.empty() ? nullptr : nodes.front().data(), childStart.data(),
                              children.empty() ? nullptr : children.data(), (uint32_t)nodes.size(), device, &m_handle));
    }
    // OnlineBow::CreateTree (OnlineBow.cpp:325-337) over training descriptors on the GPU
    // (BagOfWordsSettings TrainingTreeLevels / TrainingTreeBranchingFactor / MaxTrainingIteration)
    explicit OnlineBowTree(const std::vector<Descriptor>& training, unsigned levels = 2, unsigned branching = 6,
                           unsigned maxIterations = 12, int device = 0)
    {
        check(mage_bow_train(training.empty() ? nullptr : training.front().data(), (uint32_t)training.size(), levels,
                             branching, maxIterations, device, &m_handle));
    }
    ~OnlineBowTree() { mage_bow_destroy(m_handle); }
    OnlineBowTree(const OnlineBowTree&) = delete;
    OnlineBowTree& operator=(const OnlineBowTree&) = delete;
    ptrdiff_t FindLeafNode(const Descriptor& d) const
    {
        uint32_t leaf = 0;
        check(mage_bow_find_leaves(m_handle, d.data(), 1, &leaf));
        return (ptrdiff_t)leaf;
    }
    mage_bow* handle() const { return m_handle; }

private:
    mage_bow* m_handle = nullptr;
};

// IndexedMatch (FeatureMatcher.cpp:192-292) with the BoW candidate lists of `tree` (what
// OnlineBowFeatureMatcher / OnlineBow::QueryFeatures return); masks as in Match.
inline unsigned IndexedMatch(const OnlineBowTree& tree, const std::vector<Descriptor>& a, const std::vector<Descriptor>& b,
                             const std::vector<bool>& maskA, const std::vector<bool>& maskB, int maxHammingDist,
                             int minHammingDifference, std::vector<DMatch>& goodMatches)
{
    std::vector<uint8_t> ma(maskA.begin(), maskA.end()), mb(maskB.begin(), maskB.end());
    goodMatches.resize(a.size());
    uint32_t n = 0;
    check(mage_indexed_match(tree.handle(), a.empty() ? nullptr : a.front().data(), (uint32_t)a.size(),
                             ma.empty() ? nullptr : ma.data(), b.empty() ? nullptr : b.front().data(), (uint32_t)b.size(),
                             mb.empty() ? nullptr : mb.data(), maxHammingDist, minHammingDifference, goodMatches.data(),
                             (uint32_t)goodMatches.size(), &n));
    goodMatches.resize(n);
    return n;
}

struct BundlerParameters {
    bool ArePointsFixed{false};
};

// BundlerLib (Dependencies/BundlerLib/Include/BundlerLib.h:20-66).  The Set* calls buffer on
// the host; the problem is uploaded at the first StepBundleAdjustment.
class BundlerLib {
public:
    explicit BundlerLib(const BundlerParameters& params, int device = 0) : m_params(params)
    {
        check(mage_ba_create(params.ArePointsFixed ? 1 : 0, device, &m_handle));
    }
    ~BundlerLib() { mage_ba_destroy(m_handle); }
    BundlerLib(const BundlerLib&) = delete;
    BundlerLib& operator=(const BundlerLib&) = delete;

    void AllocateCameras(size_t count)
    {
        m_pos.assign(3 * count, 0.f);
        m_rot.assign(9 * count, 0.f);
        m_intr.assign(4 * count, 0.f);
        m_fixed.assign(count, 0);
        m_dirty = true;
    }
    // position: view-space t (3); orientation: Eigen::Map<const Matrix3f> data (column-major 9);
    // intrinsics: {cx, cy, fx, fy}
    void SetCameraPose(size_t idx, const float* position, const float* orientationColMajor, const float* intrinsics,
                       bool isFixed)
    {
        std::copy(position, position + 3, &m_pos[3 * idx]);
        std::copy(orientationColMajor, orientationColMajor + 9, &m_rot[9 * idx]);
        std::copy(intrinsics, intrinsics + 4, &m_intr[4 * idx]);
        m_fixed[idx] = isFixed ? 1 : 0;
        m_dirty = true;
    }
    void FixCameraPose(size_t idx, bool value)
    {
        m_fixed[idx] = value ? 1 : 0;
        if (!m_dirty) check(mage_ba_fix_camera(m_handle, (uint32_t)idx, value ? 1 : 0));
    }
    void AllocateMapPoints(size_t count)
    {
        m_points.assign(3 * count, 0.f);
        m_dirty = true;
    }
    void SetMapPoint(size_t idx, const float* point)
    {
        std::copy(point, point + 3, &m_points[3 * idx]);
        m_dirty = true;
    }
    void AllocateObservations(size_t count)
    {
        m_uv.assign(2 * count, 0.f);
        m_cam.assign(count, 0);
        m_pt.assign(count, 0);
        m_info.assign(count, 0.f);
        m_dirty = true;
    }
    void SetObservation(size_t idx, const float* position, size_t cameraIndex, size_t mapPointIndex,
                        float informationMatrixScalar)
    {
        m_uv[2 * idx] = position[0];
        m_uv[2 * idx + 1] = position[1];
        m_cam[idx] = (uint32_t)cameraIndex;
        m_pt[idx] = (uint32_t)mapPointIndex;
        m_info[idx] = informationMatrixScalar;
        m_dirty = true;
    }
    // Tether constraints (BundlerLib.cpp:229-257, 311-350); quaternions are (x, y, z, w).
    void AllocateFixedDistanceConstraints(size_t count) { m_teth[MAGE_TETHER_DISTANCE].resize(count); m_dirty = true; }
    void SetFixedDistanceConstraint(size_t idx, size_t cameraIndex1, size_t cameraIndex2, float distance = 1.0f,
                                    float weight = 1.0f)
    {
        m_teth[MAGE_TETHER_DISTANCE][idx] = {(uint32_t)cameraIndex1, (uint32_t)cameraIndex2, weight, {distance}};
        m_dirty = true;
    }
    void AllocateRelativeRotationConstraints(size_t count) { m_teth[MAGE_TETHER_ROTATION].resize(count); m_dirty = true; }
    void SetRelativeRotationConstraint(size_t idx, size_t cameraIndex1, size_t cameraIndex2, const float* deltaRotationXYZW,
                                       float weight = 1.0f)
    {
        Tether t{(uint32_t)cameraIndex1, (uint32_t)cameraIndex2, weight, {}};
        std::copy(deltaRotationXYZW, deltaRotationXYZW + 4, t.params);
        m_teth[MAGE_TETHER_ROTATION][idx] = t;
        m_dirty = true;
    }
    void AllocateRelativeTransformConstraints(size_t count) { m_teth[MAGE_TETHER_TRANSFORM].resize(count); m_dirty = true; }
    void SetRelativeTransformConstraint(size_t idx, size_t cameraIndex1, size_t cameraIndex2, const float* deltaPosition,
                                        const float* deltaRotationXYZW, float weight)
    {
        Tether t{(uint32_t)cameraIndex1, (uint32_t)cameraIndex2, weight, {}};
        std::copy(deltaPosition, deltaPosition + 3, t.params);
        std::copy(deltaRotationXYZW, deltaRotationXYZW + 4, t.params + 3);
        m_teth[MAGE_TETHER_TRANSFORM][idx] = t;
        m_dirty = true;
    }
    void SetCurrentLambda(float userLambda) { check(mage_ba_set_lambda(m_handle, userLambda)); }
    float GetCurrentLambda() const
    {
        float l = 0;
        check(mage_ba_get_lambda(m_handle, &l));
        return l;
    }
    // Runs one LM iteration per Huber width; returns the mean squared error of the kept edges
    // and appends the outlier observation indices.
    float StepBundleAdjustment(const std::vector<float>& huberWidthPerIteration, float maxErrorSquare,
                               std::vector<unsigned>& outliers)
    {
        upload();
        std::vector<uint32_t> out(std::max<size_t>(m_cam.size(), 1));
        uint32_t n = 0;
        float ms = 0;
        check(mage_ba_step(m_handle, huberWidthPerIteration.data(), (uint32_t)huberWidthPerIteration.size(),
                           maxErrorSquare, out.data(), (uint32_t)out.size(), &n, &ms));
        outliers.insert(outliers.end(), out.begin(), out.begin() + n);
        return ms;
    }
    void GetPose(size_t idx, float* position, float* orientationColMajor) const
    {
        std::vector<float> pos(m_pos.size()), rot(m_rot.size());
        check(mage_ba_get_poses(m_handle, pos.data(), rot.data()));
        std::copy(&pos[3 * idx], &pos[3 * idx] + 3, position);
        std::copy(&rot[9 * idx], &rot[9 * idx] + 9, orientationColMajor);
    }
    void GetPoint(size_t idx, float* position) const
    {
        std::vector<float> xyz(m_points.size());
        check(mage_ba_get_points(m_handle, xyz.data()));
        std::copy(&xyz[3 * idx], &xyz[3 * idx] + 3, position);
    }

private:
    void upload()
    {
        if (!m_dirty) return;
        check(mage_ba_set_cameras(m_handle, (uint32_t)m_fixed.size(), m_pos.data(), m_rot.data(), m_intr.data(),
                                  m_fixed.data()));
        check(mage_ba_set_points(m_handle, (uint32_t)(m_points.size() / 3), m_points.data()));
        check(mage_ba_set_observations(m_handle, (uint32_t)m_cam.size(), m_uv.data(), m_cam.data(), m_pt.data(),
                                       m_info.data()));
        static const int stride[3] = {1, 4, 7};
        for (uint32_t kind = 0; kind < 3; kind++) {
            const auto& v = m_teth[kind];
            std::vector<uint32_t> c1(v.size()), c2(v.size());
            std::vector<float> params(v.size() * stride[kind]), weight(v.size());
            for (size_t i = 0; i < v.size(); i++) {
                c1[i] = v[i].cam1;
                c2[i] = v[i].cam2;
                weight[i] = v[i].weight;
                std::copy(v[i].params, v[i].params + stride[kind], &params[i * stride[kind]]);
            }
            check(mage_ba_set_tethers(m_handle, kind, (uint32_t)v.size(), c1.data(), c2.data(), params.data(),
                                      weight.data()));
        }
        m_dirty = false;
    }

    struct Tether {
        uint32_t cam1, cam2;
        float weight;
        float params[7];
    };
    std::vector<Tether> m_teth[3];

    BundlerParameters m_params;
    mage_ba* m_handle = nullptr;
    bool m_dirty = true;
    std::vector<float> m_pos, m_rot, m_intr, m_points, m_uv, m_info;
    std::vector<uint8_t> m_fixed;
    std::vector<uint32_t> m_cam, m_pt;
};

}  // namespace hot
}  // namespace mage
