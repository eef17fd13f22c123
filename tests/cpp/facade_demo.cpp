// facade_demo.cpp — drives the C++ facades (include/mage/mage.hpp) the way the reference's
// callers drive OrbDetector / Match / BundlerLib.  Usage: facade_demo <gray.raw> <w> <h> <out.bin>
// Writes: u32 n, n keypoints (28 B), n descriptors (32 B), u32 self-matches, float BA mean_sq,
// u32 radius self-matches (radius 2 px).
// Exits 3 if no GPU is usable (MAGE_EDEVICE), so the CPU test suite can still run it.
#include <cstdio>
#include <fstream>
#include <iostream>
#include <vector>

#include "mage/mage.hpp"

int main(int argc, char** argv)
{
    if (argc < 5) return 2;
    const int w = std::atoi(argv[2]), h = std::atoi(argv[3]);
    std::vector<uint8_t> img((size_t)w * h);
    std::ifstream(argv[1], std::ios::binary).read((char*)img.data(), (std::streamsize)img.size());
    try {
        // FeatureExtractorSettings defaults (MageSettings.h:151-167) with 2000 features
        mage::hot::OrbDetector det(7, 2000, 1.5f, 1, 15, 4, false, 1.5f, 0.9f, 20, 1.1f, 2.0f, 32, 32);
        std::vector<mage::hot::KeyPoint> kps;
        std::vector<mage::hot::Descriptor> desc;
        det.DetectAndCompute(img.data(), w, h, w, kps, desc);
        std::vector<mage::hot::DMatch> matches;
        const unsigned nm = mage::hot::Match(desc, desc, std::vector<bool>(desc.size(), true),
                                             std::vector<bool>(desc.size(), true), 30, 1, matches);
        // a 3-camera, 40-point BA through the BundlerLib facade
        mage::hot::BundlerLib ba(mage::hot::BundlerParameters{});
        ba.AllocateCameras(3);
        const float I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, K[4] = {320, 240, 500, 500};
        for (int c = 0; c < 3; c++) {
            const float t[3] = {-0.2f * c, 0.f, 0.f};
            ba.SetCameraPose(c, t, I, K, c == 0);
        }
        ba.AllocateMapPoints(40);
        ba.AllocateObservations(120);
        for (int p = 0; p < 40; p++) {
            const float X[3] = {-1.f + 0.05f * p, 0.3f * ((p % 5) - 2), 4.f + 0.1f * (p % 7)};
            const float Xn[3] = {X[0] + 0.01f, X[1] - 0.01f, X[2] + 0.02f};
            ba.SetMapPoint(p, Xn);
            for (int c = 0; c < 3; c++) {
                const float x = X[0] - 0.2f * c;
                const float uv[2] = {500.f * x / X[2] + 320.f, 500.f * X[1] / X[2] + 240.f};
                ba.SetObservation(3 * p + c, uv, c, p, 1.0f);
            }
        }
        ba.AllocateFixedDistanceConstraints(1);  // cameras 1 and 2 are 0.2 apart
        ba.SetFixedDistanceConstraint(0, 1, 2, 0.2f, 50.f);
        const float qI[4] = {0, 0, 0, 1}, d12[3] = {-0.2f, 0.f, 0.f};
        ba.AllocateRelativeTransformConstraints(1);
        ba.SetRelativeTransformConstraint(0, 1, 2, d12, qI, 10.f);
        // a two-level tree whose nodes are the first keypoints' descriptors
        std::vector<mage::hot::Descriptor> nodes(desc.begin(), desc.begin() + 7);
        const std::vector<uint32_t> childStart = {0, 3, 6, 6, 6, 6, 6, 6}, children = {1, 2, 3, 4, 5, 6};
        mage::hot::OnlineBowTree tree(nodes, childStart, children);
        std::vector<mage::hot::DMatch> imatches;
        const unsigned ni = mage::hot::IndexedMatch(tree, desc, desc, std::vector<bool>(desc.size(), true),
                                                    std::vector<bool>(desc.size(), true), 30, 1, imatches);
        // OnlineBow::CreateTree over the frame's descriptors (defaults), then IndexedMatch through it
        mage::hot::OnlineBowTree trained(desc);
        std::vector<mage::hot::DMatch> tmatches;
        const unsigned nt = mage::hot::IndexedMatch(trained, desc, desc, std::vector<bool>(desc.size(), true),
                                                    std::vector<bool>(desc.size(), true), 30, 1, tmatches);
        std::vector<mage::hot::DMatch> rmatches;
        const unsigned nr = mage::hot::RadiusMatch(kps, nullptr, nullptr, desc, kps, nullptr, desc, 2.0f, 30, 1, rmatches);
        // TrackLocalMap's per-map-point matching: the frame's own keypoints as projected map points
        std::vector<float> lpos;
        std::vector<int32_t> loct;
        for (const auto& k : kps) {
            lpos.push_back(k.x);
            lpos.push_back(k.y);
            loct.push_back(k.octave);
        }
        std::vector<bool> unassociated(kps.size(), true);
        const std::vector<int32_t> lres =
            mage::hot::LocalMapMatch(lpos, loct, desc, {}, kps, desc, unassociated, 2.0f, 30, 1);
        uint32_t nl = 0;
        for (int32_t v : lres) nl += v >= 0;
        std::vector<unsigned> outliers;
        float ms = 0;
        for (int it = 0; it < 5; it++) ms = ba.StepBundleAdjustment({1.8f}, 1e6f, outliers);
        std::ofstream o(argv[4], std::ios::binary);
        uint32_t n = (uint32_t)kps.size();
        o.write((const char*)&n, 4);
        o.write((const char*)kps.data(), (std::streamsize)(28 * n));
        o.write((const char*)desc.data(), (std::streamsize)(32 * n));
        o.write((const char*)&nm, 4);
        o.write((const char*)&ms, 4);
        o.write((const char*)&nr, 4);
        o.write((const char*)&ni, 4);
        o.write((const char*)&nt, 4);
        o.write((const char*)&nl, 4);
        o.write((const char*)lres.data(), (std::streamsize)(4 * lres.size()));
        std::cout << "keypoints " << n << " self-matches " << nm << " ba_mean_sq " << ms << "\n";
    } catch (const mage::hot::Error& e) {
        std::cerr << "mage error: " << e.what() << "\n";
        return e.status == MAGE_EDEVICE ? 3 : 1;
    }
    return 0;
}
