// common.hpp — shared host/device helpers for the MI355X hot-path library (libmage_hot.so).
#pragma once

#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wc++20-extensions"  // inside the ROCm header's templates
#include <hip/hip_ext.h>
#pragma clang diagnostic pop
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/mage_hot.h"

namespace mage {

// Thread-local last error (mage_last_error()).
void set_error(const std::string& msg);
const char* last_error();

#define MAGE_HIP(expr)                                                                      \
    do {                                                                                    \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess) {                                                             \
            ::mage::set_error(std::string(#expr " failed: ") + hipGetErrorString(_e) +     \
                              " at " + __FILE__ + ":" + std::to_string(__LINE__));          \
            return MAGE_EDEVICE;                                                            \
        }                                                                                   \
    } while (0)

#define MAGE_REQUIRE(cond, code, msg)                                                       \
    do {                                                                                    \
        if (!(cond)) {                                                                      \
            ::mage::set_error(msg);                                                         \
            return code;                                                                    \
        }                                                                                   \
    } while (0)

// Selects `device` and verifies it is a gfx950 part; returns MAGE_OK or MAGE_EDEVICE.
mage_status bind_device(int device);

// Block cache for allocations that are created and dropped per task (BundlerLib per local-BA
// window, MappingWorker's MakeBundler): hipFree / hipHostFree synchronise the whole device and cost
// ~0.1 ms each.  Only blocks whose owner has synchronised every stream that used them are retired
// here (retire_*), so a block handed out again is idle; any buffer's first allocation may take one.
// Kind 0: device memory, 1: page-locked host memory, 2: mapped (coherent) host memory.  Thread safe.
void* pool_take(int kind, size_t n, size_t* got);
void pool_retire(int kind, void* p, size_t bytes);
// Frees the idle blocks of `kind` (-1: every kind) on `device` (-1: every device) for real;
// returns the bytes freed.  The buffers below call it when an allocation fails and retry once.
size_t pool_trim(int kind, int device);
inline int current_device()
{
    int d = 0;
    return hipGetDevice(&d) == hipSuccess ? d : -1;
}
hipStream_t stream_take();  // an idle retired stream of the current device, or nullptr
void stream_retire(hipStream_t s);

// Grow-only device buffer.
struct DeviceBuffer {
    void* ptr = nullptr;
    size_t bytes = 0;
    mage_status reserve(size_t n) {
        if (n <= bytes) return MAGE_OK;
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        bytes = 0;
        if ((ptr = pool_take(0, n, &bytes)) != nullptr) return MAGE_OK;
        if (hipMalloc(&ptr, n) != hipSuccess &&
            (pool_trim(0, current_device()) == 0 || hipMalloc(&ptr, n) != hipSuccess)) {
            ptr = nullptr;
            set_error("hipMalloc of " + std::to_string(n) + " bytes failed");
            return MAGE_ENOMEM;
        }
        bytes = n;
        return MAGE_OK;
    }
    void release() {
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        bytes = 0;
    }
    // release into the block cache: the caller has synchronised every stream that used the buffer
    void retire() {
        if (ptr) pool_retire(0, ptr, bytes);
        ptr = nullptr;
        bytes = 0;
    }
    template <typename T>
    T* as() const {
        return static_cast<T*>(ptr);
    }
};

// Page-locked host staging for the synchronous host-buffer entry points: the caller's inputs are
// packed at their device offsets and moved with ONE copy each way (a per-array hipMemcpyAsync costs
// ~5 us of DMA setup each, which dominated the per-frame tracker calls)
struct PinnedBuffer {
    void* ptr = nullptr;
    size_t bytes = 0;
    mage_status reserve(size_t n) {
        if (n <= bytes) return MAGE_OK;
        if (ptr) (void)hipHostFree(ptr);
        ptr = nullptr;
        bytes = 0;
        if ((ptr = pool_take(1, n, &bytes)) != nullptr) return MAGE_OK;
        if (hipHostMalloc(&ptr, n, hipHostMallocDefault) != hipSuccess &&
            (pool_trim(1, current_device()) == 0 || hipHostMalloc(&ptr, n, hipHostMallocDefault) != hipSuccess)) {
            ptr = nullptr;
            set_error("hipHostMalloc of " + std::to_string(n) + " bytes failed");
            return MAGE_ENOMEM;
        }
        bytes = n;
        return MAGE_OK;
    }
    void release() {
        if (ptr) (void)hipHostFree(ptr);
        ptr = nullptr;
        bytes = 0;
    }
    void retire() {
        if (ptr) pool_retire(1, ptr, bytes);
        ptr = nullptr;
        bytes = 0;
    }
    template <typename T>
    T* as() const {
        return static_cast<T*>(ptr);
    }
};

// Host memory that kernels write directly (pinned, coherent, mapped): results a host decision
// needs right after a completion wait arrive without a D2H copy + stream sync.
struct MappedBuffer {
    void* ptr = nullptr;  // host view
    void* dev = nullptr;  // device view
    size_t bytes = 0;
    mage_status reserve(size_t n) {
        if (n <= bytes) return MAGE_OK;
        release();
        if ((ptr = pool_take(2, n, &bytes)) != nullptr) {
            if (hipHostGetDevicePointer(&dev, ptr, 0) == hipSuccess) return MAGE_OK;
            pool_retire(2, ptr, bytes);
            ptr = nullptr;
            bytes = 0;
        }
        auto alloc = [&] { return hipHostMalloc(&ptr, n, hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess; };
        if (!alloc() && (ptr = nullptr, pool_trim(2, current_device()) == 0 || !alloc())) ptr = nullptr;
        if (!ptr || hipHostGetDevicePointer(&dev, ptr, 0) != hipSuccess) {
            release();
            set_error("mapped hipHostMalloc of " + std::to_string(n) + " bytes failed");
            return MAGE_ENOMEM;
        }
        bytes = n;
        return MAGE_OK;
    }
    void release() {
        if (ptr) (void)hipHostFree(ptr);
        ptr = dev = nullptr;
        bytes = 0;
    }
    void retire() {
        if (ptr) pool_retire(2, ptr, bytes);
        ptr = dev = nullptr;
        bytes = 0;
    }
    template <typename T>
    T* host() const {
        return static_cast<T*>(ptr);
    }
    template <typename T>
    T* device() const {
        return static_cast<T*>(dev);
    }
};

// Scratch of a synchronous host-buffer entry point (device staging, pinned staging, a private
// stream), one per (calling thread, device, entry point): concurrent callers never share buffers
// or a stream.  The reference calls these paths from several threads at once — both stereo
// frames' OrbFeatureDetector::Process (UndistortKeypoints) run in parallel
// (ImageAnalyzer.cpp:160-216) and the matchers take a per-thread thread_memory.  Released when the
// thread exits.
enum ScratchSlot : int { SCRATCH_RADIUS = 0, SCRATCH_POSE = 1, SCRATCH_UNDISTORT = 2, SCRATCH_MATCH = 3, SCRATCH_LOCALMAP = 4 };
struct HostScratch {
    DeviceBuffer buf, aux;
    PinnedBuffer host;
    hipStream_t st = nullptr;
    HostScratch() = default;
    HostScratch(const HostScratch&) = delete;
    HostScratch& operator=(const HostScratch&) = delete;
    ~HostScratch();
};
// The calling thread's scratch for `slot` on `device` (already bound by bind_device), with its
// stream created; nullptr (and the error set) if the stream cannot be created.
HostScratch* host_scratch(int device, ScratchSlot slot);

// Device scratch private to one (calling thread, current device, stream, slot) and at least
// `bytes` long: kernels on different streams may run concurrently, so they never share it, and a
// thread that grows its buffer (sync of the stream, then free) can only free memory its own
// launches used — never a pointer another thread is about to launch on.  Freed at thread exit or
// when the stream's HostScratch is destroyed.  nullptr (error set) if the allocation fails.
enum StreamSlot : int { STREAM_MATCH_ROWS = 0, STREAM_MATCH_STATUS = 1, STREAM_RESIZE_TABLES = 2 };
void* stream_scratch(hipStream_t st, StreamSlot slot, size_t bytes);

constexpr int kWave = 64;

// TrackLocalMap's sequential per-map-point matching (localmap.hip): queries in order (projected
// position, octave, descriptor, hidden keypoint or -1), the frame's keypoints, the unassociated
// mask as bit words (bit t = keypoint t available; updated in place), result[q] = keypoint or -1.
// Counts are device words (q_cap / 4096 bound them); status bits report bad counts.
struct LocalMapArgs {
    const float* qpos;
    const int* qoct;
    const int* qhide;
    const uint8_t* qdesc;
    const uint32_t* nq;
    uint32_t q_cap;
    const mage_keypoint* tkp;
    const uint8_t* tdesc;
    const uint32_t* nt;
    uint32_t* mask_words;
    float radius;
    int max_dist, min_diff;
    int* result;
    uint32_t* status;
    const unsigned long long* keys;  // optional: the frame's band index, sorted (radius_band_index_launch)
};
size_t local_map_scratch_bytes(uint32_t q_cap);
mage_status local_map_match_launch(const LocalMapArgs& a, void* scratch, hipStream_t st);

// RadiusMatch's band index built once per target set (radius.hip): keys sorted ascending (8 B),
// positions (2 floats) and descriptors (8 words) in key order, target_pitch entries per set; and
// mage_radius_match_batch_device against sets indexed that way (same results).
mage_status radius_band_index_launch(const mage_keypoint* d_target_kp, const uint8_t* d_target_desc,
                                     const uint32_t* d_n_target, int64_t target_pitch, uint32_t sets,
                                     unsigned long long* d_keys, float* d_xy, uint32_t* d_desc, hipStream_t st);
// The tracker's fallback decision after a RadiusMatch pass (PoseEstimator.cpp:439-607: a wider
// pass runs when this one ran and is weak): once the pass's match count n is final, exec[k + 1] =
// exec[k] && (n < min_matches || n / ns < ratio) and *nq_next = exec[k + 1] ? ns : 0 (single pair).
struct RadiusFollow {
    const uint32_t* ns;
    uint32_t* exec;
    uint32_t* nq_next;
    int k;
    uint32_t min_matches;
    double ratio;
};
mage_status radius_match_indexed(const mage_keypoint* d_query_kp, const float* d_query_pos, const uint8_t* d_query_desc,
                                 int64_t query_pitch, const uint32_t* d_n_query, const mage_keypoint* d_target_kp,
                                 const uint8_t* d_target_desc, int64_t target_pitch, const uint32_t* d_n_target,
                                 const unsigned long long* d_keys, const float* d_xy, const uint32_t* d_desc,
                                 uint32_t pairs, float radius, int32_t max_distance, int32_t min_difference,
                                 int32_t* d_scratch, mage_dmatch* d_out, uint32_t cap, uint32_t* d_n, uint32_t* d_status,
                                 hipStream_t st, const RadiusFollow* follow = nullptr);

// cv::resize(INTER_LINEAR) 8UC1 of one device image (orb.hip, the pyramid's resize_linear_kernel);
// asynchronous on st.
mage_status resize_linear_device(const uint8_t* src, int sw, int sh, int sstride, uint8_t* dst, int dw, int dh,
                                 int dstride, hipStream_t st);

// Optional per-kernel timing with HIP events recorded on the launch stream (mage_profile_*).
// When disabled (the default) a KernelTimer costs one relaxed flag check.
bool profiling_enabled();
bool profile_tag_selected(const char* tag);  // mage_profile_filter
// Timed single launches: the dispatch packet itself carries the start/stop events
// (hipExtLaunchKernel), so timing adds no marker packets to the stream — the BA step launches
// ~12 short kernels per trial, where two hipEventRecord calls per launch cost ~20% throughput.
bool timed_event_pair(hipEvent_t* start, hipEvent_t* stop, int* device);  // pooled; false if off
void timed_commit(const char* tag, int device, hipEvent_t start, hipEvent_t stop);

template <typename F, typename... Args>
inline void launch(const char* tag, F kernel, dim3 grid, dim3 block, uint32_t shmem, hipStream_t st, Args... args)
{
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int dev = 0;
    if (profiling_enabled() && profile_tag_selected(tag) && timed_event_pair(&e0, &e1, &dev)) {
        hipExtLaunchKernelGGL(kernel, grid, block, shmem, st, e0, e1, 0, args...);
        timed_commit(tag, dev, e0, e1);
    } else {
        hipLaunchKernelGGL(kernel, grid, block, shmem, st, args...);
    }
}

// Scope timer for multi-launch phases (two hipEventRecord calls around the scope).
struct KernelTimer {
    hipEvent_t start = nullptr, stop = nullptr;
    hipStream_t stream = nullptr;
    const char* name = nullptr;
    int device = 0;
    KernelTimer(const char* kernel, hipStream_t st);
    ~KernelTimer();
    KernelTimer(const KernelTimer&) = delete;
    KernelTimer& operator=(const KernelTimer&) = delete;
};

}  // namespace mage
