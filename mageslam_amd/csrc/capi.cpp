// capi.cpp — library-level C-ABI entry points: version, last error, device binding.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "common.hpp"

namespace mage {

namespace {
thread_local std::string g_last_error;
}

void set_error(const std::string& msg) { g_last_error = msg; }

namespace {
struct PoolBlock {
    int dev;
    void* p;
    uint64_t stamp;  // pool_take requests of this kind when the block was retired
};
struct BlockPool {
    std::mutex mu;
    std::multimap<size_t, PoolBlock> free[3];  // bytes -> block
    size_t held[3] = {0, 0, 0};
    uint64_t takes[3] = {0, 0, 0};
    std::vector<std::pair<int, hipStream_t>> streams;
};
BlockPool& block_pool()
{
    static BlockPool* p = new BlockPool();  // never destroyed: blocks outlive static teardown order
    return *p;
}
// Retired bytes kept per kind (device / page-locked / mapped): 512 / 128 / 32 MB by default, or
// MAGE_POOL_CAP_MB (one value for device memory; host kinds get a quarter and a sixteenth of it).
size_t pool_cap(int kind)
{
    static const size_t dev_cap = [] {
        const char* e = getenv("MAGE_POOL_CAP_MB");
        const long long mb = e ? atoll(e) : 512;
        return (size_t)(mb < 0 ? 0 : mb) << 20;
    }();
    return kind == 0 ? dev_cap : kind == 1 ? dev_cap / 4 : dev_cap / 16;
}
// A block no request could use over this many pool_take calls of its kind is freed for real.
constexpr uint64_t kPoolMaxAge = 256;

void free_block(int kind, void* p)
{
    if (kind == 0)
        (void)hipFree(p);
    else
        (void)hipHostFree(p);  // page-locked (1) and mapped (2) host memory
}
// Frees (under P.mu) the idle blocks of `kind` on `dev` (all of them, or the ones older than
// kPoolMaxAge requests); returns the bytes freed.
size_t trim_locked(BlockPool& P, int kind, int dev, bool all)
{
    size_t freed = 0;
    for (auto it = P.free[kind].begin(); it != P.free[kind].end();) {
        const PoolBlock& b = it->second;
        if ((dev < 0 || b.dev == dev) && (all || P.takes[kind] - b.stamp > kPoolMaxAge)) {
            free_block(kind, b.p);
            freed += it->first;
            P.held[kind] -= it->first;
            it = P.free[kind].erase(it);
        } else {
            ++it;
        }
    }
    return freed;
}
}  // namespace

void* pool_take(int kind, size_t n, size_t* got)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    BlockPool& P = block_pool();
    std::lock_guard<std::mutex> lk(P.mu);
    P.takes[kind]++;
    // the smallest retired block that fits and wastes at most half of itself
    for (auto it = P.free[kind].lower_bound(n); it != P.free[kind].end() && it->first <= 2 * n + 4096; ++it)
        if (it->second.dev == dev) {
            void* p = it->second.p;
            *got = it->first;
            P.held[kind] -= it->first;
            P.free[kind].erase(it);
            return p;
        }
    // a miss allocates anyway: free the blocks no request has been able to use for a while
    trim_locked(P, kind, dev, false);
    return nullptr;
}

size_t pool_trim(int kind, int device)
{
    BlockPool& P = block_pool();
    std::lock_guard<std::mutex> lk(P.mu);
    size_t freed = 0;
    for (int k = 0; k < 3; k++)
        if (kind < 0 || kind == k) freed += trim_locked(P, k, device, true);
    return freed;
}

// Idle non-blocking streams of destroyed per-task objects (mage_ba), per device.
hipStream_t stream_take()
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    BlockPool& P = block_pool();
    std::lock_guard<std::mutex> lk(P.mu);
    for (auto it = P.streams.begin(); it != P.streams.end(); ++it)
        if (it->first == dev) {
            hipStream_t s = it->second;
            P.streams.erase(it);
            return s;
        }
    return nullptr;
}

void stream_retire(hipStream_t s)
{
    int dev = 0;
    (void)hipGetDevice(&dev);
    BlockPool& P = block_pool();
    std::lock_guard<std::mutex> lk(P.mu);
    if (P.streams.size() >= 64) {
        (void)hipStreamDestroy(s);
        return;
    }
    P.streams.emplace_back(dev, s);
}

void pool_retire(int kind, void* p, size_t bytes)
{
    int dev = 0;
    (void)hipGetDevice(&dev);
    BlockPool& P = block_pool();
    std::lock_guard<std::mutex> lk(P.mu);
    if (P.held[kind] + bytes > pool_cap(kind)) {  // over the cap: a real free
        free_block(kind, p);
        return;
    }
    P.free[kind].emplace(bytes, PoolBlock{dev, p, P.takes[kind]});
    P.held[kind] += bytes;
}
const char* last_error() { return g_last_error.c_str(); }

namespace {
// devices whose architecture was checked (gfx950), so the per-frame entry points do not query
// the device properties on every call
std::mutex g_arch_mu;
std::map<int, std::string> g_arch;
}  // namespace

mage_status bind_device(int device)
{
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) {
        set_error("no HIP device available");
        return MAGE_EDEVICE;
    }
    if (device < 0 || device >= count) {
        set_error("device index " + std::to_string(device) + " out of range");
        return MAGE_EDEVICE;
    }
    MAGE_HIP(hipSetDevice(device));
    std::string arch;
    {
        std::lock_guard<std::mutex> lk(g_arch_mu);
        auto it = g_arch.find(device);
        if (it != g_arch.end()) arch = it->second;
    }
    if (arch.empty()) {
        hipDeviceProp_t prop;
        MAGE_HIP(hipGetDeviceProperties(&prop, device));
        arch = prop.gcnArchName;
        std::lock_guard<std::mutex> lk(g_arch_mu);
        g_arch[device] = arch;
    }
    if (std::strncmp(arch.c_str(), "gfx950", 6) != 0) {
        set_error("device is " + arch + ", this build targets gfx950 only");
        return MAGE_EDEVICE;
    }
    return MAGE_OK;
}

namespace {
// Per-thread stream scratch (stream_scratch): keyed by (device, stream, slot) inside the calling
// thread's own map, so a buffer is only ever grown — and its old storage freed — by the one thread
// that hands it to its own launches.  Two threads on one stream get two buffers; their launches
// are ordered by the stream, and neither can free memory the other still has to launch on.
thread_local bool g_stream_scratch_alive = false;
struct StreamScratchMap {
    std::map<std::tuple<int, hipStream_t, int>, DeviceBuffer> bufs;
    StreamScratchMap() { g_stream_scratch_alive = true; }
    ~StreamScratchMap()
    {
        g_stream_scratch_alive = false;
        // the streams may be gone by now (a caller's stream destroyed before its thread exits):
        // wait for the device instead of per stream before the buffers are freed
        if (!bufs.empty()) (void)hipDeviceSynchronize();
        for (auto& kv : bufs) kv.second.release();
    }
};
StreamScratchMap& stream_scratch_map()
{
    thread_local StreamScratchMap m;
    return m;
}

// Drops the calling thread's stream scratch of `st` (before the stream is destroyed, so a later
// stream that reuses the handle value starts without it).
void release_stream_scratch(hipStream_t st)
{
    if (!g_stream_scratch_alive) return;  // the map was already destroyed at thread exit
    auto& bufs = stream_scratch_map().bufs;
    for (auto it = bufs.begin(); it != bufs.end();) {
        if (std::get<1>(it->first) == st) {
            it->second.release();
            it = bufs.erase(it);
        } else {
            ++it;
        }
    }
}
}  // namespace

HostScratch::~HostScratch()
{
    if (st) {
        (void)hipStreamSynchronize(st);
        release_stream_scratch(st);
        (void)hipStreamDestroy(st);
    }
    buf.release();
    aux.release();
    host.release();
}

HostScratch* host_scratch(int device, ScratchSlot slot)
{
    thread_local std::map<std::pair<int, int>, std::unique_ptr<HostScratch>> per_thread;
    std::unique_ptr<HostScratch>& s = per_thread[{device, (int)slot}];
    if (!s) s.reset(new HostScratch());
    if (!s->st && hipStreamCreateWithFlags(&s->st, hipStreamNonBlocking) != hipSuccess) {
        s->st = nullptr;
        set_error("hipStreamCreateWithFlags failed");
        return nullptr;
    }
    return s.get();
}

void* stream_scratch(hipStream_t st, StreamSlot slot, size_t bytes)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) {
        set_error("hipGetDevice failed");
        return nullptr;
    }
    DeviceBuffer& b = stream_scratch_map().bufs[std::make_tuple(dev, st, (int)slot)];
    // growing frees the old buffer: this thread's launches on the stream that still use it are
    // the only ones that can (the buffer is private to the thread), let them finish first
    if (bytes > b.bytes && b.ptr && hipStreamSynchronize(st) != hipSuccess) {
        set_error("hipStreamSynchronize failed");
        return nullptr;
    }
    if (b.reserve(bytes) != MAGE_OK) return nullptr;
    return b.ptr;
}

namespace {
struct TimedLaunch {
    const char* name;  // string literal of the launch site
    int device;
    hipEvent_t start, stop;
};
std::atomic<bool> g_profiling{false};
std::mutex g_prof_mu;
std::vector<TimedLaunch> g_prof_pending;
struct Totals {
    uint64_t count = 0;
    double ms = 0;
};
std::map<std::string, Totals> g_prof_totals;
std::string g_prof_text;
// Recycled events per device: a timed launch costs two hipEventRecord calls, not two event
// creations (which cost more than the short BA kernels they time).
std::map<int, std::vector<hipEvent_t>> g_event_pool;

hipEvent_t pooled_event_locked(int device)
{
    auto& pool = g_event_pool[device];
    if (!pool.empty()) {
        hipEvent_t e = pool.back();
        pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    return hipEventCreate(&e) == hipSuccess ? e : nullptr;
}

void drain_locked()
{
    for (auto& t : g_prof_pending) {
        float ms = 0;
        if (hipEventSynchronize(t.stop) == hipSuccess && hipEventElapsedTime(&ms, t.start, t.stop) == hipSuccess) {
            auto& tot = g_prof_totals[t.name];
            tot.count++;
            tot.ms += ms;
        }
        g_event_pool[t.device].push_back(t.start);
        g_event_pool[t.device].push_back(t.stop);
    }
    g_prof_pending.clear();
}
}  // namespace

bool profiling_enabled() { return g_profiling.load(std::memory_order_relaxed); }

namespace {
std::mutex g_filter_mu;
std::string g_filter;  // only tags starting with this are timed (empty: every tag)
std::atomic<bool> g_filtered{false};
}  // namespace

bool profile_tag_selected(const char* tag)
{
    if (!g_filtered.load(std::memory_order_relaxed)) return true;
    std::lock_guard<std::mutex> lk(g_filter_mu);
    return std::strncmp(tag, g_filter.c_str(), g_filter.size()) == 0;
}

bool timed_event_pair(hipEvent_t* start, hipEvent_t* stop, int* device)
{
    if (hipGetDevice(device) != hipSuccess) return false;
    std::lock_guard<std::mutex> lk(g_prof_mu);
    *start = pooled_event_locked(*device);
    if (!*start) return false;
    *stop = pooled_event_locked(*device);
    if (!*stop) {
        g_event_pool[*device].push_back(*start);
        return false;
    }
    return true;
}

void timed_commit(const char* tag, int device, hipEvent_t start, hipEvent_t stop)
{
    std::lock_guard<std::mutex> lk(g_prof_mu);
    g_prof_pending.push_back({tag, device, start, stop});
    if (g_prof_pending.size() > 4096) drain_locked();
}

KernelTimer::KernelTimer(const char* kernel, hipStream_t st) : stream(st), name(kernel)
{
    if (!profiling_enabled()) return;
    if (hipGetDevice(&device) != hipSuccess) return;
    {
        std::lock_guard<std::mutex> lk(g_prof_mu);
        start = pooled_event_locked(device);
        stop = start ? pooled_event_locked(device) : nullptr;
        if (start && !stop) g_event_pool[device].push_back(start);
    }
    if (!stop) {
        start = nullptr;
        return;
    }
    (void)hipEventRecord(start, stream);
}

KernelTimer::~KernelTimer()
{
    if (!start) return;
    (void)hipEventRecord(stop, stream);
    std::lock_guard<std::mutex> lk(g_prof_mu);
    g_prof_pending.push_back({name, device, start, stop});
    if (g_prof_pending.size() > 4096) drain_locked();
}

}  // namespace mage

extern "C" {

const char* mage_version(void) { return "mageslam_amd 0.1.0 (gfx950)"; }
const char* mage_last_error(void) { return mage::last_error(); }
uint64_t mage_pool_trim(int32_t device) { return (uint64_t)mage::pool_trim(-1, device); }

void mage_profile_enable(int32_t enable) { mage::g_profiling.store(enable != 0); }

void mage_profile_filter(const char* tag_prefix)
{
    std::lock_guard<std::mutex> lk(mage::g_filter_mu);
    mage::g_filter = tag_prefix ? tag_prefix : "";
    mage::g_filtered.store(!mage::g_filter.empty());
}

void mage_profile_reset(void)
{
    std::lock_guard<std::mutex> lk(mage::g_prof_mu);
    mage::drain_locked();
    mage::g_prof_totals.clear();
}

const char* mage_profile_report(void)
{
    std::lock_guard<std::mutex> lk(mage::g_prof_mu);
    mage::drain_locked();
    std::string s;
    for (auto& kv : mage::g_prof_totals) {
        char buf[256];
        std::snprintf(buf, sizeof(buf), "%s %llu %.6f\n", kv.first.c_str(), (unsigned long long)kv.second.count,
                      kv.second.ms);
        s += buf;
    }
    mage::g_prof_text = s;
    return mage::g_prof_text.c_str();
}

}
