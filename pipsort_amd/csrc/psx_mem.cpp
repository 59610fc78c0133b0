// psx_mem.cpp — caching pool behind psx::dmalloc / dfree / hmalloc / hfree
// (psx_mem.h).  One mutex, free lists per (device, size class); pinned host
// blocks under device -1.
#include "psx_mem.h"

#include <atomic>
#include <cstdlib>
#include <map>
#include <mutex>
#include <unordered_map>
#include <utility>
#include <vector>

namespace psx {

namespace {

constexpr size_t kDevCap = size_t(4) << 30;   // cached bytes kept per device
constexpr size_t kHostCap = size_t(1) << 30;  // cached pinned host bytes

struct Block {
    size_t cls;
    int dev;  // -1: pinned host
};

struct Pool {
    std::mutex mu;
    std::unordered_map<void*, Block> live;
    std::map<std::pair<int, size_t>, std::vector<void*>> free;  // (device, class) -> blocks
    std::map<int, size_t> cached;                                 // device -> bytes in free lists
};

Pool& pool() {
    static Pool* p = new Pool();  // never destroyed: frees may run in static destructors
    return *p;
}

size_t size_class(size_t bytes) {
    if (bytes <= 512) return 512;
    if (bytes < (size_t(1) << 20)) {
        size_t c = 1024;
        while (c < bytes) c <<= 1;
        return c;
    }
    const size_t mb = size_t(1) << 20;
    return (bytes + mb - 1) / mb * mb;
}

// dev -1: pinned host, -2: pinned host, coherent (hipHostMallocCoherent: device
// stores reach host memory uncached, in order of their acknowledgement)
hipError_t raw_alloc(void** p, size_t cls, int dev) {
    return dev == -2 ? hipHostMalloc(p, cls, hipHostMallocCoherent) : dev < 0 ? hipHostMalloc(p, cls) : hipMalloc(p, cls);
}

hipError_t raw_free(void* p, int dev) { return dev < 0 ? hipHostFree(p) : hipFree(p); }

// release every cached block of `dev` (device current)
void drain(Pool& P, int dev) {
    std::vector<std::pair<void*, int>> out;
    {
        std::lock_guard<std::mutex> g(P.mu);
        for (auto it = P.free.begin(); it != P.free.end();) {
            if (it->first.first == dev) {
                for (void* b : it->second) out.push_back({b, dev});
                it = P.free.erase(it);
            } else {
                ++it;
            }
        }
        P.cached[dev] = 0;
    }
    for (auto& b : out) (void)raw_free(b.first, b.second);
}

hipError_t alloc(void** p, size_t bytes, bool host, bool coherent = false) {
    *p = nullptr;
    int dev = coherent ? -2 : -1;
    if (!host && hipGetDevice(&dev) != hipSuccess) return hipErrorInvalidDevice;
    const size_t cls = size_class(bytes);
    Pool& P = pool();
    {
        std::lock_guard<std::mutex> g(P.mu);
        auto it = P.free.find({dev, cls});
        if (it != P.free.end() && !it->second.empty()) {
            *p = it->second.back();
            it->second.pop_back();
            P.cached[dev] -= cls;
            P.live[*p] = {cls, dev};
            return hipSuccess;
        }
    }
    hipError_t e = raw_alloc(p, cls, dev);
    if (e != hipSuccess) {  // out of memory: give the cached blocks back and retry once
        (void)hipGetLastError();
        drain(P, dev);
        e = raw_alloc(p, cls, dev);
        if (e != hipSuccess) {
            *p = nullptr;
            return e;
        }
    }
    std::lock_guard<std::mutex> g(P.mu);
    P.live[*p] = {cls, dev};
    return hipSuccess;
}

thread_local int g_idle = 0;  // IdleScope depth

hipError_t release(void* p, bool host, bool sync = true) {
    sync = sync && g_idle == 0;
    if (!p) return hipSuccess;
    Pool& P = pool();
    Block b;
    {
        std::lock_guard<std::mutex> g(P.mu);
        auto it = P.live.find(p);
        if (it == P.live.end()) return host ? hipHostFree(p) : hipFree(p);  // not ours
        b = it->second;
        P.live.erase(it);
    }
    // as hipFree: no kernel of the previous owner may still use the block when
    // it is handed out again
    int cur = 0;
    const bool other = b.dev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != b.dev;
    if (sync) {
        if (other) (void)hipSetDevice(b.dev);
        hipError_t e = hipDeviceSynchronize();
        if (other) (void)hipSetDevice(cur);
        if (e != hipSuccess) return e;
    }
    std::vector<void*> evict;
    {
        std::lock_guard<std::mutex> g(P.mu);
        P.free[{b.dev, b.cls}].push_back(p);
        size_t& c = P.cached[b.dev];
        c += b.cls;
        const size_t cap = b.dev < 0 ? kHostCap : kDevCap;
        // over the cap: drop the largest classes of this device first
        for (auto it = P.free.rbegin(); c > cap && it != P.free.rend(); ++it) {
            if (it->first.first != b.dev) continue;
            while (c > cap && !it->second.empty()) {
                evict.push_back(it->second.back());
                it->second.pop_back();
                c -= it->first.second;
            }
        }
    }
    if (!evict.empty()) {
        if (other) (void)hipSetDevice(b.dev);
        for (void* x : evict) (void)raw_free(x, b.dev);
        if (other) (void)hipSetDevice(cur);
    }
    return hipSuccess;
}

}  // namespace

// PSX_POOL_POISON=1 (tests): every device block handed out is filled with 0xFF
// bytes (NaN doubles, -1 ints), so code that relied on fresh memory being zero
// fails loudly instead of depending on which block it got
hipError_t dmalloc_raw(void** p, size_t bytes) {
    static const bool poison = std::getenv("PSX_POOL_POISON") != nullptr;
    hipError_t e = alloc(p, bytes, false);
    if (e == hipSuccess && poison && bytes) {
        e = hipMemset(*p, 0xFF, bytes);
        if (e == hipSuccess) e = hipDeviceSynchronize();
    }
    return e;
}
hipError_t dfree(void* p) { return release(p, false); }
hipError_t hmalloc_raw(void** p, size_t bytes) { return alloc(p, bytes, true); }
hipError_t hmalloc_coherent_raw(void** p, size_t bytes) { return alloc(p, bytes, true, true); }
hipError_t hfree(void* p) { return release(p, true); }
hipError_t dfree_idle(void* p) { return release(p, false, false); }
IdleScope::IdleScope() { g_idle++; }
IdleScope::~IdleScope() { g_idle--; }

namespace {
struct StreamPool {
    std::mutex mu;
    std::map<std::pair<int, int>, std::vector<hipStream_t>> idle;  // (device, priority)
    std::map<int, hipStream_t> shared;                             // single-queue mode: per device
};
std::atomic<bool> g_single_queue{false};
StreamPool& streams() {
    static StreamPool* p = new StreamPool();
    return *p;
}
}  // namespace

hipError_t stream_get(hipStream_t* s, int priority) {
    *s = nullptr;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    StreamPool& P = streams();
    if (g_single_queue.load()) {
        std::lock_guard<std::mutex> g(P.mu);
        hipStream_t& x = P.shared[dev];
        if (!x && (e = hipStreamCreateWithFlags(&x, hipStreamNonBlocking)) != hipSuccess) {
            x = nullptr;
            return e;
        }
        *s = x;
        return hipSuccess;
    }
    {
        std::lock_guard<std::mutex> g(P.mu);
        auto& v = P.idle[{dev, priority}];
        if (!v.empty()) {
            *s = v.back();
            v.pop_back();
            return hipSuccess;
        }
    }
    return hipStreamCreateWithPriority(s, hipStreamNonBlocking, priority);
}

void stream_put(hipStream_t s, int priority) {
    if (!s) return;
    {
        StreamPool& P = streams();
        std::lock_guard<std::mutex> g(P.mu);
        for (auto& kv : P.shared)
            if (kv.second == s) return;  // the single-queue mode's stream stays
    }
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipStreamSynchronize(s) != hipSuccess) {
        (void)hipStreamDestroy(s);
        return;
    }
    StreamPool& P = streams();
    std::lock_guard<std::mutex> g(P.mu);
    P.idle[{dev, priority}].push_back(s);
}

void set_single_queue(bool on) { g_single_queue.store(on); }

void pool_trim() {
    Pool& P = pool();
    std::vector<std::pair<void*, int>> out;
    {
        std::lock_guard<std::mutex> g(P.mu);
        for (auto& kv : P.free)
            for (void* b : kv.second) out.push_back({b, kv.first.first});
        P.free.clear();
        P.cached.clear();
    }
    int cur = 0;
    const bool have = hipGetDevice(&cur) == hipSuccess;
    for (auto& b : out) {
        if (b.second >= 0 && have && b.second != cur) (void)hipSetDevice(b.second);
        (void)raw_free(b.first, b.second);
        if (b.second >= 0 && have && b.second != cur) (void)hipSetDevice(cur);
    }
}

size_t pool_cached_bytes() {
    Pool& P = pool();
    std::lock_guard<std::mutex> g(P.mu);
    size_t s = 0;
    for (auto& kv : P.cached) s += kv.second;
    return s;
}

}  // namespace psx
