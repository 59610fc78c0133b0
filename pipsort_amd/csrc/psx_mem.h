// psx_mem.h — the engine's device / pinned-host allocations, through a
// per-process caching pool (psx_mem.cpp).
//
// hipMalloc of a multi-MB buffer costs ~0.1-0.3 ms on MI355X (VRAM mapping) and
// hipHostMalloc more (page pinning); a locus's setup and first pass made ~30 of
// them, several ms per locus.  Freed blocks are kept per device and size class
// and handed to the next allocation of that class (the next locus of a process
// has the same shapes).  A free synchronises the device first, as hipFree does,
// so a block is never reused while a kernel of its previous owner may run.
#ifndef PSX_MEM_H
#define PSX_MEM_H

#include <hip/hip_runtime.h>

#include <cstddef>

namespace psx {

hipError_t dmalloc_raw(void** p, size_t bytes);
hipError_t dfree(void* p);
hipError_t hmalloc_raw(void** p, size_t bytes);  // pinned host memory
hipError_t hmalloc_coherent_raw(void** p, size_t bytes);  // pinned host memory, coherent (device -> host hand-offs)
hipError_t hfree(void* p);

template <typename T>
inline hipError_t dmalloc(T** p, size_t bytes) {
    return dmalloc_raw(reinterpret_cast<void**>(p), bytes);
}
template <typename T>
inline hipError_t hmalloc(T** p, size_t bytes) {
    return hmalloc_raw(reinterpret_cast<void**>(p), bytes);
}

// Free without the device synchronisation: the caller guarantees no queued
// work uses the block (e.g. it synchronised the block's only stream).
hipError_t dfree_idle(void* p);
// While one is alive on a thread, that thread's dfree / hfree skip the device
// synchronisation (the caller synchronised the device / the streams first).
struct IdleScope {
    IdleScope();
    ~IdleScope();
};

// bytes currently held by the cache (all devices + pinned host), for tests
// release every cached (free) block of every device and the pinned host pools
// (live blocks are untouched); psx_pool_trim in the C ABI
void pool_trim();
size_t pool_cached_bytes();

// Streams: creating a HIP stream costs ~3-20 ms on MI355X (a hardware queue)
// and destroying one ~3 ms.  Non-blocking streams of a priority are kept per
// device: stream_get hands out an idle one (or creates it), stream_put
// synchronises it and keeps it for the next handle.
hipError_t stream_get(hipStream_t* s, int priority);
void stream_put(hipStream_t s, int priority);
// One hardware queue per device for the whole process (psx_single_queue in the
// C ABI, for one-locus processes such as the CLI): every stream_get hands out
// the device's one shared stream (normal priority) and stream_put keeps it.
// Every queue a process holds costs ~10-13 ms when it exits (the kernel driver
// tears it down: profiles/r06/r06late_c_exit_probe.txt).
void set_single_queue(bool on);

}  // namespace psx

#endif
