// psx_multi.hip — PostCal over several GPUs in one process (the C ABI's
// psx_multi_*).  The reference gets its whole-node parallelism in one process
// from 64 OpenMP threads over the configurations (postcal.cpp:747-769); here one
// engine handle per device entry evaluates shard i of n (psx_set_shard: the
// same equal-work slices as the one-process-per-GPU path), each driven by its
// own host thread, and the shards' accumulator images are folded on the first
// device: peer copies of the partial images (xGMI between GPUs of a node) and
// one psx_merge_partials, in rank order — the same deterministic fold the
// multi-process path runs after its RCCL all-gather.  Entries may repeat (several
// shards sharing one device: tests, and rehearsing a node on one GPU).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/pipsort_engine.h"

namespace {

thread_local std::string g_multi_err;

// In-process all-gather between the handles' host threads (psx_allgather_fn
// of the sharded SSS walk): a generation barrier around one shared buffer.
struct Gather {
    std::mutex mu;
    std::condition_variable cv;
    int n = 0, arrived = 0, generation = 0;
    bool aborted = false;
    std::vector<char> buf;

    bool barrier(std::unique_lock<std::mutex>& lk) {
        const int gen = generation;
        if (++arrived == n) {
            arrived = 0;
            generation++;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return generation != gen || aborted; });
        }
        return !aborted;
    }
    void abort() {
        std::lock_guard<std::mutex> lk(mu);
        aborted = true;
        cv.notify_all();
    }
};

struct GatherCtx {
    Gather* g;
    int rank;
};

int gather_fn(void* ctx, const void* send, void* recv, int64_t bytes) {
    GatherCtx* c = static_cast<GatherCtx*>(ctx);
    Gather& g = *c->g;
    std::unique_lock<std::mutex> lk(g.mu);
    if (g.aborted) return -1;
    if (g.buf.size() != (size_t)bytes * g.n) g.buf.resize((size_t)bytes * g.n);  // first arrival sizes it
    std::memcpy(g.buf.data() + (size_t)bytes * c->rank, send, (size_t)bytes);
    if (!g.barrier(lk)) return -1;
    std::memcpy(recv, g.buf.data(), (size_t)bytes * g.n);
    if (!g.barrier(lk)) return -1;
    return 0;
}

}  // namespace

struct psx_multi {
    std::vector<psx_engine*> h;
    std::vector<int> dev;
    std::vector<void*> stage;  // per-handle device buffer of one partial image (on its device)
    void* gathered = nullptr;  // n images on dev[0]
    int64_t bytes = 0;
    double sweep_ms = 0;
};

namespace {

template <typename F>
int on_each(psx_multi* m, F f) {
    const int n = (int)m->h.size();
    std::vector<int> rc(n, 0);
    std::vector<std::string> err(n);
    std::vector<std::thread> th;
    for (int i = 1; i < n; i++)
        th.emplace_back([&, i] {
            rc[i] = f(i);
            if (rc[i]) err[i] = psx_last_error();
        });
    rc[0] = f(0);
    if (rc[0]) err[0] = psx_last_error();
    for (auto& t : th) t.join();
    for (int i = 0; i < n; i++)
        if (rc[i]) {
            g_multi_err = "shard " + std::to_string(i) + " (device " + std::to_string(m->dev[i]) + "): " + err[i];
            return rc[i];
        }
    return 0;
}

// fold every shard's accumulator image into handle 0 (rank order)
int exchange(psx_multi* m) {
    const int n = (int)m->h.size();
    double ms = 0;
    for (int i = 0; i < n; i++) {
        psx_timing t;
        if (psx_get_timing(m->h[i], &t) == 0) ms = std::max(ms, t.sweep_ms);
    }
    m->sweep_ms = ms;
    if (n == 1) return 0;
    if (!m->gathered) {
        m->bytes = psx_partials_bytes(m->h[0]);
        if (hipSetDevice(m->dev[0]) != hipSuccess || hipMalloc(&m->gathered, (size_t)m->bytes * n) != hipSuccess) {
            g_multi_err = "out of device memory (partial images)";
            return PSX_EHIP;
        }
        m->stage.assign(n, nullptr);
        for (int i = 0; i < n; i++)
            if (m->dev[i] != m->dev[0] &&
                (hipSetDevice(m->dev[i]) != hipSuccess || hipMalloc(&m->stage[i], (size_t)m->bytes) != hipSuccess)) {
                g_multi_err = "out of device memory (partial image stage)";
                return PSX_EHIP;
            }
    }
    for (int i = 0; i < n; i++) {
        char* dst = (char*)m->gathered + (size_t)m->bytes * i;
        int rc;
        if (m->dev[i] == m->dev[0]) {
            if ((rc = psx_export_partials(m->h[i], dst))) { g_multi_err = psx_last_error(); return rc; }
        } else {
            if ((rc = psx_export_partials(m->h[i], m->stage[i]))) { g_multi_err = psx_last_error(); return rc; }
            if (hipMemcpyPeer(dst, m->dev[0], m->stage[i], m->dev[i], (size_t)m->bytes) != hipSuccess) {
                g_multi_err = "peer copy of a partial image failed";
                return PSX_EHIP;
            }
        }
    }
    const int rc = psx_merge_partials(m->h[0], m->gathered, n);
    if (rc) g_multi_err = psx_last_error();
    return rc;
}

// configurations evaluated by all shards (the folded count on handle 0)
int total_configs(psx_multi* m, uint64_t* n) {
    psx_timing t;
    int rc = psx_get_timing(m->h[0], &t);
    if (rc || m->h.size() == 1) {
        *n = rc ? 0 : t.configs;
        return rc;
    }
    *n = 0;
    for (psx_engine* e : m->h) {
        if ((rc = psx_get_timing(e, &t))) return rc;
        *n += t.configs;
    }
    return 0;
}

template <typename Create>
int create_multi(const int32_t* devices, int32_t n, psx_multi** out, Create create) {
    *out = nullptr;
    if (n < 1 || !devices) {
        g_multi_err = "need at least one device";
        return PSX_EINVAL;
    }
    psx_multi* m = new psx_multi;
    m->h.assign(n, nullptr);
    m->dev.assign(devices, devices + n);
    int rc = on_each(m, [&](int i) {
        int r = create(i, &m->h[i]);
        if (!r) r = psx_set_shard(m->h[i], i, n);
        return r;
    });
    if (rc) {
        psx_multi_destroy(m);
        return rc;
    }
    *out = m;
    return 0;
}

}  // namespace

extern "C" {

int psx_multi_create(const psx_problem* prob, const int32_t* devices, int32_t n, psx_multi** out) {
    return create_multi(devices, n, out, [&](int i, psx_engine** e) { return psx_create(prob, devices[i], e); });
}

int psx_multi_create_from_ld(const psx_ld_problem* prob, const int32_t* devices, int32_t n, psx_multi** out,
                             psx_setup_info* info) {
    std::vector<psx_setup_info> infos(std::max(n, 1));
    const int rc = create_multi(devices, n, out, [&](int i, psx_engine** e) {
        return psx_create_from_ld(prob, devices[i], e, &infos[i]);
    });
    if (rc == 0 && info) *info = infos[0];
    return rc;
}

void psx_multi_destroy(psx_multi* m) {
    if (!m) return;
    for (size_t i = 0; i < m->h.size(); i++) {
        if (m->h[i]) psx_destroy(m->h[i]);
        if (i < m->stage.size() && m->stage[i]) {
            hipSetDevice(m->dev[i]);
            hipFree(m->stage[i]);
        }
    }
    if (m->gathered) {
        hipSetDevice(m->dev[0]);
        hipFree(m->gathered);
    }
    delete m;
}

int32_t psx_multi_count(psx_multi* m) { return m ? (int32_t)m->h.size() : 0; }

const char* psx_multi_last_error(void) { return g_multi_err.c_str(); }

int psx_multi_run_exhaustive(psx_multi* m) {
    int rc = on_each(m, [&](int i) { return psx_run_exhaustive(m->h[i]); });
    return rc ? rc : exchange(m);
}

int psx_multi_run_configs(psx_multi* m, const int16_t* rows, int64_t n_rows, int32_t n_groups) {
    int rc = on_each(m, [&](int i) { return psx_run_configs(m->h[i], rows, n_rows, n_groups); });
    return rc ? rc : exchange(m);
}

int psx_multi_run_sss(psx_multi* m, int32_t* iterations_out) {
    const int n = (int)m->h.size();
    Gather g;
    g.n = n;
    std::vector<GatherCtx> ctx(n);
    std::vector<int32_t> it(n, 0);
    for (int i = 0; i < n; i++) ctx[i] = GatherCtx{&g, i};
    int rc = on_each(m, [&](int i) {
        const int r = psx_run_sss_sharded(m->h[i], gather_fn, &ctx[i], &it[i]);
        if (r) g.abort();  // release the other ranks from the barrier
        return r;
    });
    if (rc) return rc;
    if (iterations_out) *iterations_out = it[0];
    return exchange(m);
}

int psx_multi_get_accum(psx_multi* m, psx_accum* out) {
    const int rc = psx_get_accum(m->h[0], out);
    if (rc) g_multi_err = psx_last_error();
    return rc;
}

int psx_multi_get_timing(psx_multi* m, psx_timing* t) {
    const int rc = psx_get_timing(m->h[0], t);
    if (rc) {
        g_multi_err = psx_last_error();
        return rc;
    }
    t->sweep_ms = m->sweep_ms;  // the slowest shard's pass
    uint64_t n = 0;
    if (total_configs(m, &n) == 0) t->configs = n;
    return 0;
}

}  // extern "C"
