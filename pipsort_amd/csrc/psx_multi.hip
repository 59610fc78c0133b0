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
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/pipsort_engine.h"
#include "psx_mem.h"

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

// Persistent host threads, one per handle after the first (which runs on the
// caller's thread): created once with the handle set, woken per call.
class ShardPool {
  public:
    explicit ShardPool(int n) : n_(n), rc_(n, 0), err_(n) {
        for (int i = 1; i < n; i++) th_.emplace_back([this, i] { loop(i); });
    }
    ~ShardPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    // run f(i) for every shard i, concurrently; returns the shards' codes
    template <typename F>
    const std::vector<int>& run(F f) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            job_ = f;
            pending_ = n_ - 1;
            gen_++;
        }
        cv_.notify_all();
        one(0);
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [this] { return pending_ == 0; });
        job_ = nullptr;
        return rc_;
    }
    const std::string& err(int i) const { return err_[i]; }

  private:
    void one(int i) {
        rc_[i] = job_(i);
        err_[i] = rc_[i] ? psx_last_error() : "";  // the engine's message is per thread
    }
    void loop(int i) {
        int seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
            }
            one(i);
            std::lock_guard<std::mutex> lk(mu_);
            if (--pending_ == 0) done_.notify_all();
        }
    }
    int n_;
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    std::function<int(int)> job_;
    int gen_ = 0, pending_ = 0;
    bool stop_ = false;
    std::vector<int> rc_;
    std::vector<std::string> err_;
};

}  // namespace

struct psx_multi {
    std::vector<psx_engine*> h;
    std::vector<int> dev;
    std::vector<hipStream_t> st;    // per handle, on its device: export / merge only enqueue there
    std::vector<hipEvent_t> exported;  // per handle: its image has landed in `gathered`
    void* gathered = nullptr;       // n images on dev[0]
    int64_t bytes = 0;
    double sweep_ms = 0;
    uint64_t configs = 0;
    int32_t exact = 0;  // the last exhaustive step took the EXACT rerun
    ShardPool* pool = nullptr;
};

namespace {

// Run f on every shard concurrently.  A failing shard names itself; when one
// shard's failure makes the others fail too (the sharded SSS walk aborts its
// in-process all-gather: PSX_EEXCHANGE), the root cause is reported.
template <typename F>
int on_each(psx_multi* m, F f) {
    const std::vector<int>& rc = m->pool->run(std::function<int(int)>(f));
    int pick = -1;
    for (int i = 0; i < (int)rc.size(); i++)
        if (rc[i] && (pick < 0 || (rc[pick] == PSX_EEXCHANGE && rc[i] != PSX_EEXCHANGE))) pick = i;
    if (pick < 0) return 0;
    g_multi_err = "shard " + std::to_string(pick) + " (device " + std::to_string(m->dev[pick]) + "): " +
                  m->pool->err(pick);
    return rc[pick];
}

// Enqueue shard i's partial image into its slot of `gathered` on dev[0] (a peer
// copy over xGMI between devices, a plain copy on a repeated device) and mark it.
int export_one(psx_multi* m, int i) {
    char* dst = (char*)m->gathered + (size_t)m->bytes * i;
    int rc = psx_export_partials(m->h[i], dst);  // enqueued on st[i] (psx_set_stream)
    if (rc) return rc;
    if (hipSetDevice(m->dev[i]) != hipSuccess || hipEventRecord(m->exported[i], m->st[i]) != hipSuccess) return PSX_EHIP;
    return 0;
}

// Enqueue the fold of every shard's accumulator image into handle 0 (rank
// order) on dev[0]'s stream, after every shard's export (each enqueued by the
// shard's own host thread as soon as its run returned).
int merge_gathered(psx_multi* m) {
    const int n = (int)m->h.size();
    if (n == 1) return 0;
    if (hipSetDevice(m->dev[0]) != hipSuccess) return PSX_EHIP;
    for (int i = 0; i < n; i++)
        if (hipStreamWaitEvent(m->st[0], m->exported[i], 0) != hipSuccess) {
            g_multi_err = "stream wait on a partial image failed";
            return PSX_EHIP;
        }
    const int rc = psx_merge_partials(m->h[0], m->gathered, n);  // enqueued on st[0]
    if (rc) g_multi_err = std::string("merge of partial images: ") + psx_last_error();
    return rc;
}

// the slowest shard's pass (psx_timing.sweep_ms of each handle's last run / sync)
void shard_times(psx_multi* m) {
    double ms = 0;
    for (psx_engine* e : m->h) {
        psx_timing t;
        if (psx_get_timing(e, &t) == 0) ms = std::max(ms, t.sweep_ms);
    }
    m->sweep_ms = ms;
}

// configurations evaluated by all shards: summed over the handles' own counts
// (each psx_run_* reads its status before the fold), or — after an asynchronous
// exhaustive step, whose psx_sync on handle 0 reads the folded scalars — handle 0's
void total_configs(psx_multi* m, bool folded) {
    psx_timing t;
    m->configs = 0;
    if (folded || m->h.size() == 1) {
        if (psx_get_timing(m->h[0], &t) == 0) m->configs = t.configs;
        return;
    }
    for (psx_engine* e : m->h)
        if (psx_get_timing(e, &t) == 0) m->configs += t.configs;
}

// the merged result on dev[0], complete
int exchange(psx_multi* m) {
    shard_times(m);
    total_configs(m, false);
    int rc = merge_gathered(m);
    if (!rc && m->h.size() > 1 && hipStreamSynchronize(m->st[0]) != hipSuccess) rc = PSX_EHIP;
    return rc;
}

// run f on every shard, then (n > 1) export each image from the shard's own thread
template <typename F>
int run_and_gather(psx_multi* m, F f) {
    const int n = (int)m->h.size();
    int rc = on_each(m, [&](int i) {
        int r = f(i);
        if (!r && n > 1) r = export_one(m, i);
        return r;
    });
    return rc ? rc : exchange(m);
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
    m->st.assign(n, nullptr);
    m->exported.assign(n, nullptr);
    m->pool = new ShardPool(n);
    int rc = on_each(m, [&](int i) {
        int r = create(i, &m->h[i]);
        if (!r) r = psx_set_shard(m->h[i], i, n);
        if (r || n == 1) return r;
        // the shard's export / merge stream (only enqueue there) and its event
        if (hipSetDevice(m->dev[i]) != hipSuccess ||
            psx::stream_get(&m->st[i], 0) != hipSuccess ||
            hipEventCreateWithFlags(&m->exported[i], hipEventDisableTiming) != hipSuccess)
            return PSX_EHIP;
        return psx_set_stream(m->h[i], m->st[i]);
    });
    if (!rc && n > 1) {
        // peer access once per pair of distinct devices (shard i's image is written
        // straight into dev[0]'s gather buffer), then the gather buffer itself
        for (int i = 1; i < n && !rc; i++) {
            if (m->dev[i] == m->dev[0]) continue;
            for (int dir = 0; dir < 2 && !rc; dir++) {
                const int a = dir ? m->dev[0] : m->dev[i], b = dir ? m->dev[i] : m->dev[0];
                int can = 0;
                if (hipDeviceCanAccessPeer(&can, a, b) != hipSuccess || !can) continue;  // staged by the runtime
                hipSetDevice(a);
                const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
                    g_multi_err = std::string("peer access: ") + hipGetErrorString(e);
                    rc = PSX_EHIP;
                }
                (void)hipGetLastError();  // clear an already-enabled status
            }
        }
        if (!rc) {
            m->bytes = psx_partials_bytes(m->h[0]);
            if (hipSetDevice(m->dev[0]) != hipSuccess || psx::dmalloc(&m->gathered, (size_t)m->bytes * n) != hipSuccess) {
                g_multi_err = "out of device memory (partial images)";
                rc = PSX_EHIP;
            }
        }
    }
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
        if (m->h[i]) {
            psx_set_stream(m->h[i], nullptr);  // drains st[i]
            psx_destroy(m->h[i]);
        }
        hipSetDevice(m->dev[i]);
        if (m->exported[i]) hipEventDestroy(m->exported[i]);
        if (m->st[i]) psx::stream_put(m->st[i], 0);
    }
    if (m->gathered) {
        hipSetDevice(m->dev[0]);
        psx::dfree(m->gathered);
    }
    delete m->pool;
    delete m;
}

int32_t psx_multi_count(psx_multi* m) { return m ? (int32_t)m->h.size() : 0; }

const char* psx_multi_last_error(void) { return g_multi_err.c_str(); }

int psx_multi_run_exhaustive(psx_multi* m) {
    // Every shard's pass enqueued without a host sync (psx_run_exhaustive_async:
    // sweep on the handle's compute stream, merge and then the export on st[i]),
    // the fold on dev[0] ordered after all exports, then one psx_sync per shard.
    // The merged EXACT flag (any shard's notSharedLL group too far below its set
    // maximum) sends the whole step through the synchronous path, which reruns
    // the exact variant where needed.
    const int n = (int)m->h.size();
    int rc = on_each(m, [&](int i) {
        int r = psx_run_exhaustive_async(m->h[i]);
        if (!r && n > 1) r = export_one(m, i);
        return r;
    });
    if (!rc) rc = merge_gathered(m);
    int32_t exact = 0;
    if (!rc)
        rc = on_each(m, [&](int i) {
            int32_t x = 0;
            const int r = psx_sync(m->h[i], &x);  // h[0]: after the fold, so every shard's flag
            if (i == 0) exact = x;
            return r;
        });
    if (rc) return rc;
    m->exact = exact;
    if (exact) return run_and_gather(m, [&](int i) { return psx_run_exhaustive(m->h[i]); });
    shard_times(m);
    total_configs(m, true);
    return 0;
}

int psx_multi_run_configs(psx_multi* m, const int16_t* rows, int64_t n_rows, int32_t n_groups) {
    m->exact = 0;
    return run_and_gather(m, [&](int i) { return psx_run_configs(m->h[i], rows, n_rows, n_groups); });
}

int psx_multi_run_sss(psx_multi* m, int32_t* iterations_out) {
    const int n = (int)m->h.size();
    Gather g;
    g.n = n;
    std::vector<GatherCtx> ctx(n);
    std::vector<int32_t> it(n, 0);
    m->exact = 0;
    for (int i = 0; i < n; i++) ctx[i] = GatherCtx{&g, i};
    int rc = run_and_gather(m, [&](int i) {
        const int r = psx_run_sss_sharded(m->h[i], gather_fn, &ctx[i], &it[i]);
        if (r) g.abort();  // release the other ranks from the barrier
        return r;
    });
    if (!rc && iterations_out) *iterations_out = it[0];
    return rc;
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
    t->configs = m->configs;
    // any shard's flag: handle 0's own may be clear while another shard reran
    t->exact_rerun = m->exact;
    for (psx_engine* e : m->h) {
        psx_timing u;
        if (psx_get_timing(e, &u) == 0) t->exact_rerun |= u.exact_rerun;
    }
    return 0;
}

}  // extern "C"
