// context.cpp -- hdb_ctx lifetime, scratch arenas, kernel timing, host/device staging.
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <algorithm>
#include <cstdlib>

#include "common.hpp"

namespace hdb {

// Opt-in native backtrace on a fatal signal (HDB_NATIVE_BACKTRACE=1, set by bench.py): the
// library's frames go to stderr, then the previous handler (Python's faulthandler, which dumps
// every thread's Python stack, or the default action) runs.  Off by default: a JVM host uses
// SIGSEGV itself (implicit null checks), so a library must not take it unasked.
static struct sigaction g_prev_act[32];
static void native_backtrace(int sig) {
    static const char head[] = "\n[hdbmi] fatal signal, native backtrace:\n";
    (void)!write(2, head, sizeof(head) - 1);
    void *fr[64];
    const int n = backtrace(fr, 64);
    backtrace_symbols_fd(fr, n, 2);
    sigaction(sig, &g_prev_act[sig], nullptr);
    raise(sig);
}
__attribute__((constructor)) static void install_native_backtrace() {
    const char *e = getenv("HDB_NATIVE_BACKTRACE");
    if (!e || atoi(e) == 0) return;
    void *warm[2];
    (void)backtrace(warm, 2);  // loads libgcc's unwinder now, not inside the handler
    for (int sig : {SIGSEGV, SIGBUS, SIGILL, SIGFPE, SIGABRT}) {
        struct sigaction sa {};
        sa.sa_handler = native_backtrace;
        sigemptyset(&sa.sa_mask);
        sa.sa_flags = SA_RESETHAND;
        sigaction(sig, &sa, &g_prev_act[sig]);
    }
}

static thread_local std::string g_last_error;
void set_error(const std::string &msg) { g_last_error = msg; }
const char *last_error() { return g_last_error.c_str(); }

// small pinned host buffer for asynchronous device -> host counters (PINNED_WORDS int64)
int64_t *pinned_words(hdb_ctx *ctx) {
    if (!ctx->pinned) HIP_CHECK(hipHostMalloc((void **)&ctx->pinned, sizeof(int64_t) * PINNED_WORDS));
    return ctx->pinned;
}

void *host_arena(hdb_ctx *ctx, size_t bytes) {
    if (ctx->host_stage_bytes < bytes) {
        if (ctx->host_stage) {
            HIP_CHECK(hipStreamSynchronize(ctx->stream));
            HIP_CHECK(hipHostFree(ctx->host_stage));
            ctx->host_stage = nullptr;
        }
        size_t nb = bytes + bytes / 4 + 4096;
        HIP_CHECK(hipHostMalloc(&ctx->host_stage, nb));
        ctx->host_stage_bytes = nb;
    }
    return ctx->host_stage;
}

void *arena(hdb_ctx *ctx, int slot, size_t bytes) {
    Arena &a = ctx->arenas[slot];
    if (bytes == 0) bytes = 16;
    if (a.bytes < bytes) {
        if (a.ptr) {
            // the old buffer may still be in use by queued work on this stream
            HIP_CHECK(hipStreamSynchronize(ctx->stream));
            HIP_CHECK(hipFree(a.ptr));
            a.ptr = nullptr;
            a.bytes = 0;
        }
        size_t nb = bytes + bytes / 4 + 4096;
        void *p = nullptr;
        HIP_CHECK(hipMalloc(&p, nb));  // on failure the slot stays empty (never a stale size)
        a.ptr = p;
        a.bytes = nb;
    }
    return a.ptr;
}

static hipEvent_t get_event(hdb_ctx *ctx) {
    if (!ctx->event_pool.empty()) {
        hipEvent_t e = ctx->event_pool.back();
        ctx->event_pool.pop_back();
        return e;
    }
    hipEvent_t e;
    HIP_CHECK(hipEventCreate(&e));
    return e;
}

void stream_fence(hdb_ctx *ctx, hipStream_t from, hipStream_t to) {
    if (from == to) return;
    hipEvent_t e = get_event(ctx);
    HIP_CHECK(hipEventRecord(e, from));
    HIP_CHECK(hipStreamWaitEvent(to, e, 0));
    ctx->event_pool.push_back(e);  // reusable: re-recording only affects later waits
}

void time_begin(hdb_ctx *ctx, const char *name, TimedLaunch &t) {
    t.name = name;
    t.a = get_event(ctx);
    t.b = get_event(ctx);
    HIP_CHECK(hipEventRecord(t.a, ctx->stream));
}
void time_end(hdb_ctx *ctx, TimedLaunch &t) {
    HIP_CHECK(hipEventRecord(t.b, ctx->stream));
    ctx->pending.push_back(t);
}

static void drain_timing(hdb_ctx *ctx) {
    for (auto &t : ctx->pending) {
        HIP_CHECK(hipEventSynchronize(t.b));
        float ms = 0;
        HIP_CHECK(hipEventElapsedTime(&ms, t.a, t.b));
        auto &e = ctx->acc[t.name];
        e.first += ms;
        e.second += 1;
        ctx->event_pool.push_back(t.a);
        ctx->event_pool.push_back(t.b);
    }
    ctx->pending.clear();
}

bool is_device_ptr(const void *p) {
    if (!p) return false;
    hipPointerAttribute_t attr;
    hipError_t e = hipPointerGetAttributes(&attr, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged;
}

Stager::Stager(hdb_ctx *ctx) : ctx_(ctx) {
    mark_chunks_ = ctx->stage.size();
    mark_used_ = mark_chunks_ ? ctx->stage.back().used : 0;
    ctx->stage_depth++;
}

// carve from the top chunk; a new chunk (at least twice the last) when it does not fit.  Chunks
// are never freed while a Stager lives: queued copies and kernels may still use them
void *Stager::carve(size_t bytes) {
    const size_t nb = (std::max<size_t>(bytes, 16) + 255) & ~size_t(255);
    auto &ch = ctx_->stage;
    if (ch.empty() || ch.back().bytes - ch.back().used < nb) {
        const size_t want = std::max<size_t>(nb, ch.empty() ? (size_t)1 << 20 : 2 * ch.back().bytes);
        StageChunk c;
        HIP_CHECK(hipMalloc(&c.ptr, want));
        c.bytes = want;
        ch.push_back(c);
    }
    void *p = (char *)ch.back().ptr + ch.back().used;
    ch.back().used += nb;
    return p;
}

Stager::~Stager() {
    auto &ch = ctx_->stage;
    // pop this Stager's carvings: chunks it added keep their memory (stream-ordered reuse)
    for (size_t i = mark_chunks_; i < ch.size(); i++) ch[i].used = 0;
    if (mark_chunks_) ch[mark_chunks_ - 1].used = mark_used_;
    if (--ctx_->stage_depth == 0 && ch.size() > 1) {
        // outermost Stager and the stack grew: fold the chunks into one of their total size
        // once the stream has drained (the next call's carvings then never straddle chunks)
        size_t total = 0;
        for (auto &c : ch) total += c.bytes;
        if (hipStreamSynchronize(ctx_->stream) == hipSuccess) {
            for (auto &c : ch) (void)hipFree(c.ptr);
            ch.clear();
            StageChunk c;
            if (hipMalloc(&c.ptr, total) == hipSuccess) {
                c.bytes = total;
                ch.push_back(c);
            }
        }
    }
}

const void *Stager::in_raw(const void *p, size_t bytes) {
    if (!p) return nullptr;
    if (is_device_ptr(p)) return p;
    any_host_ = true;
    void *d = carve(bytes);
    bufs_.push_back({d, nullptr, bytes});
    if (bytes) HIP_CHECK(hipMemcpyAsync(d, p, bytes, hipMemcpyHostToDevice, ctx_->stream));
    return d;
}

void *Stager::out_raw(void *p, size_t bytes, bool copy_in) {
    if (!p) return nullptr;
    if (is_device_ptr(p)) return p;
    any_host_ = true;
    void *d = carve(bytes);
    bufs_.push_back({d, p, bytes});
    if (copy_in && bytes) HIP_CHECK(hipMemcpyAsync(d, p, bytes, hipMemcpyHostToDevice, ctx_->stream));
    return d;
}

void Stager::finish() {
    if (finished_) return;
    finished_ = true;
    for (auto &b : bufs_)
        if (b.host_dst && b.bytes)
            HIP_CHECK(hipMemcpyAsync(b.host_dst, b.dev, b.bytes, hipMemcpyDeviceToHost, ctx_->stream));
    if (any_host_) HIP_CHECK(hipStreamSynchronize(ctx_->stream));
}

}  // namespace hdb

using namespace hdb;

extern "C" {

const char *hdb_last_error(void) { return hdb::last_error(); }
int hdb_version(void) { return 100; }

int hdb_ctx_create(int device, hdb_ctx **out) {
    try {
        if (!out) HDB_THROW(HDB_EINVAL, "out is NULL");
        int count = 0;
        HIP_CHECK(hipGetDeviceCount(&count));
        if (device < 0 || device >= count) HDB_THROW(HDB_EDEVICE, "no such HIP device");
        HIP_CHECK(hipSetDevice(device));
        hdb_ctx *c = new hdb_ctx();
        c->device = device;
        HIP_CHECK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        c->own_stream = true;
        HIP_CHECK(hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
        hipDeviceProp_t prop;
        HIP_CHECK(hipGetDeviceProperties(&prop, device));
        c->num_cus = prop.multiProcessorCount;
        for (const char *k : {"prim_coop_plain_retries", "prim_coop_steps", "prim_coop_launches", "bubble_knn_replay_overflows",
                              "boruvka_visits_sum", "boruvka_evals_sum", "boruvka_bound_ns_sum"})
            c->stats[k] = 0;
        if (const char *e = getenv("HDB_PRIM_COOP_SLOTS"))  // A/B knob
            c->prim_coop_slots = (atoi(e) == 6 && !hdb_prim_spec_built()) ? 4 : atoi(e);
        // per-kernel HIP-event timing from birth (contexts created on worker threads, bench.py)
        if (const char *e = getenv("HDB_KERNEL_TIMING")) c->timing = atoi(e) != 0;
        if (const char *e = getenv("HDB_FLAT_BLOCK_LOG")) c->flat_block_log = atoi(e);  // A/B knob
        if (const char *e = getenv("HDB_PRIM_XCD")) c->prim_coop_xcd = atoi(e) != 0;       // A/B knob
        if (const char *e = getenv("HDB_BUBBLE_SPLIT")) c->bubble_knn_split = atoi(e) != 0;  // A/B knob
        if (const char *e = getenv("HDB_PRIM_XCD_MAX_WG")) c->prim_coop_xcd_max_wg = atoi(e);  // A/B knob
        if (const char *e = getenv("HDB_PRIM_COOP_BS")) c->prim_coop_bs = atoi(e);             // A/B knob
        if (const char *e = getenv("HDB_FLAT_LINK")) c->flat_link_variant = atoi(e);      // A/B knob
        if (const char *e = getenv("HDB_FLAT_ROOT")) c->flat_root_variant = atoi(e);      // A/B knob
        if (const char *e = getenv("HDB_MERGE_RUNS")) c->merge_runs = atoi(e) != 0;      // A/B knob
        if (const char *e = getenv("HDB_SSORT")) c->ssort = atoi(e) != 0;                // A/B knob
        if (const char *e = getenv("HDB_FLAT_RELABEL")) c->flat_relabel = atoi(e) != 0;  // A/B knob
        if (const char *e = getenv("HDB_FLAT_DEEP")) c->flat_deep_depth = atoi(e);          // A/B knob
        if (const char *e = getenv("HDB_FLAT_MID")) c->flat_mid_log = atoi(e);              // A/B knob
        if (const char *e = getenv("HDB_FLAT_DEEP_ROOT")) c->flat_deep_root = atoi(e);      // A/B knob
        if (const char *e = getenv("HDB_FLAT_DEEP_LINK")) c->flat_deep_link = atoi(e);      // A/B knob
        if (const char *e = getenv("HDB_BOR_EARLY_PTS")) c->boruvka_early_pts = atoi(e);    // A/B knob
        if (const char *e = getenv("HDB_BOR_ADJ")) c->boruvka_adj_seed = atoi(e) != 0;      // A/B knob
        if (const char *e = getenv("HDB_K1T_XCD")) c->k1t_xcd_chunks = atoi(e);             // A/B knob
        if (const char *e = getenv("HDB_BOR_XCD")) c->bor_xcd_chunks = atoi(e);             // A/B knob
        if (const char *e = getenv("HDB_BOR_EARLY_ROUNDS")) c->boruvka_early_rounds = atoi(e);  // A/B knob
        *out = c;
        return HDB_OK;
    } catch (const Error &e) {
        set_error(e.msg);
        return e.code;
    }
}

void hdb_ctx_destroy(hdb_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    for (auto &t : ctx->pending) {
        (void)hipEventDestroy(t.a);
        (void)hipEventDestroy(t.b);
    }
    for (auto e : ctx->event_pool) (void)hipEventDestroy(e);
    for (auto &a : ctx->arenas)
        if (a.ptr) (void)hipFree(a.ptr);
    for (auto &c : ctx->stage)
        if (c.ptr) (void)hipFree(c.ptr);
    if (ctx->pinned) (void)hipHostFree(ctx->pinned);
    if (ctx->host_stage) (void)hipHostFree(ctx->host_stage);
    if (ctx->own_stream) (void)hipStreamDestroy(ctx->stream);
    if (ctx->side) {
        (void)hipStreamSynchronize(ctx->side);
        (void)hipStreamDestroy(ctx->side);
    }
    delete ctx;
}

int hdb_ctx_set_stream(hdb_ctx *ctx, void *stream) {
    try {
        if (!ctx) HDB_THROW(HDB_EINVAL, "ctx is NULL");
        HIP_CHECK(hipSetDevice(ctx->device));
        HIP_CHECK(hipStreamSynchronize(ctx->stream));
        if (ctx->own_stream) HIP_CHECK(hipStreamDestroy(ctx->stream));
        // NULL selects the device's default (null) stream -- what PyTorch reports as
        // current_stream().cuda_stream == 0 -- never a private stream, so work stays
        // ordered with the caller's.
        ctx->stream = (hipStream_t)stream;
        ctx->own_stream = false;
        return HDB_OK;
    } catch (const Error &e) {
        set_error(e.msg);
        return e.code;
    }
}

int hdb_ctx_set_timing(hdb_ctx *ctx, int enable) {
    if (!ctx) return HDB_EINVAL;
    ctx->timing = enable != 0;
    return HDB_OK;
}

int hdb_ctx_kernel_time(hdb_ctx *ctx, const char *name, double *ms_total, int64_t *launches, int reset) {
    try {
        if (!ctx || !name) HDB_THROW(HDB_EINVAL, "NULL argument");
        HIP_CHECK(hipSetDevice(ctx->device));
        drain_timing(ctx);
        auto it = ctx->acc.find(name);
        double ms = 0;
        int64_t n = 0;
        if (it != ctx->acc.end()) {
            ms = it->second.first;
            n = it->second.second;
            if (reset) ctx->acc.erase(it);
        }
        if (ms_total) *ms_total = ms;
        if (launches) *launches = n;
        return HDB_OK;
    } catch (const Error &e) {
        set_error(e.msg);
        return e.code;
    }
}

int hdb_ctx_set_option(hdb_ctx *ctx, const char *name, int64_t value) {
    if (!ctx || !name) return HDB_EINVAL;
    const std::string k(name);
    if (k == "knn_fp32_screen") {
        ctx->force_fp64 = value == 0;
        return HDB_OK;
    }
    if (k == "knn_tree") {
        ctx->knn_tree = value != 0;
        return HDB_OK;
    }
    if (k == "knn_mfma") {
        ctx->knn_mfma = value != 0;
        return HDB_OK;
    }
    if (k == "knn_mfma_two_pass") {
        ctx->knn_mfma_two_pass = value != 0;
        return HDB_OK;
    }
    if (k == "nearest_grouped") {
        ctx->nearest_grouped = value != 0;
        return HDB_OK;
    }
    if (k == "knn_mfma_prune") {
        ctx->knn_mfma_prune = value != 0;
        return HDB_OK;
    }
    if (k == "knn_mfma_single") {
        ctx->knn_mfma_single = value != 0;
        return HDB_OK;
    }
    if (k == "knn_mfma_min_n") {
        ctx->knn_mfma_min_n = value;
        return HDB_OK;
    }
    if (k == "knn_tree_min_n") {
        ctx->knn_tree_min_n = value;
        return HDB_OK;
    }
    if (k == "prim_coop_plain") {
        ctx->prim_coop_plain = value != 0;
        return HDB_OK;
    }
    if (k == "bubble_fold_dim") {
        ctx->bubble_fold_dim = value != 0;
        return HDB_OK;
    }
    if (k == "bubble_knn_split") {
        ctx->bubble_knn_split = value != 0;
        return HDB_OK;
    }
    if (k == "prim_coop_xcd") {
        ctx->prim_coop_xcd = value != 0;
        return HDB_OK;
    }
    if (k == "prim_coop_plain_spin_log2") {
        if (value < 0 || value > 24) return HDB_EINVAL;
        ctx->prim_coop_plain_spin_log2 = (int)value;
        return HDB_OK;
    }
    if (k == "prim_coop") {
        ctx->prim_coop = value != 0;
        return HDB_OK;
    }
    if (k == "prim_coop_bs") {
        if (value != 0 && value != 128 && value != 256 && value != 512 && value != 1024) return HDB_EINVAL;
        ctx->prim_coop_bs = (int)value;
        return HDB_OK;
    }
    if (k == "prim_coop_slots") {
        if (value < 0 || value > 6) return HDB_EINVAL;
        if (value == 6 && !hdb_prim_spec_built()) {  // csrc/prim.hip: only with -DHDB_PRIM_SPEC=1
            set_error("prim_coop_slots 6: the speculative Prim is not in this build (-DHDB_PRIM_SPEC=1)");
            return HDB_EUNSUPPORTED;
        }
        ctx->prim_coop_slots = (int)value;
        return HDB_OK;
    }
    if (k == "leaf_seed_k") {
        if (value < -1 || value > 31) return HDB_EINVAL;
        ctx->leaf_seed_k = (int)value;
        return HDB_OK;
    }
    if (k == "leaf_list_rounds") {
        if (value < 0) return HDB_EINVAL;
        ctx->leaf_list_rounds = (int)value;
        return HDB_OK;
    }
    if (k == "boruvka_seed") {
        ctx->boruvka_seed = value != 0;
        return HDB_OK;
    }
    if (k == "trav_pop_test") {
        ctx->trav_pop_test = (int)value;
        return HDB_OK;
    }
    if (k == "bor_xcd_chunks") {
        if (value < 0 || value > 4096) return HDB_EINVAL;
        ctx->bor_xcd_chunks = (int)value;
        return HDB_OK;
    }
    if (k == "k1t_xcd_chunks") {
        if (value < 0 || value > 4096) return HDB_EINVAL;
        ctx->k1t_xcd_chunks = (int)value;
        return HDB_OK;
    }
    if (k == "boruvka_adj_seed") {
        ctx->boruvka_adj_seed = value != 0;
        return HDB_OK;
    }
    if (k == "boruvka_wave_pts") {
        ctx->boruvka_wave_pts = (int)value;
        return HDB_OK;
    }
    if (k == "boruvka_early_pts") {
        ctx->boruvka_early_pts = (int)value;
        return HDB_OK;
    }
    if (k == "boruvka_early_rounds") {
        ctx->boruvka_early_rounds = (int)value;
        return HDB_OK;
    }
    if (k == "boruvka_knn_seed") {
        ctx->boruvka_knn_seed = value != 0;
        return HDB_OK;
    }
    if (k == "flat_mid_log") {
        if (value < 0 || value > 24) return HDB_EINVAL;
        ctx->flat_mid_log = (int)value;
        return HDB_OK;
    }
    if (k == "flat_relabel") {
        ctx->flat_relabel = value != 0;
        return HDB_OK;
    }
    if (k == "ssort") {
        ctx->ssort = value != 0;
        return HDB_OK;
    }
    if (k == "ssort_cap") {
        if (value < 0 || value > 4096) return HDB_EINVAL;
        ctx->ssort_cap = (int)value;
        return HDB_OK;
    }
    if (k == "count_evals") {
        ctx->count_evals = value != 0;
        return HDB_OK;
    }
    set_error(std::string("unknown option ") + name);
    return HDB_EINVAL;
}

int hdb_ctx_get_stat(hdb_ctx *ctx, const char *name, int64_t *value) {
    if (!ctx || !name || !value) return HDB_EINVAL;
    auto it = ctx->stats.find(name);
    if (it != ctx->stats.end()) {
        *value = it->second;
        return HDB_OK;
    }
    set_error(std::string("unknown stat ") + name);
    return HDB_EINVAL;
}

int hdb_ctx_synchronize(hdb_ctx *ctx) {
    try {
        if (!ctx) HDB_THROW(HDB_EINVAL, "ctx is NULL");
        HIP_CHECK(hipStreamSynchronize(ctx->stream));
        return HDB_OK;
    } catch (const Error &e) {
        set_error(e.msg);
        return e.code;
    }
}

}  // extern "C"
