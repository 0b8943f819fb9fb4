// mqvs.hip -- C-ABI of libmqvs.so: segments, workspaces, search orchestration.
//
// Search = the whole of MergeTreeVSManager::vectorScanWithoutIndex for one data
// part (MergeTreeVSManager.cpp:960-1536) in a handful of launches:
//   1. query prep        (norms; cosine re-normalisation variants)
//   2. probe scan        dense values for rows [0, P) (P ~ 3k*n/4096)
//   3. probe select      per-query k-th key -> threshold tau; first candidates
//   4. main scan         rows [P, n), append rows with key <= tau
//   5. final select      sort candidates by the reference's total order, emit k
// If a candidate list overflows (adversarial ties), tau is tightened from the
// stored candidates and the part is re-scanned (rare; counted in the stats).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "mqvs_internal.h"


namespace mqvs {

static thread_local std::string g_error;
static thread_local mqvs_search_stats g_stats{};
// Process-wide defaults of the per-call mode flags (mqvs_set_*): atomics, read
// once at the entry of a call, so a setter racing with searches on other
// threads never switches a search's path midway (per-call flags override them).
static std::atomic<int> g_timing{0};
static std::atomic<int> g_prefilter{2};  // planes built by new segments (mqvs_set_prefilter)
static std::atomic<size_t> g_scratch_budget{(size_t)1 << 30};  // bytes per scratch buffer of one call

size_t scratch_budget() { return g_scratch_budget.load(std::memory_order_relaxed); }

void set_error(const std::string &msg) { g_error = msg; }


// ---------------------------------------------------------------------------
// Workspace HBM budget (mqvs_set_workspace_budget).  The reference admits up
// to 2 x physical cores concurrent scans (MergeTreeVSManager.cpp:972-975,
// ScanThreadLimiter.h:25-58), each of which here keeps a per-thread device
// workspace (~1 GB at nq 1000).  A call is admitted with a reservation of
// the workspace it is expected to grow to (its thread's last call, or the last
// call of any thread); when that would take the sum of all workspaces and
// reservations past the budget, idle workspaces (threads between calls) are
// freed first, then the call waits until running calls finish and give their
// memory back (a call that ends while others wait frees its workspace).
// Growth beyond the reservation passes the same gate inside the call; only
// if every running call is then waiting does it go over the budget (counted)
// rather than deadlock.
// the pinned record [padded, selected, generation] of k_chunk_count (int64
// words at host_flags + kCountRec), and how long a filtered search polls it
constexpr int kCountRec = 32;
constexpr int kCountSpinUs = 200;

struct Workspace;
struct WsGate {
    std::mutex mu;
    std::condition_variable cv;
    size_t held = 0, peak = 0;  // device bytes of all workspaces
    size_t reserved = 0;        // admitted calls' expected growth not yet allocated
    size_t typical = 0;         // the last finished call's workspace (a new thread's estimate)
    int active = 0;             // threads inside a call
    int blocked = 0;            // of them, waiting for memory
    int admitting = 0;          // threads waiting to start a call
    int trimming = 0;           // workspaces being freed outside the mutex (their bytes still in held)
    int64_t waits = 0, trims = 0, over = 0;
    std::vector<Workspace *> all;
};
static WsGate &gate() {
    static WsGate *g = new WsGate();  // (leaked: workspaces of exited threads stay registered)
    return *g;
}
static std::atomic<size_t> g_ws_budget{0};  // 0 = not set: a quarter of the device's memory, fixed at first use
static size_t ws_budget() {
    size_t b = g_ws_budget.load(std::memory_order_relaxed);
    if (b) return b;
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess || tot == 0) tot = (size_t)64 << 30;
    b = tot / 4;
    size_t expect = 0;
    g_ws_budget.compare_exchange_strong(expect, b);
    return g_ws_budget.load(std::memory_order_relaxed);
}

struct Workspace {
    hipStream_t stream = nullptr;
    hipEvent_t ev[6] = {};
    static constexpr int kSegEv = 64;
    hipEvent_t seg_ev[kSegEv] = {};  // per main-scan segment: start, end
    DevBuf queries, qvars, qnorms, qmu, qlam, status, filter, exists, ord, probe, tau, count, cand,
        overflow, out_ids, out_dist, misc, qhi, bq, thr, cand2, count2, gcount, goff, glist, large, sticky, surv,
        recs, flags, p4q, qord;
    int *host_flags = nullptr;  // pinned (64 ints; the selected-row count record at kCountRec)
    HostBuf pin_q, pin_f, pin_e, pin_o;  // pinned staging of host-pointer calls (stage_in / stage_out_results)
    int64_t count_gen = 0;      // generation of the last selected-row count record asked for
    bool pending_timing = false, pending_bf16 = false;  // search_collect_stats
    int device = 0;
    std::mutex use;     // held by the owning thread during a call (WsCall); trimmers only try_lock it
    hipStream_t last = nullptr;  // the stream of the current call (the caller's, or `stream`)
    hipEvent_t done = nullptr;   // recorded on it at the end of every call: a trimmer waits for it
    int depth = 0;      // the owner's nested calls
    size_t held = 0;    // device bytes of the buffers (the gate's share of this workspace)
    size_t resv = 0;    // the current call's reservation left
    size_t call_peak = 0, recent = 0;  // most held during the current / the last call
    WsExt *ext = nullptr;  // the thread's index workspace: its scratch is counted and trimmed with this one
    bool trimming = false;  // picked by a trimmer, which waits and frees outside the gate mutex
    void init(int dev) {
        if (stream) return;
        device = dev;
        MQVS_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        for (auto &e : ev) MQVS_HIP(hipEventCreate(&e));
        for (auto &e : seg_ev) MQVS_HIP(hipEventCreate(&e));
        MQVS_HIP(hipEventCreateWithFlags(&done, hipEventDisableTiming));
        MQVS_HIP(hipHostMalloc((void **)&host_flags, 64 * sizeof(int), hipHostMallocDefault));
        WsGate &g = gate();
        std::lock_guard<std::mutex> lk(g.mu);
        g.all.push_back(this);
    }
    // the buffers, sticky word included (gate accounting is the caller's)
    size_t free_buffers(bool keep_sticky) {
        DevBuf *all[] = {&queries, &qvars, &qnorms, &qmu,  &qlam,   &status,  &filter,   &exists, &ord,
                         &probe,   &tau,   &count,  &cand, &overflow, &out_ids, &out_dist, &misc,
                         &qhi, &bq, &thr, &cand2, &count2, &gcount, &goff, &glist, &large, &sticky, &surv,
                         &recs, &flags, &p4q, &qord};
        size_t b = 0;
        for (auto *x : all) {
            if (keep_sticky && x == &sticky) continue;
            b += x->cap;
            x->release();
        }
        for (HostBuf *x : {&pin_q, &pin_f, &pin_e, &pin_o}) x->release();  // (host memory: not counted)
        return b;
    }
    // free every buffer but the ASYNC sticky word (and the index scratch
    // counted here), once the last call's work has drained -- on whichever
    // stream it ran, the caller's included (an ASYNC call returns with its
    // kernels in flight).  Called WITHOUT the gate mutex (GPU waits and frees
    // must not stall every other thread's admission) by a thread that holds
    // `use`; the caller updates `held` and the gate under the mutex.
    size_t trim() {
        int cur = -1;
        (void)hipGetDevice(&cur);
        (void)hipSetDevice(device);
        (void)hipEventSynchronize(done);
        (void)hipStreamSynchronize(stream);
        size_t b = free_buffers(true);
        if (ext) b += ext->free_scratch();
        if (cur >= 0) (void)hipSetDevice(cur);
        return b;
    }
    void release() {
        {
            WsGate &g = gate();
            std::lock_guard<std::mutex> lk(g.mu);
            g.all.erase(std::remove(g.all.begin(), g.all.end(), this), g.all.end());
            g.held -= std::min(g.held, held);
            held = 0;
        }
        if (ext) (void)ext->free_scratch();
        ext = nullptr;
        (void)free_buffers(false);
        if (host_flags) (void)hipHostFree(host_flags);
        host_flags = nullptr;
        for (auto &e : ev)
            if (e) (void)hipEventDestroy(e);
        for (auto &e : seg_ev)
            if (e) (void)hipEventDestroy(e);
        if (done) (void)hipEventDestroy(done);
        done = nullptr;
        if (stream) (void)hipStreamDestroy(stream);
        stream = nullptr;
    }
    void *get(DevBuf &b, size_t bytes);
};

// lk holds the gate mutex: free idle workspaces of other threads until `need`
// more bytes fit under the budget.  The victims are picked (their `use` taken,
// marked) under the mutex; their GPU waits and frees run with it released, and
// the accounting is updated once it is re-taken.  Returns whether anything was
// trimmed (the caller re-checks its condition either way).
static bool trim_idle(std::unique_lock<std::mutex> &lk, WsGate &g, Workspace *me, size_t need, size_t budget) {
    std::vector<Workspace *> victims;
    size_t expect = 0;
    for (Workspace *w : g.all) {
        if (g.held - std::min(g.held, expect) + g.reserved + need <= budget) break;
        if (w == me || w->trimming || w->held <= w->sticky.cap || !w->use.try_lock()) continue;
        w->trimming = true;
        victims.push_back(w);
        expect += w->held - w->sticky.cap;
    }
    if (victims.empty()) return false;
    g.trimming += (int)victims.size();
    lk.unlock();
    for (Workspace *w : victims) (void)w->trim();
    lk.lock();
    for (Workspace *w : victims) {
        // (the gate counted held - sticky of it: every gated buffer is gone)
        g.held -= std::min(g.held, w->held - std::min(w->held, w->sticky.cap));
        w->held = std::min(w->held, w->sticky.cap);
        w->trimming = false;
        ++g.trims;
        --g.trimming;
        w->use.unlock();
    }
    g.cv.notify_all();
    return true;
}

void *Workspace::get(DevBuf &b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (bytes <= b.cap) return b.p;
    const size_t old = b.cap, delta = bytes - old;
    {
        WsGate &g = gate();
        std::unique_lock<std::mutex> lk(g.mu);
        // the admitted reservation first
        const size_t take = std::min(delta, resv);
        resv -= take;
        g.reserved -= std::min(g.reserved, take);
        const size_t rest = delta - take;
        g.held += take;
        held += take;
        if (rest) {
            const size_t B = ws_budget();
            bool counted = false;
            while (g.held + g.reserved + rest > B) {
                trim_idle(lk, g, this, rest, B);
                if (g.held + g.reserved + rest <= B) break;
                // (memory being freed outside the mutex comes back: wait for it)
                const int others = g.active - g.blocked - (depth > 0 ? 1 : 0);
                if (others <= 0 && g.trimming == 0) {
                    ++g.over;  // every running call waits: go over rather than deadlock
                    break;
                }
                if (!counted) ++g.waits;
                counted = true;
                ++g.blocked;
                g.cv.wait(lk);
                --g.blocked;
            }
            g.held += rest;
            held += rest;
        }
        call_peak = std::max(call_peak, held);
        g.peak = std::max(g.peak, g.held);
    }
    try {
        b.get(bytes);
    } catch (...) {
        // (the old buffer is gone too)
        WsGate &g = gate();
        std::lock_guard<std::mutex> lk(g.mu);
        g.held -= std::min(g.held, bytes);
        held -= std::min(held, bytes);
        g.cv.notify_all();
        throw;
    }
    return b.p;
}

// one call of the owning thread on its workspace (nests): counted as running;
// at the end, if other calls wait for memory (or the gate is over budget), the
// workspace is freed for them
struct WsCall {
    Workspace &ws;
    explicit WsCall(Workspace &w) : ws(w) {
        if (ws.depth++ != 0) return;
        ws.use.lock();
        WsGate &g = gate();
        std::unique_lock<std::mutex> lk(g.mu);
        // admission: reserve the expected workspace
        const size_t B = ws_budget();
        const size_t need = std::max(ws.recent ? ws.recent : g.typical, ws.held);
        const size_t extra = need - ws.held;
        bool counted = false;
        while (g.held + g.reserved + extra > B) {
            trim_idle(lk, g, &ws, extra, B);
            // (nobody to wait for: no running call, no trim in flight)
            if (g.held + g.reserved + extra <= B || (g.active == 0 && g.trimming == 0)) break;
            if (!counted) ++g.waits;
            counted = true;
            ++g.admitting;
            g.cv.wait(lk);
            --g.admitting;
        }
        ++g.active;
        ws.resv = extra;
        g.reserved += extra;
        ws.call_peak = ws.held;
    }
    ~WsCall() {
        if (--ws.depth != 0) return;
        (void)hipEventRecord(ws.done, ws.last ? ws.last : ws.stream);
        ws.last = nullptr;
        WsGate &g = gate();
        bool self_trim = false;
        {
            std::lock_guard<std::mutex> lk(g.mu);
            --g.active;
            g.reserved -= std::min(g.reserved, ws.resv);
            ws.resv = 0;
            ws.recent = ws.call_peak;
            g.typical = ws.call_peak;
            const size_t B = g_ws_budget.load(std::memory_order_relaxed);
            self_trim = (g.blocked > 0 || g.admitting > 0 || (B && g.held > B)) && ws.held > ws.sticky.cap &&
                        hipEventQuery(ws.done) == hipSuccess;
            if (self_trim) ++g.trimming;  // (waiters wait for these bytes instead of going over)
            g.cv.notify_all();
        }
        if (self_trim) {
            // (the frees run outside the gate mutex; `use` is still held, so
            // no trimmer picks this workspace meanwhile)
            (void)ws.trim();
            std::lock_guard<std::mutex> lk(g.mu);
            g.held -= std::min(g.held, ws.held - std::min(ws.held, ws.sticky.cap));
            ws.held = std::min(ws.held, ws.sticky.cap);
            ++g.trims;
            --g.trimming;
            g.cv.notify_all();
        }
        ws.use.unlock();
    }
    WsCall(const WsCall &) = delete;
    WsCall &operator=(const WsCall &) = delete;
};

static thread_local std::map<int, Workspace> *g_ws = nullptr;

static Workspace &workspace(int device) {
    if (!g_ws) g_ws = new std::map<int, Workspace>();  // leaked at exit on purpose
    Workspace &w = (*g_ws)[device];
    w.init(device);
    return w;
}

// WsScope (mqvs_internal.h): a WsCall on the thread's workspace, made the
// current one for GBuf growth
struct WsScopeImpl {
    Workspace &ws;
    WsCall call;
    explicit WsScopeImpl(Workspace &w) : ws(w), call(w) {}
};
static thread_local WsScopeImpl *t_scope = nullptr;

WsScope::WsScope(int device, WsExt *ext) {
    Workspace &w = workspace(device);
    auto *im = new WsScopeImpl(w);  // admission (may wait for memory)
    w.ext = ext;                    // (one ext per thread and device; `use` is held)
    prev_ = t_scope;
    t_scope = im;
    impl_ = im;
}
WsScope::~WsScope() {
    t_scope = static_cast<WsScopeImpl *>(prev_);
    delete static_cast<WsScopeImpl *>(impl_);
}
void WsScope::set_stream(hipStream_t s) { static_cast<WsScopeImpl *>(impl_)->ws.last = s; }

void *GBuf::get(size_t bytes) {
    if (!t_scope) fail(MQVS_ERR_LOGICAL, "gated scratch grown outside a workspace scope");
    return t_scope->ws.get(*this, bytes);
}

static thread_local int t_fault_status = MQVS_OK, t_fault_calls = 0;
static thread_local bool t_fault_mid = false;  // MQVS_FAULT_MID_CALL: fire inside the call instead

void fault_point() {
    if (t_fault_calls <= 0 || t_fault_mid) return;
    --t_fault_calls;
    fail(t_fault_status, "injected fault (mqvs_inject_fault)");
}

// the mid-call drill point: a filtered mqvs_search right after its
// selected-row count is queued (the count kernel is then still in flight)
static void fault_point_mid() {
    if (t_fault_calls <= 0 || !t_fault_mid) return;
    --t_fault_calls;
    fail(t_fault_status, "injected fault (mqvs_inject_fault, mid-call)");
}

// ---------------------------------------------------------------------------
// Host waits (mqvs_set_wait_mode).  The reference admits up to 2 x physical
// cores concurrent scans (ScanThreadLimiter.h:25-58, MergeTreeVSManager.cpp:
// 974-975); here each of them waits for its GPU work, and a waiting thread
// that spins holds a host core for the whole search.  On ROCm neither
// hipStreamSynchronize nor hipEventSynchronize on a hipEventBlockingSync
// event sleeps (the runtime documents BlockingSync as a synonym of Yield;
// measured: thread CPU time = wall time in every runtime mode,
// profiles/r06/host_cpu_wait_runtime.jsonl), so the library sleeps itself:
// HYBRID polls the work's completion event for up to spin_us (a short
// search returns without a wake-up), then sleeps most of the time this
// thread's recent waits took (the shorter of the last two: searches of one
// thread are alike, and a shorter one must not wait behind a longer one's
// estimate): to 97 % of it, then polls through its end (at most a tenth of
// it), then -- a first wait, or a longer one -- polls with sleeps of 1/32 of
// the time waited so far (10-200 us: the overshoot stays a few per cent of
// the wait).  Sleeps are shortened by how late this thread's wake-ups have
// landed; a wait found done on waking halves the estimate, so the estimate
// never learns the sleep's overshoot; an expected wait under 3 wake-up
// latenesses is polled through (a sleep cannot save much of it), and in
// HYBRID so is one under 10 spin_us.  The history
// is kept per call shape and wait position (WaitScope): one history for every
// call made nq 1 searches after nq 1000 ones sleep 13 ms for 2.4 ms of work.
// BLOCK skips both polls.
static std::atomic<int> g_wait_mode{MQVS_WAIT_HYBRID};
static std::atomic<int> g_wait_spin_us{50};

void cpu_relax() {
#if defined(__x86_64__) || defined(__i386__)
    __builtin_ia32_pause();
#endif
}

int device_cus() {
    static std::atomic<int> cache[64];
    int dev = 0;
    MQVS_HIP(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64) {
        int cus = 0;
        MQVS_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        return cus;
    }
    int cus = cache[dev].load(std::memory_order_relaxed);
    if (cus <= 0) {
        MQVS_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        cache[dev].store(cus, std::memory_order_relaxed);
    }
    return cus;
}

int wait_spin_us() {
    const int m = g_wait_mode.load(std::memory_order_relaxed);
    return m == MQVS_WAIT_RUNTIME ? -1 : m == MQVS_WAIT_BLOCK ? 0 : g_wait_spin_us.load(std::memory_order_relaxed);
}

// one completion event per thread and device (the current one)
static hipEvent_t wait_event() {
    struct Events {
        std::map<int, hipEvent_t> ev;
        ~Events() {
            for (auto &e : ev) (void)hipEventDestroy(e.second);
        }
    };
    static thread_local Events t_ev;
    int dev = 0;
    MQVS_HIP(hipGetDevice(&dev));
    hipEvent_t &e = t_ev.ev[dev];
    if (!e) MQVS_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return e;
}

static thread_local uint64_t t_wait_key = 0;  // the current API call's shape (0: none)
static thread_local int t_wait_ord = 0;        // waits so far in that call

static uint64_t wait_mix(uint64_t h, uint64_t v) {
    h ^= v + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
    return h * 0xFF51AFD7ED558CCDull;
}

WaitScope::WaitScope(std::initializer_list<uint64_t> parts) : prev_key(t_wait_key), prev_ord(t_wait_ord) {
    uint64_t h = 0x6A09E667F3BCC909ull;
    for (uint64_t v : parts) h = wait_mix(h, v);
    t_wait_key = h | 1;
    t_wait_ord = 0;
}

WaitScope::~WaitScope() {
    t_wait_key = prev_key;
    t_wait_ord = prev_ord;
}

void host_wait(hipStream_t s) {
    const int spin = wait_spin_us();
    if (spin < 0) {
        MQVS_HIP(hipStreamSynchronize(s));
        return;
    }
    using clk = std::chrono::steady_clock;
    // this thread's last two waits (us) per wait key: (call shape, position in
    // the call), 16 keys, least recently used out
    struct Hist {
        uint64_t key;
        double h[2];
        uint64_t used;
    };
    static thread_local Hist t_tab[16];
    static thread_local uint64_t t_use = 0;
    static thread_local double t_late = 60.0;  // how late this thread's sleeps wake (us)
    const uint64_t key = t_wait_key ? wait_mix(t_wait_key, (uint64_t)t_wait_ord++) | 1 : 1;
    Hist *hs = nullptr;
    for (Hist &e : t_tab)
        if (e.key == key) hs = &e;
    if (!hs) {
        hs = &t_tab[0];
        for (Hist &e : t_tab)
            if (e.used < hs->used) hs = &e;
        *hs = Hist{key, {0.0, 0.0}, 0};
    }
    hs->used = ++t_use;
    hipEvent_t e = wait_event();
    MQVS_HIP(hipEventRecord(e, s));
    const auto t0 = clk::now();
    auto since = [](clk::time_point a) { return std::chrono::duration<double, std::micro>(clk::now() - a).count(); };
    auto done = [&]() {
        const hipError_t q = hipEventQuery(e);
        if (q == hipSuccess) return true;
        if (q != hipErrorNotReady) MQVS_HIP(q);
        return false;
    };
    bool fin = done();
    auto poll_to = [&](double stop_us) {
        while (!fin && since(t0) < stop_us) {
            for (int i = 0; i < 32; ++i) cpu_relax();
            fin = done();
        }
    };
    auto nap = [&](double us) {  // sleep, learning how late the wake-up lands
        const auto a = clk::now();
        std::this_thread::sleep_for(std::chrono::microseconds((int64_t)us));
        t_late = 0.8 * t_late + 0.2 * std::min(1000.0, std::max(0.0, since(a) - us));
        fin = done();
    };
    // 1. poll (HYBRID)
    poll_to(spin);
    const double hint = std::min(hs->h[0], hs->h[1]);
    // what this wait tells the next one: the time waited, except when the
    // work was found done on waking from step 2 -- it ended somewhere before,
    // and recording the wake-up time would ratchet the estimate up by the
    // sleep's overshoot every search; halve the estimate instead (a shorter
    // search than the history's is then re-timed within two waits), and the
    // next wait's step 3 or 4 times it again
    double learned = -1;
    if (!fin && hint > 0) {
        if (spin > 0 && hint < std::max(3 * t_late, 10.0 * spin)) {
            // (HYBRID, a short wait -- under 10 spin_us, 500 us by default, or
            // 3 wake-up latenesses: polled through.  A sleep there saves
            // little CPU and its wake-up jitter is a large share of the wait:
            // 1 % of 50M rows at nq 1, 0.420 ms polled vs 0.457 ms with the
            // sleep, tools/wait_ab.py.  Under load waits grow past it.)
            poll_to(2 * hint + spin);
        } else {
            // 2. sleep to 97 % of the expected time, less the wake-up's lateness
            const double until = 0.97 * hint - t_late, now_us = since(t0);
            if (until > now_us + 20) {
                nap(until - now_us);
                if (fin) learned = std::min(since(t0), 0.5 * hint);
            }
            // 3. poll through the expected end (at most a tenth of the expected time)
            poll_to(std::min(1.1 * hint, since(t0) + 0.1 * hint));
        }
    }
    // 4. sleep-poll (a first wait, or one longer than expected)
    while (!fin) nap(std::min(200.0, std::max(10.0, since(t0) / 32)));
    // (a wait the first poll covers -- a status copy after the work, say --
    // says nothing about the next search's length)
    const double w = learned > 0 ? learned : since(t0);
    if (w > 50.0) {
        hs->h[1] = hs->h[0];
        hs->h[0] = w;
    }
}

void stage_out_begin(HostBuf &pin, const int64_t *dids, const float *ddist, size_t m, hipStream_t s) {
    auto *h = (unsigned char *)pin.get(12 * m);
    if (!m) return;
    MQVS_HIP(hipMemcpyAsync(h, dids, 8 * m, hipMemcpyDeviceToHost, s));
    MQVS_HIP(hipMemcpyAsync(h + 8 * m, ddist, 4 * m, hipMemcpyDeviceToHost, s));
}

void stage_out_end(const HostBuf &pin, int64_t *ids, float *dist, size_t m) {
    if (!m) return;
    const auto *h = (const unsigned char *)pin.p;
    std::memcpy(ids, h, 8 * m);
    std::memcpy(dist, h + 8 * m, 4 * m);
}

void stage_out_results(HostBuf &pin, int64_t *ids, float *dist, const int64_t *dids, const float *ddist, size_t m,
                       hipStream_t s) {
    stage_out_begin(pin, dids, ddist, m, s);
    host_wait(s);
    stage_out_end(pin, ids, dist, m);
}

void ws_detach_ext(int device, WsExt *ext) {
    if (!g_ws) return;
    auto it = g_ws->find(device);
    if (it == g_ws->end()) return;
    Workspace &w = it->second;
    std::lock_guard<std::mutex> u(w.use);
    if (w.ext != ext) return;
    const size_t b = ext->free_scratch();
    WsGate &g = gate();
    std::lock_guard<std::mutex> lk(g.mu);
    g.held -= std::min(g.held, b);
    w.held -= std::min(w.held, b);
    w.ext = nullptr;
    g.cv.notify_all();
}


// ---------------------------------------------------------------------------
// segments

static void prepare_segment(mqvs_segment *s, const uint8_t *dev_nonempty_bytes,
                            hipStream_t st) {
    if (dev_nonempty_bytes) {
        MQVS_HIP(hipMalloc((void **)&s->nonempty_bits, (size_t)(s->n + 7) / 8));
        s->bytes += (size_t)(s->n + 7) / 8;
        launch_pack_nonempty(dev_nonempty_bytes, s->n, s->nonempty_bits, st);
        const int64_t nchunks = (s->n + s->granule - 1) / s->granule;
        MQVS_HIP(hipMalloc((void **)&s->chunk_ord, sizeof(int) * std::max<int64_t>(nchunks, 1)));
        s->bytes += sizeof(int) * nchunks;
        launch_chunk_ordinals(nullptr, s->nonempty_bits, nullptr, s->n, s->granule, 0,
                              s->chunk_ord, st);
    }
    if (s->metric == MQVS_METRIC_COSINE) launch_normalize_rows(s->rows, s->n, s->d, st);
    // |y|^2 per row: the BLAS-branch L2 norms, and (all metrics) the bound of
    // the bf16 pre-filter
    MQVS_HIP(hipMalloc((void **)&s->norms, sizeof(float) * std::max<int64_t>(s->n, 1)));
    s->bytes += sizeof(float) * s->n;
    launch_row_norms(s->rows, s->n, s->d, s->norms, st);
    // bf16 plane of the rows for the nq >= 20 pre-filter (rows padded to kBfK)
    s->dpad = (s->d + kBfK - 1) / kBfK * kBfK;
    MQVS_HIP(hipMalloc((void **)&s->ynorm_max, 16 + sizeof(float) * kMxRec));
    MQVS_HIP(hipMemsetAsync(s->ynorm_max, 0, 16 + sizeof(float) * kMxRec, st));
    launch_max_norm(s->norms, s->n, s->ynorm_max, st);
    const int64_t nr = std::max<int64_t>(s->n, 1);
    const int64_t nr16 = (nr + 15) / 16 * 16;  // row-blocked planes: blocks of 16 rows
    const int split = g_prefilter.load(std::memory_order_relaxed);
    const size_t hb = (size_t)nr16 * s->dpad * sizeof(uint16_t);
    if (split == kHiSplit && hipMalloc((void **)&s->rows_hi, hb) == hipSuccess) {
        s->bytes += hb;
        launch_to_hi(s->rows, s->n, s->d, s->d, s->dpad, 1, nr16, s->rows_hi, nullptr, s->ynorm_max + 4, st);
        s->split = split;
        s->plane_bytes = hb;
    } else {
        (void)hipGetLastError();  // no room (or planes off): exact fp32 batch path only
        s->rows_hi = nullptr;
    }
    MQVS_HIP(hipGetLastError());
    float ymax = 0.f;
    MQVS_HIP(hipMemcpyAsync(&ymax, s->ynorm_max, sizeof(float), hipMemcpyDeviceToHost, st));
    MQVS_HIP(hipStreamSynchronize(st));
    // the bound needs finite, moderate norms (FLT_MAX-filled empty arrays of
    // L2/IP parts overflow): otherwise the exact fp32 path serves nq >= 20
    s->approx_ok = s->rows_hi != nullptr && ymax == ymax && ymax < 1e18f;
}

static void check_seg_args(int64_t n, int32_t d, int32_t metric, int64_t granule,
                           int64_t row_offset) {
    if (n < 0 || n >= ((int64_t)1 << 32)) fail(MQVS_ERR_BAD_ARGUMENTS, "segment rows must be in [0, 2^32)");
    if (d <= 0) fail(MQVS_ERR_BAD_ARGUMENTS, "dimension must be positive");
    if (metric != MQVS_METRIC_L2 && metric != MQVS_METRIC_IP && metric != MQVS_METRIC_COSINE)
        fail(MQVS_ERR_NOT_IMPLEMENTED, "Metric not implemented in brute force search for Float32 Vector");
    if (granule <= 0) fail(MQVS_ERR_BAD_ARGUMENTS, "granule_rows must be positive");
    if (row_offset < 0 || row_offset % granule != 0)
        fail(MQVS_ERR_BAD_ARGUMENTS, "row_offset must be a non-negative multiple of granule_rows");
}

static mqvs_segment *new_segment(int64_t n, int32_t d, int32_t metric, int64_t granule,
                                 int64_t row_offset) {
    auto *s = new mqvs_segment();
    MQVS_HIP(hipGetDevice(&s->device));
    s->n = n;
    s->d = d;
    s->metric = metric;
    s->granule = granule;
    s->row_offset = row_offset;
    const size_t bytes = (size_t)std::max<int64_t>(n, 1) * d * sizeof(float);
    hipError_t e = hipMalloc((void **)&s->rows, bytes);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        delete s;
        fail(MQVS_ERR_MEMORY_LIMIT, "HBM allocation of " + std::to_string(bytes) + " bytes failed");
    }
    s->bytes = bytes;
    return s;
}

static void free_segment(mqvs_segment *s) {
    if (!s) return;
    int cur = -1;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(s->device);
    if (s->rows_host)
        (void)hipHostFree(s->rows_host);
    else if (s->rows)
        (void)hipFree(s->rows);
    if (s->norms) (void)hipFree(s->norms);
    if (s->nonempty_bits) (void)hipFree(s->nonempty_bits);
    if (s->rows_hi) (void)hipFree(s->rows_hi);
    if (s->ynorm_max) (void)hipFree(s->ynorm_max);
    if (s->chunk_ord) (void)hipFree(s->chunk_ord);
    if (s->codes) (void)hipFree(s->codes);
    if (cur >= 0) (void)hipSetDevice(cur);
    delete s;
}

static bool all_nonempty(const uint8_t *ne, int64_t n) {
    for (int64_t i = 0; i < n; ++i)
        if (!ne[i]) return false;
    return true;
}

// ---------------------------------------------------------------------------
// search

struct Range {
    int64_t begin, end, tiles, tiles_per_chunk;
};

static Range make_range(int64_t b, int64_t e, int64_t tile_rows, int64_t chunk_rows, bool aligned) {
    Range r{b, e, 0, 0};
    if (e <= b) return r;
    if (aligned) {
        r.tiles_per_chunk = (chunk_rows + tile_rows - 1) / tile_rows;
        const int64_t nch = (e - b + chunk_rows - 1) / chunk_rows;
        r.tiles = nch * r.tiles_per_chunk;
    } else {
        r.tiles = (e - b + tile_rows - 1) / tile_rows;
    }
    return r;
}

enum ScanKind { kScanSmall = 0, kScanMfma32 = 1, kScanBf16 = 2 };

// tile_rows: the range's tile length when not the kind's (kBfRowsSmall: a
// bf16 scan that scan_hi_small_tiles_ok admits)
static void run_scan(ScanParams p, const Range &r, int kind, int metric, bool probe, hipStream_t st,
                     int64_t tile_rows = 0) {
    if (r.tiles <= 0) return;
    p.row_begin = r.begin;
    p.row_end = r.end;
    p.tiles = r.tiles;
    p.tiles_per_chunk = r.tiles_per_chunk;
    p.tile_rows = tile_rows > 0 ? tile_rows : kind == kScanSmall ? kSmallRows : kind == kScanBf16 ? kBfRows : kMfmaRows;
    if (kind == kScanMfma32)
        launch_scan_mfma(p, metric, probe, st);
    else if (kind == kScanBf16)
        launch_scan_hi(p, metric, probe, st);
    else
        launch_scan_small(p, metric, probe, st);
    MQVS_HIP(hipGetLastError());
}

static int64_t round_up(int64_t v, int64_t m) { return (v + m - 1) / m * m; }

// Query variants.  Cosine re-normalises the query once per searched chunk
// (VIWithDataPart.h:358, the query object shared across chunks); the chain
// x, x/|x|, ... is stored until it repeats (mu, lambda per query).  The
// default table of kMaxVariants covers the chains of typical data (Gaussian
// and mixture parts repeat within ~15 steps).  When a part has more chunk
// ordinals than that and some chain did not repeat (small-integer vectors
// wander for hundreds of steps), the table is rebuilt with one variant per
// ordinal (up to kMaxVariantsCap) -- one host sync, only on such parts.
// Returns maxv; ASYNC calls cannot sync and keep the default table (their
// outcome goes to mqvs_async_check).
// zeroed_status: 4 ints the caller has already zeroed on this stream (saves a
// memset launch), or null
static int prep_variants(Workspace &ws, const float *dq, int nq, int d, bool cos, bool l2norms, int64_t ords,
                         bool may_sync, float *&qvars, float *&qnorms, int *&qmu, int *&qlam, int *&status,
                         hipStream_t s, int *zeroed_status = nullptr, int maxv_override = 0) {
    const int64_t qstride = round_up(d, 32);
    qnorms = (float *)ws.get(ws.qnorms, sizeof(float) * nq);
    qmu = (int *)ws.get(ws.qmu, sizeof(int) * nq);
    qlam = (int *)ws.get(ws.qlam, sizeof(int) * nq);
    status = zeroed_status ? zeroed_status : (int *)ws.get(ws.status, sizeof(int) * 4);
    int maxv = cos ? (maxv_override > 0 ? maxv_override : kMaxVariants) : 1;
    for (int pass = 0; pass < 2; ++pass) {
        const size_t bytes = sizeof(float) * (size_t)nq * maxv * qstride;
        // (no clear of the table: the prep writes every stored variant,
        // zeros past a query's chain)
        qvars = (float *)ws.get(ws.qvars, bytes);
        if (pass > 0 || !zeroed_status) launch_fill2((uint32_t *)status, 4, 0u, nullptr, 0, 0u, s);
        launch_query_prep(dq, nq, d, cos ? MQVS_METRIC_COSINE : MQVS_METRIC_L2, l2norms, qvars, maxv, qnorms, qmu,
                          qlam, status, s);
        MQVS_HIP(hipGetLastError());
        if (pass > 0 || !cos || ords <= maxv || !may_sync || maxv_override > 0) break;
        MQVS_HIP(hipMemcpyAsync(ws.host_flags + 12, status, sizeof(int), hipMemcpyDeviceToHost, s));
        host_wait(s);
        if (!ws.host_flags[12]) break;
        maxv = (int)std::min<int64_t>(ords, kMaxVariantsCap);
    }
    return maxv;
}

// metric: public metric, or kMetricIpRaw for the faiss-contract entry point
static std::atomic<int> g_batch_mode{0};   // 0: bf16 pre-filter + exact re-rank when possible, 1: fp32 MFMA
static std::atomic<int> g_gather_mode{1};  // selective PREWHERE: 0 never gather, 1 when <= 60% selected, 2 always

static int call_batch_mode(uint32_t flags) {
    return (flags & MQVS_F_EXACT) ? 1 : g_batch_mode.load(std::memory_order_relaxed);
}
static int call_gather_mode(uint32_t flags) {
    if (flags & MQVS_F_GATHER_NEVER) return 0;
    if (flags & MQVS_F_GATHER_ALWAYS) return 2;
    return g_gather_mode.load(std::memory_order_relaxed);
}
static bool call_timing(uint32_t flags) {
    return (flags & MQVS_F_TIMING) || g_timing.load(std::memory_order_relaxed) != 0;
}
bool timing_on(uint32_t flags) { return call_timing(flags); }

// ASYNC searches cannot run the host-driven fallbacks (exact re-scan after a
// pre-filter overflow, tightened re-scan, the cosine variant check): their
// device flags are OR-ed into this thread's sticky word, which
// mqvs_async_check reads and clears.
static int *sticky_word(Workspace &ws, hipStream_t s) {
    if (!ws.sticky.p) {
        ws.get(ws.sticky, 16);
        MQVS_HIP(hipMemsetAsync(ws.sticky.p, 0, 16, s));
    }
    return (int *)ws.sticky.p;
}

int *async_sticky(int device, hipStream_t s) { return sticky_word(workspace(device), s); }

// per-stage times of the search just synchronised (HIP events on its stream)
static void read_search_times(Workspace &ws, mqvs_search_stats &st) {
    float a = 0, b = 0, c = 0, e = 0, f = 0;
    MQVS_HIP(hipEventElapsedTime(&a, ws.ev[5], ws.ev[1]));
    MQVS_HIP(hipEventElapsedTime(&b, ws.ev[1], ws.ev[2]));
    MQVS_HIP(hipEventElapsedTime(&c, ws.ev[2], ws.ev[3]));
    MQVS_HIP(hipEventElapsedTime(&e, ws.ev[3], ws.ev[4]));
    MQVS_HIP(hipEventElapsedTime(&f, ws.ev[0], ws.ev[4]));
    st.probe_ms = a;
    st.probe_select_ms = b;
    // main_ms: the scan kernels only; refine_ms: the refinements between
    float scan = 0.f;
    const int ns = std::min(st.segments, Workspace::kSegEv / 2);
    for (int i = 0; i < ns; ++i) {
        float x = 0.f;
        MQVS_HIP(hipEventElapsedTime(&x, ws.seg_ev[2 * i], ws.seg_ev[2 * i + 1]));
        scan += x;
    }
    st.main_ms = ns > 0 ? scan : c;
    st.refine_ms = ns > 0 ? c - scan : 0.0;
    st.final_ms = e;
    st.total_ms = f;
}

// Large k (above the LDS sort): the global-scratch sort of the final select,
// and query sub-batches small enough that the candidate lists and the dense
// probe matrix stay within a fixed HBM budget.
static int large_k_cap(int k) { return (int)std::min<int64_t>(kCandMax, (int64_t)16 * k); }
static int large_k_batch(int64_t n, int k) {
    const int64_t cap = large_k_cap(k);
    const int64_t probe = std::min<int64_t>(n, (int64_t)((double)k * (double)n / (double)(cap / 3)) + 1);
    const int64_t budget = (int64_t)scratch_budget();
    const int64_t by_cand = budget / 8 / cap;                          // 8-B candidates
    const int64_t by_probe = budget / 4 / std::max<int64_t>(probe, 1);  // fp32 probe values
    return (int)std::max<int64_t>(1, std::min(by_cand, by_probe));
}

// the gather list launched before the selected count is read (search_impl)
// is sized for every row: up to 64M rows' worth
constexpr size_t kSpecListBytes = (size_t)256 << 20;

// Main-scan segmentation: the first segment is `first` probe lengths, each
// next one `growth` times the previous; the probe aims at `target`
// candidates.  Few queries: fewer, longer segments (each refinement is a
// launch boundary plus a one-workgroup kernel; measured at 10M x 768, nq 1:
// 7 segments 2.81 ms, 3 segments 2.72 ms; nq 1000 prefers 2, 2).
// MQVS_SEG="first,growth,target" overrides (tools/ab_split.py).
constexpr int64_t kMinSegRows = 65536;
struct SegTune {
    int64_t first = 2, growth = 2, target = 16384;
};
static SegTune seg_tune(int nq) {
    SegTune v;
    if (nq <= 4) {
        v.first = 8;
        v.growth = 4;
        // one or two queries: a 4x shorter probe (its single-workgroup select
        // 53 -> 21 us at 10M x 768; one more segment; wall median 2.80 ->
        // 2.75 ms at nq 1, no gain at nq 4, profiles/r02/smallnq/seg_ab.jsonl);
        // round 6: half that probe and a first segment of 16 probe lengths
        // (3 segments, 2 refinements): kernels 2.386 -> 2.365 ms, wall median
        // 2.418-2.439 -> 2.394-2.404 ms (profiles/r06/seg_ab_nq1.jsonl)
        if (nq <= 2) {
            v.first = 16;
            v.target = 32768;
        }
    } else if (nq < 256) {
        v.first = 4;
        v.growth = 4;
    }
    if (const char *e = tune_env("MQVS_SEG")) {
        long long a = 0, b = 0, c = 0;
        if (std::sscanf(e, "%lld,%lld,%lld", &a, &b, &c) == 3 && a >= 1 && b >= 2 && c >= 256) {
            v.first = a;
            v.growth = b;
            v.target = c;
        }
    }
    return v;
}

// formula_nq: the batch size that selects faiss's distance formula (0: nq).
// Query sub-batches of one call (large k) keep the call's formula: faiss
// decides it from the whole batch (BruteForceSearch.h:80-87, nx >= 20).
// async_word (ASYNC calls only): where the search's fallback flags go instead
// of the thread's sticky word (the sharded search exchanges them); the
// survivor counts and event times are then collected by search_collect_stats
// after the caller's own stream sync.
static void search_impl(mqvs_segment *seg, const float *queries, int nq, int k, int metric,
                        const uint8_t *filter, const uint8_t *exists, int64_t *out_ids,
                        float *out_dist, uint32_t flags, hipStream_t user_stream,
                        bool force_exact = false, int64_t ord_base = -1, int maxv_hint = 0, int formula_nq = 0,
                        int *async_word = nullptr) {
    const int fnq = formula_nq > 0 ? formula_nq : nq;
    if (!seg) fail(MQVS_ERR_BAD_ARGUMENTS, "null segment");
    if (seg->binary) fail(MQVS_ERR_LOGICAL, "binary (FixedString) segment: search it with mqvs_search_binary");
    if (nq < 0 || k < 0) fail(MQVS_ERR_BAD_ARGUMENTS, "nq and k must be non-negative");
    if (nq > 0 && k > 0 && (!queries || !out_ids || !out_dist))
        fail(MQVS_ERR_BAD_ARGUMENTS, "null query or output pointer");
    const bool cos = metric == MQVS_METRIC_COSINE;
    if (metric != MQVS_METRIC_L2 && metric != MQVS_METRIC_IP && !cos && metric != kMetricIpRaw)
        fail(MQVS_ERR_NOT_IMPLEMENTED, "Metric not implemented in brute force search for Float32 Vector");
    if (cos != (seg->metric == MQVS_METRIC_COSINE))
        fail(MQVS_ERR_LOGICAL, "segment was prepared for a different metric (cosine segments are "
                               "normalised in HBM and serve only cosine searches)");
    if (k > kMaxK) fail(MQVS_ERR_BAD_ARGUMENTS, "k above " + std::to_string(kMaxK) + " not supported");
    mqvs_search_stats st{};
    g_stats = st;
    if (nq == 0 || k == 0) return;
    if (k > kSortCap) {
        // large k: query sub-batches (queries are independent searches)
        const int qb = large_k_batch(seg->n, k);
        if (nq > qb) {
            for (int q0 = 0; q0 < nq; q0 += qb) {
                const int m = std::min(qb, nq - q0);
                search_impl(seg, queries + (size_t)q0 * seg->d, m, k, metric, filter, exists,
                            out_ids + (size_t)q0 * k, out_dist + (size_t)q0 * k, flags, user_stream, force_exact,
                            ord_base, maxv_hint, fnq, async_word);
            }
            return;
        }
    }
    if (maxv_hint > kMaxVariants) {
        // a grown cosine variant table (chains that did not repeat within the
        // default table): its fp32 variants and their bf16 plane are
        // maxv x (4 qstride + 2 dpad) bytes per query -- query sub-batches
        // keep them within the scratch budget (same formula, same bits)
        const int64_t per_q = (int64_t)maxv_hint * (round_up(seg->d, 32) * 4 + round_up(seg->d, kBfK) * 2);
        const int64_t qb = std::max<int64_t>(1, (int64_t)scratch_budget() / per_q);
        if (nq > qb) {
            for (int q0 = 0; q0 < nq; q0 += (int)qb) {
                const int m = (int)std::min<int64_t>(qb, nq - q0);
                search_impl(seg, queries + (size_t)q0 * seg->d, m, k, metric, filter, exists,
                            out_ids + (size_t)q0 * k, out_dist + (size_t)q0 * k, flags, user_stream, force_exact,
                            ord_base, maxv_hint, fnq, async_word);
            }
            return;
        }
    }

    DeviceGuard guard(seg->device);
    Workspace &ws = workspace(seg->device);
    WsCall ws_call(ws);
    hipStream_t s = user_stream ? (hipStream_t)user_stream : ws.stream;
    ws.last = s;
    // a filtered search waits for its selected-row count mid-call: behind
    // earlier work on the caller's stream (e.g. ASYNC searches) it sleeps
    // instead of spinning (below)
    const bool queued_on_entry = filter && hipStreamQuery(s) == hipErrorNotReady;
    const bool dev = flags & MQVS_F_DEVICE_PTRS;
    const int64_t n = seg->n;
    const int d = seg->d;
    const int64_t bm_bytes = (n + 7) / 8;
    const bool timing = call_timing(flags);
    const int batch_mode = call_batch_mode(flags);
    const int gather_mode = call_gather_mode(flags);
    if (timing) MQVS_HIP(hipEventRecord(ws.ev[0], s));

    // ---- inputs on device
    const float *dq = queries;
    const uint8_t *dfilter = filter, *dexists = exists;
    if (!dev) {
        float *q = (float *)ws.get(ws.queries, sizeof(float) * (size_t)nq * d);
        stage_in(ws.pin_q, q, queries, sizeof(float) * (size_t)nq * d, s);
        dq = q;
        if (filter) {
            auto *f = (uint8_t *)ws.get(ws.filter, bm_bytes);
            stage_in(ws.pin_f, f, filter, bm_bytes, s);
            dfilter = f;
        }
        if (exists) {
            auto *f = (uint8_t *)ws.get(ws.exists, bm_bytes);
            stage_in(ws.pin_e, f, exists, bm_bytes, s);
            dexists = f;
        }
    }
    int64_t *dids = out_ids;
    float *ddist = out_dist;
    if (!dev) {
        dids = (int64_t *)ws.get(ws.out_ids, sizeof(int64_t) * (size_t)nq * k);
        ddist = (float *)ws.get(ws.out_dist, sizeof(float) * (size_t)nq * k);
    }

    // ---- selective PREWHERE: count the rows that pass (filter, non-empty,
    // not deleted); a selective scan then walks a gather list of just those
    // rows (per chunk in row order, padded to whole tiles) and reads
    // selectivity x n rows instead of all of them
    static_assert(kSmallRows == kBfRows, "gather-list padding is one tile of either kernel");
    int64_t selected = -1, gpadded = 0;
    int *gcount = nullptr;
    int64_t *goff = nullptr;
    // Cosine pads each chunk's run to whole tiles (a tile's query variant is
    // its chunk's); L2 / IP have one variant, so their list is dense and only
    // its end is padded (at 1 % selectivity per-chunk padding made the list
    // 3x the selected rows: 82 rows per 8192-row chunk, padded to 256)
    const int gtile = cos ? (int)kSmallRows : 1;
    // one zeroed block for the status words: [overflow 4][status 4][count nq]
    // [gather-count ticket 1]
    int *fl = (int *)ws.get(ws.flags, sizeof(int) * (9 + (size_t)nq));
    launch_fill2((uint32_t *)fl, 9 + (int64_t)nq, 0u, nullptr, 0, 0u, s);
    // (armed between the count launch and the host's read of its totals: an
    // exception in between drains the stream, so that no count kernel of this
    // call is still in flight when the next call on this workspace rearms the
    // pinned record)
    struct CountDrain {
        hipStream_t s = nullptr;
        ~CountDrain() {
            if (s) (void)hipStreamSynchronize(s);
        }
    } count_drain;
    int64_t count_gen = 0;
    if (dfilter && gather_mode != 0 && n > 0) {
        const int64_t nch = (n + seg->granule - 1) / seg->granule;
        gcount = (int *)ws.get(ws.gcount, sizeof(int) * nch);
        goff = (int64_t *)ws.get(ws.goff, sizeof(int64_t) * (nch + 2));
        // the totals also land in pinned host memory (k_chunk_count), read once
        // the query prep, chunk ordinals and bf16 query planes are queued: the
        // host waits for this kernel only, not for a drained stream.  The
        // record [padded, selected, generation] is this call's once its
        // generation word (written last, behind a system-scope fence) shows
        // this call's number.
        auto *htot = reinterpret_cast<int64_t *>(ws.host_flags + kCountRec);
        count_gen = ++ws.count_gen;
        htot[2] = 0;
        std::atomic_thread_fence(std::memory_order_seq_cst);
        launch_gather_count(dfilter, seg->nonempty_bits, dexists, n, seg->granule, gtile, gcount, goff, goff + nch,
                            htot, count_gen, fl + 8 + nq, s);
        MQVS_HIP(hipGetLastError());
        count_drain.s = s;
        selected = 0;
        fault_point_mid();
    }
    const bool mfma = fnq >= kBlasThreshold;
    const bool bf16_ok = seg->approx_ok && !force_exact && batch_mode == 0;

    // ---- query prep
    const int64_t ords = (ord_base >= 0 ? ord_base : seg->row_offset / seg->granule) +
                         (n + seg->granule - 1) / seg->granule;
    const int64_t qstride = round_up(d, 32);
    float *qvars = nullptr, *qnorms = nullptr;
    int *qmu = nullptr, *qlam = nullptr, *status = nullptr;
    // The query-variant table starts at kMaxVariants per query without a host
    // round trip; a chain that does not repeat within it on a part of more
    // chunk ordinals (rare: small-integer data) is caught from the status word
    // read at the end, and the search re-runs with the larger table.  (The
    // kernel choice below never changes bf16 from bf16_ok.)
    const int maxv = prep_variants(ws, dq, nq, d, cos, (mfma || bf16_ok) && metric == MQVS_METRIC_L2, ords, false,
                                   qvars, qnorms, qmu, qlam, status, s, fl + 4, maxv_hint);

    // ---- chunk ordinals
    const int *chunk_ord = nullptr;
    if (dfilter) {
        if (cos) {
            const int64_t nch = (n + seg->granule - 1) / seg->granule;
            int *o = (int *)ws.get(ws.ord, sizeof(int) * std::max<int64_t>(nch, 1));
            launch_chunk_ordinals(dfilter, seg->nonempty_bits, dexists, n, seg->granule, 1, o, s);
            MQVS_HIP(hipGetLastError());
            chunk_ord = o;
        }
    } else {
        chunk_ord = seg->chunk_ord;
    }
    // ---- kernel choice
    // faiss's formula branch is set by nq (kBlasThreshold); the bf16
    // pre-filter serves both branches (its exact re-rank uses the branch's
    // formula) whenever the segment has its plane, the exact kernels the rest.  A
    // gathered (selective) scan prefers the bf16 kernel at any nq: its LDS-DMA
    // keeps whole tiles of scattered rows in flight and gathers efficiently up
    // to ~60% selectivity, while the VALU kernel's 128-B row slices only pay
    // below ~30% (tools/sweep.py --sels, profiles/r01)
    // (the bf16 plane streams half the bytes of the fp32 rows, so it serves
    // every batch size)
    // (the gather decision below never changes bf16 from bf16_ok, so the kind
    // and the bf16 query planes are set before the selected count is known)
    const bool bf16 = bf16_ok;
    const int kind = bf16 ? kScanBf16 : !mfma ? kScanSmall : kScanMfma32;

    // ---- candidate capacity per query (a fixed budget spread over the batch)
    int cap = (int)std::min<int64_t>(kCandMax, kCandBudget / std::max(nq, 1));
    cap = std::max(cap, k > kSortCap ? large_k_cap(k) : kSortCap) / 256 * 256;

    ScanParams p{};
    p.rows = seg->rows;
    p.row_norms = seg->norms;
    p.n = n;
    p.d = d;
    p.nq = nq;
    p.qvars = qvars;
    p.qnorms = qnorms;
    p.qmu = qmu;
    p.qlam = qlam;
    p.maxv = maxv;
    p.chunk_rows = seg->granule;
    p.chunk_ord = chunk_ord;
    // a row-range shard of a part continues the part's chunk ordinals (all
    // earlier chunks assumed searched; see DESIGN.md, cosine + shards)
    p.ord_base = (int)(ord_base >= 0 ? ord_base : seg->row_offset / seg->granule);
    p.filter = dfilter;
    p.exists = dexists;
    p.nonempty = seg->nonempty_bits;
    p.num_qblocks = (nq + kMfmaQ - 1) / kMfmaQ;
    p.blas_nq = fnq;
    uint32_t *tau = (uint32_t *)ws.get(ws.tau, sizeof(uint32_t) * nq);
    int *count = fl + 8;  // zeroed with the status words
    Cand *cand = (Cand *)ws.get(ws.cand, sizeof(Cand) * (size_t)nq * cap);
    int *overflow = fl;
    p.tau = tau;
    p.cand_count = count;
    p.cand = cand;
    p.cand_cap = cap;

    float *bq = nullptr;
    if (kind == kScanBf16) {
        // bf16 plane of the query variants + per-query error bound
        const int64_t nvec = (int64_t)nq * maxv;
        bq = (float *)ws.get(ws.bq, sizeof(float) * nq);
        p.rows_hi = seg->rows_hi;
        p.dpad = seg->dpad;
        p.thr = (const float *)ws.get(ws.thr, sizeof(float) * nq);
        p.split = seg->split;
        // batch scans (kernels_p4.hip): per-wave candidate queues
        if (nq > 128) p.p4_queue = ws.get(ws.p4q, p4_queue_bytes());
        {
            // [hi: maxv x vpad x dpad x 2 B][records: nvec x kMxRec floats]
            const int64_t vpad = round_up(nq, 16);
            const int64_t pvec = (int64_t)maxv * vpad;
            const size_t o_rec = (size_t)round_up(pvec * seg->dpad * 2, 256);
            auto *base = (unsigned char *)ws.get(ws.qhi, o_rec + sizeof(float) * kMxRec * (size_t)nvec);
            auto *qhi = (uint16_t *)base;
            auto *qrec = (float *)(base + o_rec);
            launch_to_hi(qvars, nvec, d, qstride, seg->dpad, maxv, vpad, qhi, qrec, nullptr, s);
            p.q_vpad = vpad;
            p.q_hi = qhi;
            launch_query_bound(p, metric, seg->ynorm_max, qrec, seg->ynorm_max + 4, bq, s);
            // cosine batches: a chunk's query variants as one contiguous plane
            // (kernels_p4.hip; up to 32 planes within the scratch budget; the
            // scan keeps per-query variant reads when the chains need more)
            const int64_t plane = vpad * seg->dpad * 2;
            const int pcap = (int)std::min<int64_t>({kP4OrdPlanesMax, maxv, (int64_t)(scratch_budget() / plane)});
            if (p.p4_queue && metric == MQVS_METRIC_COSINE && maxv > 1 && pcap >= 2 && tune_int("MQVS_P4_ORD", 1)) {
                const size_t pb = (size_t)round_up((int64_t)pcap * plane, 256);
                auto *ob = (unsigned char *)ws.get(ws.qord, pb + 256);
                auto *desc = (int *)(ob + pb);
                launch_ord_planes(qhi, (uint16_t *)ob, desc, qmu, qlam, nq, vpad, seg->dpad, pcap, s);
                p.q_ord = (const uint16_t *)ob;
                p.q_ord_desc = desc;
            }
        }
        MQVS_HIP(hipGetLastError());
    }

    // ---- the gather list, launched before the host reads the count (when
    // the call may gather): k_compact_rows needs only the device offsets, and
    // pads the list's end from the device totals, so the host's round trip
    // for the count overlaps it.  Sized for every row (n entries plus the
    // chunks' tile padding); a search the count then sends to the mask scan
    // wasted one compaction beside a scan of >= 60 % of the part.
    // (Parts whose worst-case list passes kSpecListBytes -- 64M rows -- keep
    // the list sized by the count: the workspace peak is what admission
    // reserves for the thread's next call.)
    int32_t *spec_list = nullptr;
    const int64_t nch_all = (n + seg->granule - 1) / seg->granule;
    const int64_t worst = round_up(n + nch_all * (int64_t)(gtile - 1), kSmallRows);
    if (selected >= 0 && (gather_mode == 2 || bf16_ok || (!bf16 && !mfma)) &&
        (size_t)worst * sizeof(int32_t) <= kSpecListBytes) {
        const int64_t nch = nch_all;
        spec_list = (int32_t *)ws.get(ws.glist, sizeof(int32_t) * (size_t)std::max<int64_t>(worst, 1));
        launch_gather_list(dfilter, seg->nonempty_bits, dexists, n, seg->granule, gtile, gcount, goff, spec_list, -1, s,
                           goff + nch, kSmallRows);
        MQVS_HIP(hipGetLastError());
    }

    // ---- the selected count (k_chunk_count's pinned record, polled with a
    // pause for up to kCountSpinUs; then -- or at once behind earlier work on
    // the caller's stream, or in MQVS_WAIT_BLOCK -- the host's wait)
    if (selected >= 0) {
        volatile int64_t *htot = reinterpret_cast<volatile int64_t *>(ws.host_flags + kCountRec);
        const int spin = queued_on_entry || wait_spin_us() == 0 ? 0 : kCountSpinUs;
        const auto t0 = std::chrono::steady_clock::now();
        while (htot[2] != count_gen) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin)) {
                host_wait(s);
                break;
            }
            for (int i = 0; i < 8; ++i) cpu_relax();
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        int64_t tot[2] = {htot[0], htot[1]};
        if (htot[2] != count_gen) {
            // (the pinned record never showed: the device totals, the stream drained)
            const int64_t nch = (n + seg->granule - 1) / seg->granule;
            MQVS_HIP(hipMemcpyAsync(tot, goff + nch, sizeof(tot), hipMemcpyDeviceToHost, s));
            host_wait(s);
        }
        count_drain.s = nullptr;
        gpadded = round_up(tot[0], kSmallRows);
        selected = tot[1];
    }
    bool gather = false;
    if (selected >= 0) {
        if (gather_mode == 2)
            gather = bf16 || !mfma;
        else if (bf16_ok && 10 * selected <= 6 * n)
            gather = true;
        else if (!bf16 && !mfma && 10 * selected <= 3 * n)
            gather = true;
    }

    // ---- gather list of the selected rows
    const int32_t *row_list = nullptr;
    int64_t scan_n = n;  // scan positions: rows, or gather-list entries
    if (gather) {
        int32_t *list = spec_list;
        if (!list) {
            list = (int32_t *)ws.get(ws.glist, sizeof(int32_t) * std::max<int64_t>(gpadded, 1));
            // (the list's tail up to gpadded: -1 entries, written by the last chunk)
            launch_gather_list(dfilter, seg->nonempty_bits, dexists, n, seg->granule, gtile, gcount, goff, list,
                               gpadded, s);
            MQVS_HIP(hipGetLastError());
        }
        row_list = list;
        scan_n = gpadded;
        st.gather = 1;
    }
    const bool aligned = !row_list && (cos || chunk_ord != nullptr);
    const int64_t tile_rows = kind == kScanBf16 ? kBfRows : !mfma ? kSmallRows : kMfmaRows;

    p.row_list = row_list;

    // ---- probe size: expected candidates ~ k*n/P; aim at cap/3
    // (more candidates = more appends from the scan; 16k keeps them cheap)
    const SegTune tune = seg_tune(nq);
    const int64_t target_cands = std::min<int64_t>(cap / 3, std::max<int64_t>(tune.target, 2 * (int64_t)k));
    uint4 *large = k > kSortCap ? (uint4 *)ws.get(ws.large, sizeof(uint4) * 2 * kLargeCap * (size_t)nq) : nullptr;
    int64_t P = scan_n;
    // (small k over a part much larger than k -- e.g. the index build's
    // top-1 k-means assignment against 10^4 centroids -- also takes a short
    // probe: a dense probe of every row would dominate the search)
    if (scan_n > 32768 || (k <= 16 && scan_n > 16 * tile_rows)) {
        P = (int64_t)(((double)k * (double)scan_n) / target_cands) + 1;
        // (a shorter probe is cheaper but its looser threshold sends more
        // waves of the first segments down the append path: measured net
        // loss at nq = 1000 with a 64 MB cap on the probe matrix)
        P = std::max<int64_t>(P, 8 * (int64_t)k);
        // A gathered scan's appends take the per-row path (list lookup,
        // bitmap tests, norms), so a loose first threshold is costly there:
        // at 1 % of 50M rows a 1024-position probe left ~10 % of the first
        // segment's rows passing (110 us for 66k positions, then a 45 us
        // refinement).  A probe of scan_n / 16 positions (<= 16384) costs
        // about the same launch and cuts the first segment's appends ~16x.
        if (row_list) P = std::max<int64_t>(P, std::min<int64_t>(scan_n / 16, 16384));
        P = round_up(P, aligned ? seg->granule : tile_rows);
        if (P > scan_n) P = scan_n;
    }

    // the dense probe of a few queries in kBfRowsSmall-row tiles: 4x the
    // workgroups (a 16384-position probe is 64 tiles of 256 -- a quarter of
    // the CUs, each wave walking four blocks in a row).  Gathered probes at
    // nq <= 16: 34 -> 17 us (1 % of 50M rows, nq 1: 0.447 -> 0.431 ms wall);
    // contiguous ones only at nq <= 2 (cosine 10M, nq 1: 15 -> 12 us; nq 16:
    // 23 -> 27 us), profiles/r05/small_tiles/
    const int64_t ptile =
        (kind == kScanBf16 && (row_list || nq <= 2) && scan_hi_small_tiles_ok(nq, seg->dpad)) ? kBfRowsSmall
                                                                                             : tile_rows;
    const Range pr = make_range(0, P, ptile, seg->granule, aligned);
    if (timing) MQVS_HIP(hipEventRecord(ws.ev[5], s));
    (void)take_batch_kernel_flag();
    // The batch probe (kernels_p4.hip PROBE): the batch kernel over the probe
    // rows writes one best value per (query, 128-row half tile) instead of the
    // dense [nq][P] matrix; the threshold comes from the k-th of those maxima
    // and the main scan then starts at row 0 (the probe rows are re-scanned,
    // ~P / n of the main scan).  Otherwise the dense probe and its select,
    // which also appends the probe rows that pass.
    bool bprobe = false;
    float *probe = nullptr;
    int64_t probe_cols = P, probe_ld = P;
    if (kind == kScanBf16 && p.p4_queue && !row_list && P < scan_n && pr.tiles > 0) {
        const int64_t gld = round_up(2 * pr.tiles, 4);
        probe = (float *)ws.get(ws.probe, sizeof(float) * (size_t)nq * gld);
        ScanParams pp = p;
        pp.row_begin = pr.begin;
        pp.row_end = pr.end;
        pp.tiles = pr.tiles;
        pp.tiles_per_chunk = pr.tiles_per_chunk;
        pp.tile_rows = kBfRows;
        pp.p4_gmax = probe;
        pp.p4_gld = gld;
        bprobe = launch_scan_p4_probe(pp, metric, s);
        MQVS_HIP(hipGetLastError());
        if (bprobe) {
            probe_cols = 2 * pr.tiles;
            probe_ld = gld;
        }
    }
    if (!bprobe) {
        probe = (float *)ws.get(ws.probe, sizeof(float) * (size_t)nq * P);
        p.probe = probe;
        p.probe_ld = P;
        run_scan(p, pr, kind, metric, true, s, ptile);
    }
    if (timing) MQVS_HIP(hipEventRecord(ws.ev[1], s));
    if (kind == kScanBf16)
        launch_probe_select_approx(probe, probe_cols, probe_ld, nq, k, metric, bq, (float *)p.thr, count,
                                   bprobe ? nullptr : cand, cap, row_list, s);
    else
        launch_probe_select(probe, P, P, nq, k, metric, tau, count, cand, cap, 0, row_list, s);
    MQVS_HIP(hipGetLastError());
    if (timing) MQVS_HIP(hipEventRecord(ws.ev[2], s));
    // main scan in geometrically growing segments; between segments the
    // threshold tightens from the candidates so far and the lists compact
    // into the other buffer (keeps appends and list lengths small when the
    // probe's threshold is loose, e.g. clustered data)
    {
        const int64_t align = aligned ? seg->granule : tile_rows;
        Cand *alt = (Cand *)ws.get(ws.cand2, sizeof(Cand) * (size_t)nq * cap);
        int *calt = (int *)ws.get(ws.count2, sizeof(int) * nq);
        // (the batch probe appended nothing: the first segment also covers
        // the probe rows)
        // (a segment of fewer than kMinSegRows rows cannot fill the chip --
        // 256 tiles -- and costs a launch and a refinement: small-k searches
        // over mid-size parts, e.g. the index's coarse step, 39063 centroids
        // at k = nprobe, used to run 7 segments of 2..64 tiles)
        int64_t b = bprobe ? 0 : P, seg_rows = std::max<int64_t>({tune.first * P, align, kMinSegRows});
        int segs = 0;
        // dense gathered lists (L2 / IP) at nq <= 16: segments of at most
        // 2^19 positions in kBfRowsSmall-row tiles too (a gathered row costs
        // a list lookup before its loads; 4x the waves in flight hide it):
        // 1 % of 50M rows, nq 1: 0.420 -> 0.404 ms.  Not for cosine lists,
        // padded per chunk to whole 256-row tiles (4x the workgroups, most
        // of them padding: 1 %, nq 1 0.50 -> 0.68 ms), nor long segments
        // (L2 50 %, nq 16: 8.79 -> 9.01 ms); profiles/r05/small_tiles/main_ab.jsonl
        const bool small_main = kind == kScanBf16 && row_list && !cos &&
                                tune_int("MQVS_HI_SMALL_MAIN", 1) == 1 && scan_hi_small_tiles_ok(nq, seg->dpad);
        while (b < scan_n) {
            const int64_t e = std::min(scan_n, round_up(b + seg_rows + (segs == 0 && bprobe ? P : 0), align));
            const bool tev = timing && 2 * segs + 1 < Workspace::kSegEv;
            if (tev) MQVS_HIP(hipEventRecord(ws.seg_ev[2 * segs], s));
            const int64_t mtile = (small_main && e - b <= (int64_t)1 << 19) ? kBfRowsSmall : tile_rows;
            run_scan(p, make_range(b, e, mtile, seg->granule, aligned), kind, metric, false, s, mtile);
            if (tev) MQVS_HIP(hipEventRecord(ws.seg_ev[2 * segs + 1], s));
            b = e;
            seg_rows *= tune.growth;
            ++segs;
            if (b < scan_n) {
                launch_refine(cand, count, cap, nq, k, metric, kind == kScanBf16, bq, tau,
                              (float *)p.thr, alt, calt, s);
                MQVS_HIP(hipGetLastError());
                std::swap(cand, alt);
                std::swap(count, calt);
                p.cand = cand;
                p.cand_count = count;
            }
        }
        st.segments = segs;
    }
    if (timing) MQVS_HIP(hipEventRecord(ws.ev[3], s));
    bool flags_folded = false;  // the status words stored by the final select (k_sort_emit)
    if (kind == kScanBf16) {
        // survivors of the bound: up to kSortCap per query (kLargeCap with
        // the global-scratch sort for k > kSortCap)
        const int lcap = large ? kLargeCap : kSortCap;
        const int64_t rs = large ? 2 * (int64_t)kLargeCap : kSortCap;
        auto *surv = (uint32_t *)ws.get(ws.surv, sizeof(uint32_t) * (size_t)nq * rs + sizeof(int) * nq);
        int *scnt = (int *)(surv + (size_t)nq * rs);
        uint4 *recs = large ? large : (uint4 *)ws.get(ws.recs, sizeof(uint4) * (size_t)nq * rs);
        // (a synchronous call: the final select also stores the status words
        // into the pinned record the host reads after its wait)
        const bool fold = !(dev && (flags & MQVS_F_ASYNC));
        launch_rerank_select(p, metric, bq, k, seg->row_offset, dids, ddist, overflow, surv, scnt, recs, lcap, rs,
                             s, fold ? fl : nullptr, fold ? ws.host_flags + 16 : nullptr);
        flags_folded = fold;
    } else
        launch_final_select(cand, count, cap, nq, k, metric, seg->granule, seg->row_offset, dids, ddist,
                            overflow, large, s);
    MQVS_HIP(hipGetLastError());
    if (timing) MQVS_HIP(hipEventRecord(ws.ev[4], s));

    st.path = kind;
    st.prefilter = kind == kScanBf16 ? seg->split : 0;
    st.batch_kernel = take_batch_kernel_flag();
    st.probe_rows = P;
    st.main_rows = bprobe ? scan_n : scan_n - P;
    st.rows_scanned = scan_n;
    st.nq = nq;
    st.k = k;

    const bool async = dev && (flags & MQVS_F_ASYNC);
    ws.pending_timing = false;
    if (async) {
        // no host fallback possible: leave the outcome for mqvs_async_check
        // (or the caller's word)
        const bool variants_matter = ords > maxv;
        launch_async_flags(overflow, status, variants_matter ? 1 : 0, async_word ? async_word : sticky_word(ws, s),
                           s);
        MQVS_HIP(hipGetLastError());
        if (async_word) {
            // the survivor stats land in pinned memory, read after the
            // caller's sync (search_collect_stats)
            MQVS_HIP(hipMemcpyAsync(ws.host_flags + 16, fl, 8 * sizeof(int), hipMemcpyDeviceToHost, s));
            ws.pending_timing = timing;
            ws.pending_bf16 = kind == kScanBf16;
        }
    } else {
        // [overflow 4][status 4] in one copy -> host_flags[0] overflow bits,
        // [1] status, [4..6] survivor / candidate stats
        // (host outputs: copied with the status words, one wait)
        if (!dev) stage_out_begin(ws.pin_o, dids, ddist, (size_t)nq * k, s);
        // (stored by the final select when it could; else a one-wave kernel
        // storing into the pinned words -- the runtime's device-to-host copy
        // is a 4.4 us blit kernel at the end of every search)
        if (!flags_folded) {
            launch_words_to_host(nullptr, 0, fl, 8, nullptr, ws.host_flags + 16, s);
            MQVS_HIP(hipGetLastError());
        }
        host_wait(s);
        ws.host_flags[0] = ws.host_flags[16];
        ws.host_flags[1] = ws.host_flags[20];
        ws.host_flags[4] = ws.host_flags[17];
        ws.host_flags[5] = ws.host_flags[18];
        ws.host_flags[6] = ws.host_flags[19];
        if (kind == kScanBf16) {
            st.survivors_max = ws.host_flags[4];
            st.survivors_total = (uint32_t)ws.host_flags[5];
            st.candidates_max = ws.host_flags[6];
        }
        // a query whose re-normalisation does not repeat within maxv steps is
        // exact only on the part's first maxv chunk ordinals (maxv covers
        // every ordinal unless the part has more than kMaxVariantsCap chunks)
        if (ws.host_flags[1] && ords > maxv) {
            const int want = (int)std::min<int64_t>(ords, kMaxVariantsCap);
            if (maxv < want) {
                search_impl(seg, queries, nq, k, metric, filter, exists, out_ids, out_dist, flags, user_stream,
                            force_exact, ord_base, want, fnq);
                return;
            }
            fail(MQVS_ERR_LOGICAL, "cosine query normalisation did not repeat within " + std::to_string(maxv) +
                                       " steps on a part of more chunks");
        }
        if (kind == kScanBf16 && ws.host_flags[0]) {
            // the bf16 bound left too many candidates: exact fp32 path
            search_impl(seg, queries, nq, k, metric, filter, exists, out_ids, out_dist, flags,
                        user_stream, true, ord_base, maxv, fnq);
            g_stats.rescans += 1;
            return;
        }
        int rescans = 0;
        while (ws.host_flags[0]) {
            if (++rescans > 3)
                fail(MQVS_ERR_LOGICAL, "candidate overflow: more than " + std::to_string(cap) +
                                           " rows tie at the k-th distance");
            launch_cand_tau(cand, count, cap, nq, k, metric, tau, nullptr, s);
            launch_fill2((uint32_t *)count, nq, 0u, (uint32_t *)overflow, 4, 0u, s);
            run_scan(p, make_range(0, scan_n, tile_rows, seg->granule, aligned), kind, metric, false, s);
            launch_final_select(cand, count, cap, nq, k, metric, seg->granule, seg->row_offset, dids,
                                ddist, overflow, large, s);
            MQVS_HIP(hipGetLastError());
            MQVS_HIP(hipMemcpyAsync(ws.host_flags, overflow, sizeof(int), hipMemcpyDeviceToHost, s));
            host_wait(s);
        }
        st.rescans = rescans;
        if (!dev && rescans)
            stage_out_results(ws.pin_o, out_ids, out_dist, dids, ddist, (size_t)nq * k, s);
        else if (!dev)
            stage_out_end(ws.pin_o, out_ids, out_dist, (size_t)nq * k);
        if (timing) read_search_times(ws, st);
    }
    g_stats = st;
}

// the stats of this thread's last search_segment_async on `device`, once the
// caller has synchronised its stream
void search_collect_stats(int device) {
    Workspace &ws = workspace(device);
    WsCall ws_call(ws);
    if (ws.pending_bf16) {
        g_stats.survivors_max = ws.host_flags[17];
        g_stats.survivors_total = (uint32_t)ws.host_flags[18];
        g_stats.candidates_max = ws.host_flags[19];
    }
    if (ws.pending_timing) read_search_times(ws, g_stats);
    ws.pending_timing = ws.pending_bf16 = false;
}

// the search for other translation units (sharded.hip): device pointers,
// caller stream, explicit chunk-ordinal base
void search_segment(mqvs_segment *seg, const float *queries, int nq, int k, int metric, const uint8_t *filter,
                    const uint8_t *exists, int64_t *out_ids, float *out_dist, uint32_t flags, hipStream_t stream,
                    int64_t ord_base) {
    search_impl(seg, queries, nq, k, metric, filter, exists, out_ids, out_dist, flags | MQVS_F_DEVICE_PTRS, stream,
                false, ord_base);
}

// the same without any host sync: fallback flags OR-ed into *flag_word
// (bit 0 candidate overflow, bit 1 cosine variant table too short), stats
// collected by search_collect_stats after the caller's sync
void search_segment_async(mqvs_segment *seg, const float *queries, int nq, int k, int metric, const uint8_t *filter,
                          const uint8_t *exists, int64_t *out_ids, float *out_dist, uint32_t flags,
                          hipStream_t stream, int64_t ord_base, int *flag_word) {
    search_impl(seg, queries, nq, k, metric, filter, exists, out_ids, out_dist,
                flags | MQVS_F_DEVICE_PTRS | MQVS_F_ASYNC, stream, false, ord_base, 0, 0, flag_word);
}

// Exact re-rank of caller-given candidate rows (computeTopDistanceSubset
// contract, VIWithDataPart.cpp:838-856): the distance formula and cosine
// query variant mqvs_search uses for the same batch size, then top-k by the
// reference key.  Rows < 0, >= n or deleted (row_exists) are skipped; the
// candidate list of a query is expected to hold distinct rows.
static void rerank_impl(mqvs_segment *seg, const float *queries, int nq, const int64_t *cand,
                        int ncand, int k, int metric, const uint8_t *exists, int64_t *out_ids,
                        float *out_dist, uint32_t flags, hipStream_t user_stream, int formula_nq = 0) {
    const int fnq = formula_nq > 0 ? formula_nq : nq;  // (see search_impl)
    if (!seg) fail(MQVS_ERR_BAD_ARGUMENTS, "null segment");
    if (seg->binary) fail(MQVS_ERR_NOT_IMPLEMENTED, "computeTopDistanceSubset is for Float32 vectors");
    if (nq < 0 || k < 0 || ncand < 0) fail(MQVS_ERR_BAD_ARGUMENTS, "nq, k and ncand must be non-negative");
    const bool cos = metric == MQVS_METRIC_COSINE;
    if (metric != MQVS_METRIC_L2 && metric != MQVS_METRIC_IP && !cos)
        fail(MQVS_ERR_NOT_IMPLEMENTED, "Metric not implemented in brute force search for Float32 Vector");
    if (cos != (seg->metric == MQVS_METRIC_COSINE))
        fail(MQVS_ERR_LOGICAL, "segment was prepared for a different metric");
    if (k > kMaxK || ncand > kLargeCap)
        fail(MQVS_ERR_BAD_ARGUMENTS, "k must not exceed " + std::to_string(kMaxK) + " and ncand " +
                                         std::to_string(kLargeCap));
    if (nq > 0 && k > 0 && (!queries || !out_ids || !out_dist || (ncand > 0 && !cand)))
        fail(MQVS_ERR_BAD_ARGUMENTS, "null query, candidate or output pointer");
    g_stats = mqvs_search_stats{};
    if (nq == 0 || k == 0) return;
    // more candidates than the LDS sort holds: each query's records are sorted
    // through 2 ncand records of global scratch, in query sub-batches of <= 1 GB
    const bool large = ncand > kSortCap;
    if (large) {
        const int qb = (int)std::max<int64_t>(1, (int64_t)scratch_budget() / 16 / (2 * (int64_t)ncand));
        if (nq > qb) {
            for (int q0 = 0; q0 < nq; q0 += qb) {
                const int m = std::min(qb, nq - q0);
                rerank_impl(seg, queries + (size_t)q0 * seg->d, m, cand + (size_t)q0 * ncand, ncand, k, metric,
                            exists, out_ids + (size_t)q0 * k, out_dist + (size_t)q0 * k, flags, user_stream, fnq);
            }
            return;
        }
    }

    DeviceGuard guard(seg->device);
    Workspace &ws = workspace(seg->device);
    WsCall ws_call(ws);
    hipStream_t s = user_stream ? (hipStream_t)user_stream : ws.stream;
    ws.last = s;
    const bool dev = flags & MQVS_F_DEVICE_PTRS;
    const int d = seg->d;
    const float *dq = queries;
    const int64_t *dc = cand;
    const uint8_t *dexists = exists;
    int64_t *dids = out_ids;
    float *ddist = out_dist;
    if (!dev) {
        float *q = (float *)ws.get(ws.queries, sizeof(float) * (size_t)nq * d);
        stage_in(ws.pin_q, q, queries, sizeof(float) * (size_t)nq * d, s);
        dq = q;
        int64_t *c = (int64_t *)ws.get(ws.misc, sizeof(int64_t) * std::max<size_t>((size_t)nq * ncand, 1));
        if (ncand > 0) stage_in(ws.pin_f, c, cand, sizeof(int64_t) * (size_t)nq * ncand, s);
        dc = c;
        if (exists) {
            const int64_t bm = (seg->n + 7) / 8;
            auto *f = (uint8_t *)ws.get(ws.exists, bm);
            stage_in(ws.pin_e, f, exists, bm, s);
            dexists = f;
        }
        dids = (int64_t *)ws.get(ws.out_ids, sizeof(int64_t) * (size_t)nq * k);
        ddist = (float *)ws.get(ws.out_dist, sizeof(float) * (size_t)nq * k);
    }
    const bool blas = fnq >= kBlasThreshold;
    const int64_t ords = seg->row_offset / seg->granule + (seg->n + seg->granule - 1) / seg->granule;
    float *qvars = nullptr, *qnorms = nullptr;
    int *qmu = nullptr, *qlam = nullptr, *status = nullptr;
    const int maxv = prep_variants(ws, dq, nq, d, cos, blas && metric == MQVS_METRIC_L2, ords,
                                   !(dev && (flags & MQVS_F_ASYNC)), qvars, qnorms, qmu, qlam, status, s);

    ScanParams p{};
    p.rows = seg->rows;
    p.row_norms = seg->norms;
    p.n = seg->n;
    p.d = d;
    p.nq = nq;
    p.qvars = qvars;
    p.qnorms = qnorms;
    p.qmu = qmu;
    p.qlam = qlam;
    p.maxv = maxv;
    p.blas_nq = fnq;
    p.chunk_rows = seg->granule;
    p.chunk_ord = seg->chunk_ord;
    p.ord_base = (int)(seg->row_offset / seg->granule);
    p.exists = dexists;
    p.nonempty = seg->nonempty_bits;
    uint4 *scratch = large ? (uint4 *)ws.get(ws.large, sizeof(uint4) * 2 * (size_t)ncand * nq) : nullptr;
    launch_rerank_ids(p, metric, dc, ncand, k, seg->row_offset, dids, ddist, scratch, s);
    MQVS_HIP(hipGetLastError());
    if (dev && (flags & MQVS_F_ASYNC)) {
        launch_async_flags(nullptr, status, ords > maxv ? 1 : 0, sticky_word(ws, s), s);
        MQVS_HIP(hipGetLastError());
        return;
    }
    if (!dev) stage_out_begin(ws.pin_o, dids, ddist, (size_t)nq * k, s);
    MQVS_HIP(hipMemcpyAsync(ws.host_flags, status, sizeof(int), hipMemcpyDeviceToHost, s));
    host_wait(s);
    if (ws.host_flags[0] && ords > maxv)
        fail(MQVS_ERR_LOGICAL, "cosine query normalisation did not repeat within " + std::to_string(maxv) +
                                   " steps on a part of more chunks");
    if (!dev) stage_out_end(ws.pin_o, out_ids, out_dist, (size_t)nq * k);
}


// ---------------------------------------------------------------------------
// binary vectors: vectorScanWithoutIndex<BinaryVector> for one part
// (MergeTreeVSManager.cpp:1188-1273 filtered gather, :1395-1425 whole chunks)
// on the same probe / threshold / append / select pipeline as the float VALU
// path, with the popcount scan of kernels_binary.hip and the L2 ordering key
// (both binary distances are ascending and finite).  No granule chunking is
// needed: the reference's per-chunk strict merges keep the k best by
// (distance, row) over the part, like the float L2 path.

static mqvs_segment *new_binary_segment(int64_t n, int32_t dim_bits, int32_t metric, int64_t granule,
                                        int64_t row_offset) {
    if (n < 0 || n >= ((int64_t)1 << 32)) fail(MQVS_ERR_BAD_ARGUMENTS, "segment rows must be in [0, 2^32)");
    if (dim_bits <= 0 || dim_bits % 8 != 0)
        fail(MQVS_ERR_BAD_ARGUMENTS, "binary vector dimension must be a positive multiple of 8 bits");
    if (metric != MQVS_METRIC_HAMMING && metric != MQVS_METRIC_JACCARD)
        fail(MQVS_ERR_NOT_IMPLEMENTED, "Metric not implemented in brute force search for Binary Vector");
    if (granule <= 0) fail(MQVS_ERR_BAD_ARGUMENTS, "granule_rows must be positive");
    if (row_offset < 0 || row_offset % granule != 0)
        fail(MQVS_ERR_BAD_ARGUMENTS, "row_offset must be a non-negative multiple of granule_rows");
    auto *s = new mqvs_segment();
    MQVS_HIP(hipGetDevice(&s->device));
    s->binary = true;
    s->n = n;
    s->d = dim_bits;
    s->metric = metric;
    s->granule = granule;
    s->row_offset = row_offset;
    s->code_bytes = dim_bits / 8;
    s->code_words = (int)round_up((s->code_bytes + 3) / 4, 4);
    const size_t bytes = (size_t)std::max<int64_t>(n, 1) * s->code_words * 4;
    if (hipMalloc((void **)&s->codes, bytes) != hipSuccess) {
        (void)hipGetLastError();
        delete s;
        fail(MQVS_ERR_MEMORY_LIMIT, "HBM allocation of " + std::to_string(bytes) + " bytes failed");
    }
    s->bytes = bytes;
    return s;
}

// rows of `nbytes` (host or device) -> zero-padded [n][words] on the device
static void upload_codes(uint32_t *dst, int words, const uint8_t *src, int64_t nbytes, int64_t n, bool dev,
                         hipStream_t s) {
    if (n <= 0) return;
    MQVS_HIP(hipMemsetAsync(dst, 0, (size_t)n * words * 4, s));
    MQVS_HIP(hipMemcpy2DAsync(dst, (size_t)words * 4, src, (size_t)nbytes, (size_t)nbytes, (size_t)n,
                              dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s));
}

static void search_binary_impl(mqvs_segment *seg, const uint8_t *queries, int nq, int k, int metric,
                               const uint8_t *filter, const uint8_t *exists, int64_t *out_ids, float *out_dist,
                               uint32_t flags, hipStream_t user_stream) {
    if (!seg) fail(MQVS_ERR_BAD_ARGUMENTS, "null segment");
    if (!seg->binary) fail(MQVS_ERR_LOGICAL, "Float32 segment: search it with mqvs_search");
    if (metric != MQVS_METRIC_HAMMING && metric != MQVS_METRIC_JACCARD)
        fail(MQVS_ERR_NOT_IMPLEMENTED, "Metric not implemented in brute force search for Binary Vector");
    if (nq < 0 || k < 0) fail(MQVS_ERR_BAD_ARGUMENTS, "nq and k must be non-negative");
    if (k > kMaxK) fail(MQVS_ERR_BAD_ARGUMENTS, "k above " + std::to_string(kMaxK) + " not supported");
    if (nq > 0 && k > 0 && (!queries || !out_ids || !out_dist))
        fail(MQVS_ERR_BAD_ARGUMENTS, "null query or output pointer");
    mqvs_search_stats st{};
    g_stats = st;
    if (nq == 0 || k == 0) return;
    if (k > kSortCap) {
        const int qb = large_k_batch(seg->n, k);
        if (nq > qb) {
            for (int q0 = 0; q0 < nq; q0 += qb) {
                const int m = std::min(qb, nq - q0);
                search_binary_impl(seg, queries + (size_t)q0 * seg->code_bytes, m, k, metric, filter, exists,
                                   out_ids + (size_t)q0 * k, out_dist + (size_t)q0 * k, flags, user_stream);
            }
            return;
        }
    }

    DeviceGuard guard(seg->device);
    Workspace &ws = workspace(seg->device);
    WsCall ws_call(ws);
    hipStream_t s = user_stream ? (hipStream_t)user_stream : ws.stream;
    ws.last = s;
    const bool dev = flags & MQVS_F_DEVICE_PTRS;
    const int64_t n = seg->n;
    const int64_t bm_bytes = (n + 7) / 8;
    const bool timing = call_timing(flags);
    if (timing) MQVS_HIP(hipEventRecord(ws.ev[0], s));

    uint32_t *qc = (uint32_t *)ws.get(ws.queries, (size_t)nq * seg->code_words * 4);
    upload_codes(qc, seg->code_words, queries, seg->code_bytes, nq, dev, s);
    const uint8_t *dfilter = filter, *dexists = exists;
    if (!dev) {
        if (filter) {
            auto *f = (uint8_t *)ws.get(ws.filter, bm_bytes);
            stage_in(ws.pin_f, f, filter, bm_bytes, s);
            dfilter = f;
        }
        if (exists) {
            auto *f = (uint8_t *)ws.get(ws.exists, bm_bytes);
            stage_in(ws.pin_e, f, exists, bm_bytes, s);
            dexists = f;
        }
    }
    int64_t *dids = out_ids;
    float *ddist = out_dist;
    if (!dev) {
        dids = (int64_t *)ws.get(ws.out_ids, sizeof(int64_t) * (size_t)nq * k);
        ddist = (float *)ws.get(ws.out_dist, sizeof(float) * (size_t)nq * k);
    }

    // candidate capacity and probe size as the float path (mqvs.hip search_impl)
    constexpr int64_t tile_rows = kSmallRows;
    int cap = (int)std::min<int64_t>(kCandMax, kCandBudget / std::max(nq, 1));
    cap = std::max(cap, k > kSortCap ? large_k_cap(k) : kSortCap) / 256 * 256;
    const int64_t target_cands = std::min<int64_t>(cap / 3, std::max<int64_t>(16384, 2 * (int64_t)k));
    uint4 *large = k > kSortCap ? (uint4 *)ws.get(ws.large, sizeof(uint4) * 2 * kLargeCap * (size_t)nq) : nullptr;
    int64_t P = n;
    if (n > 32768) {
        P = (int64_t)(((double)k * (double)n) / target_cands) + 1;
        // the refines between main segments keep appends near 2k per segment
        // whatever the probe, so the probe stays short on big parts (its select
        // is one workgroup per query)
        P = std::min<int64_t>(P, std::max<int64_t>(nq <= 8 ? 16384 : 65536, 8 * (int64_t)k));
        P = std::max<int64_t>(P, 8 * (int64_t)k);
        P = round_up(P, tile_rows);
        if (P > n) P = n;
    }
    ScanParams p{};
    p.n = n;
    p.nq = nq;
    p.chunk_rows = seg->granule;
    p.filter = dfilter;
    p.exists = dexists;
    p.codes = seg->codes;
    p.qcodes = qc;
    p.code_words = seg->code_words;
    p.nbits = seg->d;
    uint32_t *tau = (uint32_t *)ws.get(ws.tau, sizeof(uint32_t) * nq);
    int *count = (int *)ws.get(ws.count, sizeof(int) * nq);
    Cand *cand = (Cand *)ws.get(ws.cand, sizeof(Cand) * (size_t)nq * cap);
    int *overflow = (int *)ws.get(ws.overflow, sizeof(int) * 4);
    p.tau = tau;
    p.cand_count = count;
    p.cand = cand;
    p.cand_cap = cap;
    p.probe = (float *)ws.get(ws.probe, sizeof(float) * (size_t)nq * std::max<int64_t>(P, 1));
    p.probe_ld = P;
    auto scan = [&](int64_t b, int64_t e, bool probe, bool strict) {
        const Range r = make_range(b, e, tile_rows, seg->granule, false);
        if (r.tiles <= 0) return;
        p.row_begin = r.begin;
        p.row_end = r.end;
        p.tiles = r.tiles;
        p.tiles_per_chunk = 0;
        p.tile_rows = tile_rows;
        p.tau_strict = strict ? 1 : 0;
        launch_scan_binary(p, metric, probe, s);
        MQVS_HIP(hipGetLastError());
    };
    constexpr int kOrder = MQVS_METRIC_L2;  // ascending finite values: ord_asc key, (key, row) ties
    if (timing) MQVS_HIP(hipEventRecord(ws.ev[5], s));
    scan(0, P, true, false);
    if (timing) MQVS_HIP(hipEventRecord(ws.ev[1], s));
    launch_fill2((uint32_t *)count, nq, 0u, nullptr, 0, 0u, s);
    launch_probe_select(p.probe, P, P, nq, k, kOrder, tau, count, cand, cap, 0, nullptr, s);
    MQVS_HIP(hipGetLastError());
    if (timing) MQVS_HIP(hipEventRecord(ws.ev[2], s));
    {
        Cand *alt = (Cand *)ws.get(ws.cand2, sizeof(Cand) * (size_t)nq * cap);
        int *calt = (int *)ws.get(ws.count2, sizeof(int) * nq);
        // segments grow x4: each refine costs a launch, and appends per
        // segment stay near (growth x k) with the threshold refined
        int64_t b = P, seg_rows = std::max<int64_t>(2 * P, tile_rows);
        int segs = 0;
        while (b < n) {
            const int64_t e = std::min(n, round_up(b + seg_rows, tile_rows));
            scan(b, e, false, true);
            b = e;
            seg_rows *= 4;
            ++segs;
            if (b < n) {
                launch_refine(cand, count, cap, nq, k, kOrder, false, nullptr, tau, nullptr, alt, calt, s);
                MQVS_HIP(hipGetLastError());
                std::swap(cand, alt);
                std::swap(count, calt);
                p.cand = cand;
                p.cand_count = count;
            }
        }
        st.segments = segs;
    }
    if (timing) MQVS_HIP(hipEventRecord(ws.ev[3], s));
    launch_fill2((uint32_t *)overflow, 4, 0u, nullptr, 0, 0u, s);
    launch_final_select(cand, count, cap, nq, k, kOrder, 0, seg->row_offset, dids, ddist, overflow, large, s);
    MQVS_HIP(hipGetLastError());
    if (timing) MQVS_HIP(hipEventRecord(ws.ev[4], s));
    st.path = 3;  // binary popcount scan
    st.probe_rows = P;
    st.main_rows = n - P;
    st.rows_scanned = n;
    st.nq = nq;
    st.k = k;
    const bool async = dev && (flags & MQVS_F_ASYNC);
    if (async) {
        launch_async_flags(overflow, nullptr, 0, sticky_word(ws, s), s);
        MQVS_HIP(hipGetLastError());
    } else {
        if (!dev) stage_out_begin(ws.pin_o, dids, ddist, (size_t)nq * k, s);
        MQVS_HIP(hipMemcpyAsync(ws.host_flags, overflow, sizeof(int), hipMemcpyDeviceToHost, s));
        host_wait(s);
        int rescans = 0;
        while (ws.host_flags[0]) {
            // a list overflowed its capacity: tighten tau from what was kept and
            // rescan the part inclusively (rare: > cap rows at or under the
            // probe threshold)
            if (++rescans > 3)
                fail(MQVS_ERR_LOGICAL, "candidate overflow: more than " + std::to_string(cap) +
                                           " rows tie at the k-th distance");
            launch_cand_tau(cand, count, cap, nq, k, kOrder, tau, nullptr, s);
            launch_fill2((uint32_t *)count, nq, 0u, (uint32_t *)overflow, 4, 0u, s);
            scan(0, n, false, false);
            launch_final_select(cand, count, cap, nq, k, kOrder, 0, seg->row_offset, dids, ddist, overflow, large,
                                s);
            MQVS_HIP(hipGetLastError());
            MQVS_HIP(hipMemcpyAsync(ws.host_flags, overflow, sizeof(int), hipMemcpyDeviceToHost, s));
            host_wait(s);
        }
        st.rescans = rescans;
        if (!dev && rescans)
            stage_out_results(ws.pin_o, out_ids, out_dist, dids, ddist, (size_t)nq * k, s);
        else if (!dev)
            stage_out_end(ws.pin_o, out_ids, out_dist, (size_t)nq * k);
        if (timing) {
            float a = 0, b = 0, c = 0, e = 0, f = 0;
            MQVS_HIP(hipEventElapsedTime(&a, ws.ev[5], ws.ev[1]));
            MQVS_HIP(hipEventElapsedTime(&b, ws.ev[1], ws.ev[2]));
            MQVS_HIP(hipEventElapsedTime(&c, ws.ev[2], ws.ev[3]));
            MQVS_HIP(hipEventElapsedTime(&e, ws.ev[3], ws.ev[4]));
            MQVS_HIP(hipEventElapsedTime(&f, ws.ev[0], ws.ev[4]));
            st.probe_ms = a;
            st.probe_select_ms = b;
            st.main_ms = c;
            st.final_ms = e;
            st.total_ms = f;
        }
    }
    g_stats = st;
}


// ---------------------------------------------------------------------------
// column ingest: the compressed files of a part's Array(Float32) column,
// decoded in HBM (kernels_ingest.hip) into the rows matrix + nonempty flags of
// MergeTreeVSManager.cpp:1381-1393, then prepared like any segment.

struct IngestTmp {
    std::vector<void *> bufs;
    void *alloc(size_t bytes) {
        void *p = nullptr;
        if (hipMalloc(&p, std::max<size_t>(bytes, 16)) != hipSuccess) {
            (void)hipGetLastError();
            fail(MQVS_ERR_MEMORY_LIMIT, "HBM allocation of " + std::to_string(bytes) + " bytes failed");
        }
        bufs.push_back(p);
        return p;
    }
    // side stream for the block checksums (overlaps the decode; joined before
    // the status is read)
    hipStream_t side = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    ~IngestTmp() {
        if (side) (void)hipStreamSynchronize(side);
        for (void *p : bufs) (void)hipFree(p);
        if (fork) (void)hipEventDestroy(fork);
        if (join) (void)hipEventDestroy(join);
        if (side) (void)hipStreamDestroy(side);
    }
};

// block table of one compressed stream; returns (blocks, decompressed bytes)
static std::pair<int64_t, int64_t> stream_table(IngestTmp &tmp, const uint8_t *dsrc, int64_t n, IngestBlock **tab,
                                                int64_t *hbuf, const char *what, hipStream_t s) {
    const int64_t maxb = n / 25 + 1;
    *tab = (IngestBlock *)tmp.alloc(sizeof(IngestBlock) * (size_t)maxb);
    int64_t *dout = (int64_t *)tmp.alloc(4 * sizeof(int64_t));
    launch_block_table(dsrc, n, *tab, maxb, dout, s);
    MQVS_HIP(hipGetLastError());
    MQVS_HIP(hipMemcpyAsync(hbuf, dout, 3 * sizeof(int64_t), hipMemcpyDeviceToHost, s));
    host_wait(s);
    if (hbuf[2] == 2)
        fail(MQVS_ERR_NOT_IMPLEMENTED, std::string(what) + ": compression method other than LZ4 / NONE");
    if (hbuf[2])
        fail(MQVS_ERR_ILLEGAL_COLUMN, std::string(what) + ": malformed compressed block chain (CANNOT_DECOMPRESS)");
    return {hbuf[0], hbuf[1]};
}

constexpr int kBadDataChecksum = 8, kBadSizesChecksum = 16;  // status bits (decode uses 4)

static mqvs_segment *ingest_column(const uint8_t *data_bin, int64_t data_bytes, const uint8_t *sizes_bin,
                                   int64_t sizes_bytes, int64_t n, int32_t d, int32_t metric, int64_t granule,
                                   int64_t row_offset, uint32_t flags) {
    check_seg_args(n, d, metric, granule, row_offset);
    if (data_bytes < 0 || sizes_bytes < 0) fail(MQVS_ERR_BAD_ARGUMENTS, "negative stream size");
    if ((data_bytes > 0 && !data_bin) || (sizes_bytes > 0 && !sizes_bin))
        fail(MQVS_ERR_BAD_ARGUMENTS, "null column stream");
    const bool dev = flags & MQVS_F_DEVICE_PTRS;
    mqvs_segment *seg = new_segment(n, d, metric, granule, row_offset);
    try {
        Workspace &ws = workspace(seg->device);
        WsCall ws_call(ws);
        hipStream_t s = ws.stream;
        IngestTmp tmp;
        const uint8_t *dd = data_bin, *ds = sizes_bin;
        if (!dev) {
            auto *a = (uint8_t *)tmp.alloc((size_t)data_bytes);
            auto *b = (uint8_t *)tmp.alloc((size_t)sizes_bytes);
            if (data_bytes) MQVS_HIP(hipMemcpyAsync(a, data_bin, (size_t)data_bytes, hipMemcpyHostToDevice, s));
            if (sizes_bytes) MQVS_HIP(hipMemcpyAsync(b, sizes_bin, (size_t)sizes_bytes, hipMemcpyHostToDevice, s));
            dd = a;
            ds = b;
        }
        int64_t *h = reinterpret_cast<int64_t *>(ws.host_flags + 16);
        IngestBlock *tab_s = nullptr, *tab_d = nullptr;
        const auto sz = stream_table(tmp, ds, sizes_bytes, &tab_s, h, "array sizes stream", s);
        if (sz.second != 8 * n)
            fail(MQVS_ERR_ILLEGAL_COLUMN, "array sizes stream holds " + std::to_string(sz.second) + " bytes for " +
                                              std::to_string(n) + " rows");
        const auto dt = stream_table(tmp, dd, data_bytes, &tab_d, h, "vector data stream", s);
        if (dt.second % 4) fail(MQVS_ERR_ILLEGAL_COLUMN, "vector data stream is not a whole number of Float32");
        int *status = (int *)tmp.alloc(sizeof(int) * 4);
        MQVS_HIP(hipMemsetAsync(status, 0, sizeof(int) * 4, s));
        const bool verify = !(flags & MQVS_F_NO_CHECKSUM);
        if (verify) {  // CompressedReadBufferBase.cpp:192-196; the verdict is read before any decoded byte is used
            MQVS_HIP(hipStreamCreateWithFlags(&tmp.side, hipStreamNonBlocking));
            MQVS_HIP(hipEventCreateWithFlags(&tmp.fork, hipEventDisableTiming));
            MQVS_HIP(hipEventCreateWithFlags(&tmp.join, hipEventDisableTiming));
            MQVS_HIP(hipEventRecord(tmp.fork, s));
            MQVS_HIP(hipStreamWaitEvent(tmp.side, tmp.fork, 0));
            launch_block_checksum(ds, tab_s, sz.first, kBadSizesChecksum, status, nullptr, tmp.side);
            launch_block_checksum(dd, tab_d, dt.first, kBadDataChecksum, status, nullptr, tmp.side);
            MQVS_HIP(hipGetLastError());
            MQVS_HIP(hipEventRecord(tmp.join, tmp.side));
        }
        auto *sizes = (uint64_t *)tmp.alloc(sizeof(uint64_t) * (size_t)std::max<int64_t>(n, 1));
        launch_decode_blocks(ds, sizes_bytes, tab_s, sz.first, (uint8_t *)sizes, status, s);
        // the common case (every array has d elements) decodes straight into the rows
        const bool direct = dt.second == 4 * n * (int64_t)d;
        float *data = direct ? seg->rows : (float *)tmp.alloc((size_t)dt.second);
        launch_decode_blocks(dd, data_bytes, tab_d, dt.first, (uint8_t *)data, status, s);
        MQVS_HIP(hipGetLastError());
        const int64_t tiles = std::max<int64_t>(1, (n + 4095) / 4096);
        auto *offs = (int64_t *)tmp.alloc(sizeof(int64_t) * (size_t)std::max<int64_t>(n, 1));
        auto *scratch = (int64_t *)tmp.alloc(sizeof(int64_t) * (size_t)tiles);
        auto *st = (int64_t *)tmp.alloc(sizeof(int64_t) * 4);
        MQVS_HIP(hipMemsetAsync(st, 0, sizeof(int64_t) * 4, s));
        if (n > 0) launch_sizes_scan(sizes, n, d, offs, scratch, st, s);
        MQVS_HIP(hipGetLastError());
        MQVS_HIP(hipMemcpyAsync(h, st, 2 * sizeof(int64_t), hipMemcpyDeviceToHost, s));
        int *hstatus = reinterpret_cast<int *>(h + 2);
        if (verify) MQVS_HIP(hipStreamWaitEvent(s, tmp.join, 0));
        MQVS_HIP(hipMemcpyAsync(hstatus, status, sizeof(int), hipMemcpyDeviceToHost, s));
        host_wait(s);
        if (*hstatus & (kBadSizesChecksum | kBadDataChecksum))
            fail(MQVS_ERR_CHECKSUM, std::string("Checksum doesn't match: corrupted data (") +
                                        (*hstatus & kBadSizesChecksum ? "array sizes stream" : "vector data stream") +
                                        ", CityHash128 of a compressed block)");
        if (*hstatus)
            fail(MQVS_ERR_ILLEGAL_COLUMN, "malformed LZ4 block (CANNOT_DECOMPRESS)");
        const int64_t notd = h[0], nelem = h[1];
        if (nelem * 4 != dt.second)
            fail(MQVS_ERR_ILLEGAL_COLUMN, "array sizes sum to " + std::to_string(nelem) + " elements, the data stream "
                                              "holds " + std::to_string(dt.second / 4));
        const uint8_t *nonempty = nullptr;
        if (!(direct && notd == 0)) {
            // ragged or empty arrays: the reference's copy loop
            const float *srcdata = data;
            if (direct) {
                auto *copy = (float *)tmp.alloc((size_t)dt.second);
                MQVS_HIP(hipMemcpyAsync(copy, data, (size_t)dt.second, hipMemcpyDeviceToDevice, s));
                srcdata = copy;
            }
            auto *ne = (uint8_t *)tmp.alloc((size_t)std::max<int64_t>(n, 1));
            launch_array_rows(srcdata, offs, sizes, n, d, seg->rows, ne, s);
            MQVS_HIP(hipGetLastError());
            nonempty = ne;
        }
        prepare_segment(seg, nonempty, s);  // synchronises the stream
    } catch (...) {
        free_segment(seg);
        throw;
    }
    return seg;
}

// ---------------------------------------------------------------------------
// services for the index path (index.hip)

hipStream_t thread_stream(int device) { return workspace(device).stream; }

void search_internal(mqvs_segment *seg, const float *queries, int nq, int k, int metric,
                     const uint8_t *filter, const uint8_t *exists, int64_t *out_ids, float *out_dist,
                     uint32_t flags, hipStream_t stream) {
    search_impl(seg, queries, nq, k, metric, filter, exists, out_ids, out_dist, flags, stream);
}

mqvs_segment *segment_from_device(const float *dev_rows, int64_t n, int d, int metric, hipStream_t st) {
    mqvs_segment *s = new_segment(n, d, metric, std::max<int64_t>(n, 1), 0);
    try {
        if (n > 0)
            MQVS_HIP(hipMemcpyAsync(s->rows, dev_rows, sizeof(float) * (size_t)n * d, hipMemcpyDeviceToDevice, st));
        prepare_segment(s, nullptr, st);
    } catch (...) {
        free_segment(s);
        throw;
    }
    return s;
}

void segment_release(mqvs_segment *s) { free_segment(s); }

}  // namespace mqvs

using namespace mqvs;

// ---------------------------------------------------------------------------
extern "C" {

int mqvs_abi_version(void) { return MQVS_ABI_VERSION; }

const char *mqvs_last_error(void) { return g_error.c_str(); }

int mqvs_init(int device) {
    return guarded([&] {
        int n = 0;
        MQVS_HIP(hipGetDeviceCount(&n));
        if (device < 0 || device >= n) fail(MQVS_ERR_BAD_ARGUMENTS, "no such device");
        MQVS_HIP(hipSetDevice(device));
    });
}

int mqvs_device_count(int *count) {
    return guarded([&] {
        if (!count) fail(MQVS_ERR_BAD_ARGUMENTS, "null count");
        MQVS_HIP(hipGetDeviceCount(count));
    });
}

int mqvs_thread_release(void) {
    return guarded([&] {
        index_thread_release();
        if (!g_ws) return;
        for (auto &kv : *g_ws) {
            (void)hipSetDevice(kv.first);
            std::lock_guard<std::mutex> lk(kv.second.use);
            kv.second.release();
        }
        g_ws->clear();
    });
}

int mqvs_shutdown(void) { return mqvs_thread_release(); }

int mqvs_inject_fault(int32_t status, int32_t calls) {
    const bool mid = (status & MQVS_FAULT_MID_CALL) != 0;
    status &= ~MQVS_FAULT_MID_CALL;
    if (calls < 0 || (calls > 0 && status != MQVS_ERR_DEVICE && status != MQVS_ERR_MEMORY_LIMIT)) {
        set_error("mqvs_inject_fault: status must be MQVS_ERR_DEVICE or MQVS_ERR_MEMORY_LIMIT, calls >= 0");
        return MQVS_ERR_BAD_ARGUMENTS;
    }
    t_fault_status = status;
    t_fault_calls = calls;
    t_fault_mid = mid;
    return MQVS_OK;
}

int mqvs_segment_create(const float *host_rows, int64_t n, int32_t d, int32_t metric,
                        int64_t granule_rows, const uint8_t *nonempty, int64_t row_offset,
                        mqvs_segment_t *out) {
    return guarded([&] {
        if (!out) fail(MQVS_ERR_BAD_ARGUMENTS, "null output handle");
        *out = nullptr;
        check_seg_args(n, d, metric, granule_rows, row_offset);
        if (n > 0 && !host_rows) fail(MQVS_ERR_BAD_ARGUMENTS, "null rows");
        mqvs_segment *s = new_segment(n, d, metric, granule_rows, row_offset);
        try {
            Workspace &ws = workspace(s->device);
            WsCall ws_call(ws);
            if (n > 0)
                MQVS_HIP(hipMemcpyAsync(s->rows, host_rows, sizeof(float) * (size_t)n * d,
                                        hipMemcpyHostToDevice, ws.stream));
            const uint8_t *dne = nullptr;
            if (nonempty && n > 0 && !all_nonempty(nonempty, n)) {
                auto *b = (uint8_t *)ws.get(ws.misc, (size_t)n);
                MQVS_HIP(hipMemcpyAsync(b, nonempty, (size_t)n, hipMemcpyHostToDevice, ws.stream));
                dne = b;
            }
            prepare_segment(s, dne, ws.stream);
        } catch (...) {
            free_segment(s);
            throw;
        }
        *out = s;
    });
}

int mqvs_segment_create_device(const float *dev_rows, int64_t n, int32_t d, int32_t metric,
                               int64_t granule_rows, const uint8_t *dev_nonempty,
                               int64_t row_offset, mqvs_segment_t *out) {
    return guarded([&] {
        if (!out) fail(MQVS_ERR_BAD_ARGUMENTS, "null output handle");
        *out = nullptr;
        check_seg_args(n, d, metric, granule_rows, row_offset);
        if (n > 0 && !dev_rows) fail(MQVS_ERR_BAD_ARGUMENTS, "null rows");
        mqvs_segment *s = new_segment(n, d, metric, granule_rows, row_offset);
        try {
            Workspace &ws = workspace(s->device);
            WsCall ws_call(ws);
            if (n > 0)
                MQVS_HIP(hipMemcpyAsync(s->rows, dev_rows, sizeof(float) * (size_t)n * d,
                                        hipMemcpyDeviceToDevice, ws.stream));
            prepare_segment(s, dev_nonempty, ws.stream);
        } catch (...) {
            free_segment(s);
            throw;
        }
        *out = s;
    });
}

int mqvs_segment_generate(uint64_t seed, int32_t mode, int64_t n, int32_t d, int32_t metric,
                          int64_t granule_rows, int64_t row_offset, mqvs_segment_t *out) {
    return guarded([&] {
        if (!out) fail(MQVS_ERR_BAD_ARGUMENTS, "null output handle");
        *out = nullptr;
        check_seg_args(n, d, metric, granule_rows, row_offset);
        if (mode < 0 || mode > 3) fail(MQVS_ERR_BAD_ARGUMENTS, "generator mode must be 0, 1, 2 or 3");
        mqvs_segment *s = new_segment(n, d, metric, granule_rows, row_offset);
        try {
            Workspace &ws = workspace(s->device);
            WsCall ws_call(ws);
            launch_generate(seed, mode, row_offset, n, d, s->rows, ws.stream);
            MQVS_HIP(hipGetLastError());
            prepare_segment(s, nullptr, ws.stream);
        } catch (...) {
            free_segment(s);
            throw;
        }
        *out = s;
    });
}

int mqvs_segment_free(mqvs_segment_t seg) {
    return guarded([&] { free_segment(seg); });
}

int mqvs_segment_info(mqvs_segment_t seg, int64_t *n, int32_t *d, int32_t *metric,
                      int64_t *granule_rows, int64_t *row_offset, size_t *hbm_bytes) {
    return guarded([&] {
        if (!seg) fail(MQVS_ERR_BAD_ARGUMENTS, "null segment");
        if (n) *n = seg->n;
        if (d) *d = seg->d;
        if (metric) *metric = seg->metric;
        if (granule_rows) *granule_rows = seg->granule;
        if (row_offset) *row_offset = seg->row_offset;
        if (hbm_bytes) *hbm_bytes = seg->bytes;
    });
}

int mqvs_segment_prefilter(mqvs_segment_t seg, int32_t *split, size_t *plane_bytes, int32_t *approx_ok) {
    return guarded([&] {
        if (!seg) fail(MQVS_ERR_BAD_ARGUMENTS, "null segment");
        const bool planes = !seg->binary && seg->rows_hi != nullptr;
        if (split) *split = planes ? seg->split : 0;
        if (plane_bytes) *plane_bytes = planes ? seg->plane_bytes : 0;
        if (approx_ok) *approx_ok = !seg->binary && seg->approx_ok ? 1 : 0;
    });
}

int mqvs_segment_set_rows_host(mqvs_segment_t seg, int32_t host) {
    return guarded([&] {
        if (!seg) fail(MQVS_ERR_BAD_ARGUMENTS, "null segment");
        if (seg->binary) fail(MQVS_ERR_LOGICAL, "binary segment has no Float32 rows");
        if ((host != 0) == (seg->rows_host != nullptr)) return;
        DeviceGuard guard(seg->device);
        const size_t bytes = sizeof(float) * (size_t)std::max<int64_t>(seg->n, 1) * (size_t)seg->d;
        MQVS_HIP(hipDeviceSynchronize());  // (work queued on the rows, e.g. by the segment's creation)
        if (host) {
            void *h = nullptr;
            if (hipHostMalloc(&h, bytes, hipHostMallocMapped) != hipSuccess)
                fail(MQVS_ERR_MEMORY_LIMIT, "pinned host memory for the rows (" + std::to_string(bytes) + " bytes)");
            void *dptr = nullptr;
            const hipError_t e1 = hipMemcpy(h, seg->rows, bytes, hipMemcpyDeviceToHost);
            const hipError_t e2 = e1 == hipSuccess ? hipHostGetDevicePointer(&dptr, h, 0) : e1;
            if (e2 != hipSuccess) {
                (void)hipHostFree(h);
                MQVS_HIP(e2);
            }
            (void)hipFree(seg->rows);
            seg->rows = static_cast<float *>(dptr);
            seg->rows_host = h;
            seg->bytes -= std::min(seg->bytes, bytes);
        } else {
            float *d = nullptr;
            if (hipMalloc((void **)&d, bytes) != hipSuccess)
                fail(MQVS_ERR_MEMORY_LIMIT, "HBM for the rows (" + std::to_string(bytes) + " bytes)");
            const hipError_t e = hipMemcpy(d, seg->rows_host, bytes, hipMemcpyHostToDevice);
            if (e != hipSuccess) {
                (void)hipFree(d);
                MQVS_HIP(e);
            }
            (void)hipHostFree(seg->rows_host);
            seg->rows_host = nullptr;
            seg->rows = d;
            seg->bytes += bytes;
        }
    });
}

int mqvs_segment_rows_host(mqvs_segment_t seg, int32_t *host) {
    return guarded([&] {
        if (!seg || !host) fail(MQVS_ERR_BAD_ARGUMENTS, "null argument");
        *host = seg->rows_host != nullptr ? 1 : 0;
    });
}

int mqvs_segment_rows(mqvs_segment_t seg, const float **dev_rows) {
    return guarded([&] {
        if (!seg || !dev_rows) fail(MQVS_ERR_BAD_ARGUMENTS, "null argument");
        if (seg->binary) fail(MQVS_ERR_LOGICAL, "binary segment has no Float32 rows");
        *dev_rows = seg->rows;
    });
}

int mqvs_search(mqvs_segment_t seg, const float *queries, int32_t nq, int32_t k, int32_t metric,
                const uint8_t *filter, const uint8_t *row_exists, int64_t *out_ids, float *out_dist,
                uint32_t flags, mqvs_stream_t stream) {
    return guarded([&] {
        fault_point();
        WaitScope wsc{1, (uint64_t)(uintptr_t)seg, (uint64_t)nq, (uint64_t)k, (uint64_t)metric, filter != nullptr,
                      row_exists != nullptr, flags};
        search_impl(seg, queries, nq, k, metric, filter, row_exists, out_ids, out_dist, flags,
                    (hipStream_t)stream);
    });
}

int mqvs_search_ex(mqvs_segment_t seg, const float *queries, int32_t nq, int32_t k, int32_t metric,
                   const uint8_t *filter, const uint8_t *row_exists, int64_t chunk_ord_base,
                   int64_t *out_ids, float *out_dist, uint32_t flags, mqvs_stream_t stream) {
    return guarded([&] {
        fault_point();
        if (chunk_ord_base > INT32_MAX) fail(MQVS_ERR_BAD_ARGUMENTS, "chunk_ord_base out of range");
        WaitScope wsc{1, (uint64_t)(uintptr_t)seg, (uint64_t)nq, (uint64_t)k, (uint64_t)metric, filter != nullptr,
                      row_exists != nullptr, flags};
        search_impl(seg, queries, nq, k, metric, filter, row_exists, out_ids, out_dist, flags,
                    (hipStream_t)stream, false, chunk_ord_base);
    });
}

int mqvs_knn_raw(const float *x, const float *y, int64_t d, int64_t k, int64_t nx, int64_t ny,
                 int32_t metric, int64_t *result_id, float *distance) {
    return guarded([&] {
        if (metric != MQVS_METRIC_L2 && metric != MQVS_METRIC_IP)
            fail(MQVS_ERR_NOT_IMPLEMENTED, "Metric not implemented in brute force search for Float32 Vector");
        fault_point();
        if (d <= 0 || d > INT32_MAX || k < 0 || k > INT32_MAX || nx < 0 || nx > INT32_MAX || ny < 0)
            fail(MQVS_ERR_BAD_ARGUMENTS, "bad sizes");
        if (nx == 0 || k == 0) return;
        if (ny == 0) {
            for (int64_t i = 0; i < nx * k; ++i) {
                result_id[i] = -1;
                distance[i] = metric == MQVS_METRIC_L2 ? 3.40282347e+38f : -3.40282347e+38f;
            }
            return;
        }
        mqvs_segment *s = new_segment(ny, (int)d, metric, ny, 0);
        try {
            Workspace &ws = workspace(s->device);
            WsCall ws_call(ws);
            MQVS_HIP(hipMemcpyAsync(s->rows, y, sizeof(float) * (size_t)ny * d, hipMemcpyHostToDevice,
                                    ws.stream));
            prepare_segment(s, nullptr, ws.stream);
            search_impl(s, x, (int)nx, (int)k, metric == MQVS_METRIC_IP ? kMetricIpRaw : MQVS_METRIC_L2,
                        nullptr, nullptr, result_id, distance, 0, nullptr);
        } catch (...) {
            free_segment(s);
            throw;
        }
        free_segment(s);
    });
}

int mqvs_segment_create_from_column(const uint8_t *data_bin, int64_t data_bytes, const uint8_t *sizes_bin,
                                    int64_t sizes_bytes, int64_t n, int32_t d, int32_t metric, int64_t granule_rows,
                                    int64_t row_offset, uint32_t flags, mqvs_segment_t *out) {
    return guarded([&] {
        if (!out) fail(MQVS_ERR_BAD_ARGUMENTS, "null output handle");
        *out = nullptr;
        *out = ingest_column(data_bin, data_bytes, sizes_bin, sizes_bytes, n, d, metric, granule_rows, row_offset,
                             flags);
    });
}

int mqvs_segment_create_binary(const uint8_t *codes, int64_t n, int32_t dim_bits, int32_t metric,
                               int64_t granule_rows, int64_t row_offset, uint32_t flags, mqvs_segment_t *out) {
    return guarded([&] {
        if (!out) fail(MQVS_ERR_BAD_ARGUMENTS, "null output handle");
        *out = nullptr;
        mqvs_segment *s = new_binary_segment(n, dim_bits, metric, granule_rows, row_offset);
        try {
            if (n > 0 && !codes) fail(MQVS_ERR_BAD_ARGUMENTS, "null codes");
            Workspace &ws = workspace(s->device);
            WsCall ws_call(ws);
            upload_codes(s->codes, s->code_words, codes, s->code_bytes, n, (flags & MQVS_F_DEVICE_PTRS) != 0,
                         ws.stream);
            MQVS_HIP(hipStreamSynchronize(ws.stream));
        } catch (...) {
            free_segment(s);
            throw;
        }
        *out = s;
    });
}

int mqvs_search_binary(mqvs_segment_t seg, const uint8_t *queries, int32_t nq, int32_t k, int32_t metric,
                       const uint8_t *filter, const uint8_t *row_exists, int64_t *out_ids, float *out_dist,
                       uint32_t flags, mqvs_stream_t stream) {
    return guarded([&] {
        fault_point();
        WaitScope wsc{2, (uint64_t)(uintptr_t)seg, (uint64_t)nq, (uint64_t)k, (uint64_t)metric, filter != nullptr,
                      row_exists != nullptr, flags};
        search_binary_impl(seg, queries, nq, k, metric, filter, row_exists, out_ids, out_dist, flags,
                           (hipStream_t)stream);
    });
}

int mqvs_knn_binary_raw(const uint8_t *x, const uint8_t *y, int64_t d, int64_t k, int64_t nx, int64_t ny,
                        int32_t metric, int64_t *result_id, float *distance) {
    return guarded([&] {
        if (metric != MQVS_METRIC_HAMMING && metric != MQVS_METRIC_JACCARD)
            fail(MQVS_ERR_NOT_IMPLEMENTED, "Metric not implemented in brute force search for Binary Vector");
        fault_point();
        if (d <= 0 || d % 8 != 0 || d > INT32_MAX || k < 0 || k > INT32_MAX || nx < 0 || nx > INT32_MAX ||
            ny < 0)
            fail(MQVS_ERR_BAD_ARGUMENTS, "bad sizes");
        if (nx == 0 || k == 0) return;
        if (ny == 0) {
            for (int64_t i = 0; i < nx * k; ++i) {
                result_id[i] = -1;
                if (metric == MQVS_METRIC_HAMMING)
                    reinterpret_cast<int32_t *>(distance)[i] = INT32_MAX;
                else
                    distance[i] = 3.40282347e+38f;
            }
            return;
        }
        mqvs_segment *s = new_binary_segment(ny, (int32_t)d, metric, ny, 0);
        try {
            Workspace &ws = workspace(s->device);
            WsCall ws_call(ws);
            upload_codes(s->codes, s->code_words, y, s->code_bytes, ny, false, ws.stream);
            const size_t m = (size_t)nx * k;
            auto *b = (char *)ws.get(ws.misc, m * 12 + 16);
            auto *di = (int64_t *)b;
            auto *dd = (float *)(b + m * 8);
            auto *qd = (uint8_t *)ws.get(ws.glist, (size_t)nx * (d / 8));
            MQVS_HIP(hipMemcpyAsync(qd, x, (size_t)nx * (d / 8), hipMemcpyHostToDevice, ws.stream));
            search_binary_impl(s, qd, (int)nx, (int)k, metric, nullptr, nullptr, di, dd, MQVS_F_DEVICE_PTRS,
                               nullptr);
            if (metric == MQVS_METRIC_HAMMING) launch_hamming_to_int(di, dd, (int64_t)m, ws.stream);
            MQVS_HIP(hipGetLastError());
            MQVS_HIP(hipMemcpyAsync(result_id, di, m * 8, hipMemcpyDeviceToHost, ws.stream));
            MQVS_HIP(hipMemcpyAsync(distance, dd, m * 4, hipMemcpyDeviceToHost, ws.stream));
            MQVS_HIP(hipStreamSynchronize(ws.stream));
        } catch (...) {
            free_segment(s);
            throw;
        }
        free_segment(s);
    });
}

int mqvs_merge_shards(int32_t nshards, int32_t nq, int32_t k, int32_t metric, const int64_t *in_ids,
                      const float *in_dist, int64_t *out_ids, float *out_dist, uint32_t flags,
                      mqvs_stream_t stream) {
    return guarded([&] {
        if (nshards <= 0 || nq < 0 || k < 0) fail(MQVS_ERR_BAD_ARGUMENTS, "bad sizes");
        if ((int64_t)nshards * k > ((int64_t)1 << 20)) fail(MQVS_ERR_BAD_ARGUMENTS, "nshards * k above 2^20");
        if (nq == 0 || k == 0) return;
        int dev = 0;
        MQVS_HIP(hipGetDevice(&dev));
        Workspace &ws = workspace(dev);
        WsCall ws_call(ws);
        hipStream_t s = stream ? (hipStream_t)stream : ws.stream;
        ws.last = s;
        const size_t nin = (size_t)nshards * nq * k, nout = (size_t)nq * k;
        const int64_t *di = in_ids;
        const float *dd = in_dist;
        int64_t *oi = out_ids;
        float *od = out_dist;
        const bool devp = flags & MQVS_F_DEVICE_PTRS;
        if (!devp) {
            auto *b = (char *)ws.get(ws.misc, nin * 12 + nout * 12 + 64);
            auto *bi = (int64_t *)b;
            auto *bd = (float *)(b + nin * 8);
            oi = (int64_t *)(b + nin * 12 + 16 - (nin * 12) % 16);
            od = (float *)((char *)oi + nout * 8);
            MQVS_HIP(hipMemcpyAsync(bi, in_ids, nin * 8, hipMemcpyHostToDevice, s));
            MQVS_HIP(hipMemcpyAsync(bd, in_dist, nin * 4, hipMemcpyHostToDevice, s));
            di = bi;
            dd = bd;
        }
        // binary distances (Hamming, Jaccard) are ascending finite values: the L2 order
        const int order = (metric == MQVS_METRIC_HAMMING || metric == MQVS_METRIC_JACCARD) ? MQVS_METRIC_L2 : metric;
        uint4 *scratch = (int64_t)nshards * k > kSortCap
                             ? (uint4 *)ws.get(ws.large, sizeof(uint4) * 2 * (size_t)nshards * k * nq)
                             : nullptr;
        launch_merge_shards(nshards, nq, k, order, di, dd, oi, od, (flags & MQVS_F_PART_MERGE) != 0, scratch, s);
        MQVS_HIP(hipGetLastError());
        if (!devp) {
            MQVS_HIP(hipMemcpyAsync(out_ids, oi, nout * 8, hipMemcpyDeviceToHost, s));
            MQVS_HIP(hipMemcpyAsync(out_dist, od, nout * 4, hipMemcpyDeviceToHost, s));
        }
        if (!(devp && (flags & MQVS_F_ASYNC))) host_wait(s);
    });
}

int mqvs_generate_device(uint64_t seed, int32_t mode, int64_t row0, int64_t n, int32_t d,
                         float *dev_out, mqvs_stream_t stream) {
    return guarded([&] {
        if (mode < 0 || mode > 3 || n < 0 || d <= 0) fail(MQVS_ERR_BAD_ARGUMENTS, "bad arguments");
        int dev = 0;
        MQVS_HIP(hipGetDevice(&dev));
        Workspace &ws = workspace(dev);
        WsCall ws_call(ws);
        hipStream_t s = stream ? (hipStream_t)stream : ws.stream;
        ws.last = s;
        launch_generate(seed, mode, row0, n, d, dev_out, s);
        MQVS_HIP(hipGetLastError());
        host_wait(s);
    });
}

int mqvs_rerank(mqvs_segment_t seg, const float *queries, int32_t nq, const int64_t *cand,
                int32_t ncand, int32_t k, int32_t metric, const uint8_t *row_exists, int64_t *out_ids,
                float *out_dist, uint32_t flags, mqvs_stream_t stream) {
    return guarded([&] {
        WaitScope wsc{3, (uint64_t)(uintptr_t)seg, (uint64_t)nq, (uint64_t)ncand, (uint64_t)k, (uint64_t)metric,
                      row_exists != nullptr, flags};
        rerank_impl(seg, queries, nq, cand, ncand, k, metric, row_exists, out_ids, out_dist, flags,
                    (hipStream_t)stream);
    });
}

int mqvs_last_search_stats(mqvs_search_stats *out) {
    if (!out) return MQVS_ERR_BAD_ARGUMENTS;
    *out = g_stats;
    return MQVS_OK;
}

int mqvs_set_batch_mode(int mode) {
    if (mode != 0 && mode != 1) return MQVS_ERR_BAD_ARGUMENTS;
    g_batch_mode.store(mode);
    return MQVS_OK;
}

int mqvs_set_prefilter(int split) {
    if (split != kHiSplit && split != 0) return MQVS_ERR_BAD_ARGUMENTS;
    g_prefilter.store(split);
    return MQVS_OK;
}

int mqvs_measure_read_bandwidth(size_t bytes, int32_t reps, double *gbs, double *best_ms) {
    return guarded([&] {
        if (!gbs || bytes < ((size_t)1 << 20) || reps < 1) fail(MQVS_ERR_BAD_ARGUMENTS, "bad read-sweep arguments");
        hipStream_t s = nullptr;
        MQVS_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        try {
            *gbs = measure_read_sweep(bytes, reps, s, best_ms);
        } catch (...) {
            (void)hipStreamDestroy(s);
            throw;
        }
        MQVS_HIP(hipStreamDestroy(s));
    });
}

size_t mqvs_set_workspace_budget(size_t bytes) {
    const size_t prev = ws_budget();
    if (bytes) {
        g_ws_budget.store(bytes, std::memory_order_relaxed);
        WsGate &g = gate();
        std::lock_guard<std::mutex> lk(g.mu);
        g.cv.notify_all();
    }
    return prev;
}

int mqvs_workspace_stats(mqvs_workspace_stats_t *out, int32_t reset_peak) {
    return guarded([&] {
        if (!out) fail(MQVS_ERR_BAD_ARGUMENTS, "null stats");
        const size_t b = ws_budget();
        WsGate &g = gate();
        std::lock_guard<std::mutex> lk(g.mu);
        out->budget = b;
        out->held = g.held;
        out->peak = g.peak;
        out->waits = g.waits;
        out->trims = g.trims;
        out->over_budget = g.over;
        out->active = g.active;
        out->workspaces = (int32_t)g.all.size();
        if (reset_peak) {
            g.peak = g.held;
            g.waits = g.trims = g.over = 0;
        }
    });
}

size_t mqvs_set_scratch_budget(size_t bytes) {
    if (bytes == 0) return g_scratch_budget.load();
    return g_scratch_budget.exchange(std::max<size_t>(bytes, (size_t)1 << 20));
}

int mqvs_set_gather_mode(int mode) {
    if (mode < 0 || mode > 2) return MQVS_ERR_BAD_ARGUMENTS;
    g_gather_mode.store(mode);
    return MQVS_OK;
}

int mqvs_set_timing(int enabled) {
    g_timing.store(enabled ? 1 : 0);
    return MQVS_OK;
}

int mqvs_set_wait_mode(int mode, int spin_us) {
    if (mode < MQVS_WAIT_RUNTIME || mode > MQVS_WAIT_BLOCK) {
        set_error("mqvs_set_wait_mode: mode must be MQVS_WAIT_RUNTIME, MQVS_WAIT_HYBRID or MQVS_WAIT_BLOCK");
        return -MQVS_ERR_BAD_ARGUMENTS;
    }
    if (spin_us >= 0) g_wait_spin_us.store(spin_us);
    return g_wait_mode.exchange(mode);
}

int mqvs_async_check(mqvs_stream_t stream) {
    return guarded([&] {
        int dev = 0;
        MQVS_HIP(hipGetDevice(&dev));
        Workspace &ws = workspace(dev);
        WsCall ws_call(ws);
        hipStream_t s = stream ? (hipStream_t)stream : ws.stream;
        ws.last = s;
        host_wait(s);
        if (!ws.sticky.p) return;
        int word = 0;
        MQVS_HIP(hipMemcpy(&word, ws.sticky.p, sizeof(int), hipMemcpyDeviceToHost));
        MQVS_HIP(hipMemset(ws.sticky.p, 0, 16));
        if (word & 1)
            fail(MQVS_ERR_LOGICAL, "an ASYNC search needed its candidate-overflow fallback (results invalid): "
                                   "repeat it without MQVS_F_ASYNC");
        if (word & 2)
            fail(MQVS_ERR_LOGICAL, "an ASYNC cosine search's query normalisation did not repeat within " +
                                       std::to_string(kMaxVariants) + " steps on a part of more chunks");
    });
}

}  // extern "C"
