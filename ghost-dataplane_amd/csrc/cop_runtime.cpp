// cop_runtime.cpp — GPU context behind the C ABI (include/cop_gpu.h).
//
// One context = one HIP device + 1..4 launch lanes (a HIP stream each, with
// its own ticket counters and look-back words, so launches on different
// lanes can run concurrently) + the device copies of the NF tables. It
// replaces the process-global NF state of the reference
// (lpm_tbl / rules / stats globals, firewall.h:107-110, shared and raced by
// the five coprocessor threads) with per-context state: one context per
// coprocessor thread or per GPU, no globals.
#include <hip/hip_runtime.h>

#include <dlfcn.h>
#include <errno.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#include "cop_gpu.h"
#include "cop_internal.h"
#include "cop_kernels.h"
#include <rccl/rccl.h>   // types only: librccl is dlopen-ed on first use

namespace {

constexpr uint32_t IVT_MAX = 8192;          // LDS interval entries per table (64 KiB)
// counter block: [shards 64 x 16][port shards 64 x 16][per-rule words]
constexpr size_t SHARD_WORDS = (size_t)COPK_COUNTER_SHARDS * COP_N_COUNTERS;
constexpr size_t PORT_WORDS = (size_t)COPK_COUNTER_SHARDS * COPK_PORT_WORDS;
constexpr size_t RULE_OFF = SHARD_WORDS + PORT_WORDS;
constexpr uint32_t LOOK_TILE_MIN = COPK_BLOCK;
constexpr int TIMING_SLOTS = 256;   // per lane
constexpr int MAX_LANES = 4;

struct DevLpm {
    bool loaded = false;
    uint32_t m = 0;                 // padded interval count (power of two) or 0
    // bucketed interval form: starts = sorted starts (m words) then the
    // bucket index (iw words: 2^ib + 1 u16 first-candidate positions);
    // lv = binary-search levels inside the widest bucket
    uint32_t ib = 0, lv = 0, iw = 0;
    uint32_t *starts = nullptr, *vals = nullptr;
    uint32_t *tbl24 = nullptr, *tbl8 = nullptr;
    uint32_t n_ext = 0;
    bool tbl8_packed = false;       // tbl8 as packed run blocks (COPK_TBL_DIR form note)
    size_t tbl8_bytes = 0;
    // multibit-trie form (lpm_trie.c): top level, nodes, leaves; null if not built
    uint32_t *tl0 = nullptr, *tnodes = nullptr, *tleaves = nullptr;
    uint32_t t_nodes = 0, t_leaves = 0;
    // bucketed global form (COP_CFG_LPM_BKT; m == 0, ib / lv its own):
    // bidx = 2^ib + 1 first-candidate positions, bpairs = (start, value)
    // pairs padded with COP_BKT_PADS (8) {0xFFFFFFFF, last value}; null if not built
    uint32_t *bidx = nullptr, *bpairs = nullptr;
    uint32_t b_m = 0;
};

struct Lane {
    hipStream_t s = nullptr;
    // two ticket buffers (COPK_MAX_LAUNCH_BATCHES lines of 16 u64): launch k
    // on this lane draws from buffer k%2 and zeroes the other one's dirty lines
    unsigned long long *tickets[2] = {nullptr, nullptr};
    uint32_t dirty[2] = {0, 0};
    int parity = 0;
    unsigned long long *look = nullptr;
    uint32_t look_cap = 0;
    // per-rule hit binning buffers of this lane's launches (grown on demand)
    uint32_t *hit_region = nullptr, *hit_off = nullptr;
    size_t hit_region_cap = 0, hit_off_cap = 0;   // bytes
    uint32_t epoch = 0;
    hipEvent_t ev[TIMING_SLOTS][2];
    int ev_head = 0, ev_count = 0, ev_created = 0;
    hipEvent_t join = nullptr;                      // timer joins
    // streaming host-path slot (zc: staging and records in mapped pinned
    // memory, m_* their device addresses; the kernel reads and writes them
    // over PCIe, no copy-engine transfers)
    uint8_t *h_stage = nullptr, *d_stage = nullptr, *m_stage = nullptr;
    cop_result *h_res = nullptr, *d_res = nullptr, *m_res = nullptr;
    uint32_t cap = 0;
    int zc = -1;   // the COP_STREAM_ZC mode the slot was allocated for
    hipEvent_t done = nullptr;
    bool busy = false;
    uint64_t first = 0;
    uint32_t n = 0;
};

// Host gather pool for the end-to-end path: the caller and n-1 persistent
// workers each pack one contiguous slice of the packets' 16-byte header
// records into pinned staging (scattered mbuf reads are DRAM-latency bound
// per thread) and, in the same job, copy one slice of a finished batch's
// records out of pinned memory (8 bytes per packet: one thread alone moves
// them at about 9 GB/s, 1.1 Gpkt/s, below the gather's rate). Workers spin
// on the job word for a while before they sleep, so a job reaches them
// within a few hundred ns while batches stream, and the caller spins for
// the job's end.
struct GatherPool {
    std::vector<std::thread> th;
    std::mutex m;
    std::condition_variable cv;
    std::atomic<uint64_t> gen{0};
    std::atomic<int> pending{0};
    std::atomic<bool> stop{false};
    std::atomic<int> sleepers{0};
    const void *const *src = nullptr;
    uint8_t *dst = nullptr;
    uint32_t n = 0;
    const uint8_t *cp_src = nullptr;   // copy-out job (may be empty)
    uint8_t *cp_dst = nullptr;
    size_t cp_bytes = 0;
    int parts = 1;

    // packed header records: 16 bytes (COP_HDR16_STRIDE: frame bytes 12..15,
    // 24..35) or 12 (COP_HDR12_STRIDE: 12..15, 26..33)
    static void slice(const void *const *src, uint8_t *dst, uint32_t n, int parts, int i, uint32_t rec = 16)
    {
        const uint32_t lo = (uint32_t)((uint64_t)n * i / parts), hi = (uint32_t)((uint64_t)n * (i + 1) / parts);
        // scattered mbuf reads are DRAM-latency bound: keep PF lines in flight
        constexpr uint32_t PF = 16;
        for (uint32_t q = lo; q < hi && q < lo + PF; q++) __builtin_prefetch((const uint8_t *)src[q] + 12);
        if (rec == COP_HDR12_STRIDE) {
            for (uint32_t q = lo; q < hi; q++) {
                if (q + PF < hi) __builtin_prefetch((const uint8_t *)src[q + PF] + 12);
                const uint8_t *p = (const uint8_t *)src[q];
                uint8_t *d = dst + (size_t)q * COP_HDR12_STRIDE;
                memcpy(d, p + 12, 4);
                memcpy(d + 4, p + 26, 8);
            }
            return;
        }
        for (uint32_t q = lo; q < hi; q++) {
            if (q + PF < hi) __builtin_prefetch((const uint8_t *)src[q + PF] + 12);
            const uint8_t *p = (const uint8_t *)src[q];
            uint8_t *d = dst + (size_t)q * COP_HDR16_STRIDE;
            memcpy(d, p + 12, 4);
            memcpy(d + 4, p + 24, 12);
        }
    }
    uint32_t rec = 16;   // the job's record size
    // the job's slices: jparts of them, participant i takes slice i - joff
    // (a synchronous job: the caller is participant 0 and takes slice 0; an
    // asynchronous one: the workers alone)
    int jparts = 1, joff = 0;
    // participant i's slice of the job: the copy-out slice (64-byte aligned
    // pieces), then the gather slice
    void part(int i)
    {
        i -= joff;
        if (cp_bytes) {
            const size_t units = (cp_bytes + 63) / 64;
            const size_t lo = std::min(cp_bytes, units * (size_t)i / jparts * 64),
                         hi = std::min(cp_bytes, units * (size_t)(i + 1) / jparts * 64);
            if (hi > lo) memcpy(cp_dst + lo, cp_src + lo, hi - lo);
        }
        if (n) slice(src, dst, n, jparts, i, rec);
    }
    void worker(int i)
    {
        uint64_t seen = 0;
        for (;;) {
            // spin about 50 us for the next job, then sleep until notified
            uint64_t g = gen.load(std::memory_order_acquire);
            for (int spin = 0; g == seen && !stop.load(std::memory_order_relaxed) && spin < 20000; spin++) {
                __builtin_ia32_pause();
                g = gen.load(std::memory_order_acquire);
            }
            if (g == seen && !stop.load()) {
                std::unique_lock<std::mutex> lk(m);
                sleepers.fetch_add(1);
                cv.wait(lk, [&] { return stop.load() || gen.load(std::memory_order_seq_cst) != seen; });
                sleepers.fetch_sub(1);
                g = gen.load(std::memory_order_acquire);
            }
            if (stop.load()) return;
            seen = g;
            part(i);
            pending.fetch_sub(1, std::memory_order_acq_rel);
        }
    }
    void start(int nthreads)
    {
        parts = nthreads;
        for (int i = 1; i < nthreads; i++) th.emplace_back(&GatherPool::worker, this, i);
    }
    // one job on every participant: gather n packets' records into d_, and
    // copy cp_n bytes from cp_s to cp_d (either may be empty)
    void run(const void *const *s_, uint8_t *d_, uint32_t n_, const void *cp_s = nullptr, void *cp_d = nullptr,
             size_t cp_n = 0, uint32_t rec_ = 16)
    {
        if (th.empty() || (n_ < 4096 && cp_n < (size_t)1 << 18)) {
            if (cp_n) memcpy(cp_d, cp_s, cp_n);
            if (n_) slice(s_, d_, n_, 1, 0, rec_);
            return;
        }
        rec = rec_;
        post(s_, d_, n_, cp_s, cp_d, cp_n, false);
        part(0);
        wait();
    }
    // the same job on the workers alone; the caller goes on (wait() joins it)
    void start_async(const void *const *s_, uint8_t *d_, uint32_t n_, const void *cp_s = nullptr,
                     void *cp_d = nullptr, size_t cp_n = 0, uint32_t rec_ = 16)
    {
        rec = rec_;
        post(s_, d_, n_, cp_s, cp_d, cp_n, true);
    }
    void wait()
    {
        while (pending.load(std::memory_order_acquire) != 0) __builtin_ia32_pause();
    }
    void post(const void *const *s_, uint8_t *d_, uint32_t n_, const void *cp_s, void *cp_d, size_t cp_n, bool async)
    {
        src = s_;
        dst = d_;
        n = n_;
        cp_src = (const uint8_t *)cp_s;
        cp_dst = (uint8_t *)cp_d;
        cp_bytes = cp_n;
        jparts = async ? (int)th.size() : parts;
        joff = async ? 1 : 0;
        pending.store((int)th.size(), std::memory_order_relaxed);
        gen.fetch_add(1, std::memory_order_seq_cst);
        if (sleepers.load(std::memory_order_seq_cst)) {
            std::lock_guard<std::mutex> lk(m);   // (a sleeper checks gen under the lock)
            cv.notify_all();
        }
    }
    void gather(const void *const *s_, uint8_t *d_, uint32_t n_) { run(s_, d_, n_); }
    ~GatherPool()
    {
        {
            std::lock_guard<std::mutex> lk(m);
            stop.store(true);
        }
        cv.notify_all();
        for (auto &t : th) t.join();
    }
};

}  // namespace

struct cop_ctx {
    int device = 0;
    hipStream_t stream = nullptr;   // lane 0's stream (helpers, uploads)
    Lane lane[MAX_LANES];
    int n_lanes = 1;
    int next_lane = 0;
    cop_config cfg{};
    int ncu = 256;
    int ppt_override = 0;      // $COP_PPT (1, 4, 8) for experiments; 0 = auto
    bool coalesced = true;     // one-shot kernel: coalesced header loads where eligible ($COP_LOADS=strided: off)
    bool stage_lists = true;   // one-shot kernel: forward lists staged in LDS ($COP_STAGE_LISTS=0: off)
    bool hit_bins = true;      // per-rule hit counters by binning ($COP_HIT_BINS=0: one atomic per hit)
    bool static_small = true;  // small launches in blockIdx tile order ($COP_STATIC_ORDER=0: tickets)
    bool rec_paired = false;   // one-shot kernel: records as 16-byte stores from lane pairs ($COP_REC_PAIRED=1)
    bool probe_nt = false;     // tbl24 probes as non-temporal loads ($COP_PROBE_NT=1, experiment)
    uint32_t bkt_xbits = COP_BKT_XBITS;   // bucketed route form: 2^x buckets per interval ($COP_BKT_XBITS)
    uint32_t dbg = 0;          // $COP_DBG: timing-only kernel ablations
    uint32_t lds_pad = 0;      // $COP_LDS_PAD: extra LDS bytes per workgroup (occupancy experiments)
    unsigned long long *stamps = nullptr;   // dbg bit 8: per-workgroup phase stamps
    uint32_t inject_submit = 0, inject_wait = 0;   // cop_debug_inject: failures to fake (tests)
    char err[256] = {0};

    uint32_t *rt_top = nullptr;
    uint16_t *rt_leaf = nullptr;
    uint32_t rt_nleaf = 0;
    DevLpm fw, lpm;

    uint32_t look_cap = 0;
    unsigned long long *counters = nullptr;     // COPK_COUNTER_SHARDS x 16 u64 [+ per-rule u64]
    uint32_t n_rule_ctr = 0;                    // per-rule words after the shards
    unsigned long long *ctr_sum = nullptr;      // RCCL all-reduce destination
    size_t ctr_sum_words = 0;
    ncclComm_t comm = nullptr;
    // host-mapped error words, one per lane (word 4*l): a look-back timeout
    // fails only the waits on the lane whose launch timed out
    uint32_t *h_err = nullptr;
    uint32_t *d_err = nullptr;

    hipEvent_t t0 = nullptr, t1 = nullptr;
    bool timing = false;
    double ev_sum_ms = 0;
    uint64_t ev_n = 0;

    // host path staging
    uint8_t *h_stage = nullptr;
    uint8_t *d_stage = nullptr;
    cop_result *d_res = nullptr;
    uint32_t *d_fwd = nullptr;
    uint32_t *d_fwdn = nullptr;
    uint32_t stage_cap = 0;
    GatherPool *gather = nullptr;   // cop_set_host_threads
    // zero-copy form of cop_process_host for small batches: the kernel reads
    // the header records from, and writes its records to, mapped pinned host
    // memory (no copy-engine round trips); up to zc_max packets ($COP_ZC_MAX)
    uint32_t zc_max = 65536;
    // cop_process_host_stream: the staged records copied H2D by the copy
    // engine and the result records written by the kernel straight into
    // mapped pinned memory (2, the default: the copy engine, which
    // serialises a lane's H2D and D2H copies, moves 16 bytes per packet
    // instead of 24), staging and records both mapped and moved by the
    // kernel over PCIe (1), or both copied (0); $COP_STREAM_ZC
    int stream_zc = 2;
    // cop_process_host_stream's staged header record: COP_HDR12_STRIDE
    // (default: src and dst only, a quarter fewer bytes over PCIe) or
    // COP_HDR16_STRIDE; $COP_STREAM_REC
    uint32_t stream_rec = COP_HDR12_STRIDE;
    uint8_t *zc_stage = nullptr;      // mapped pinned: records in
    cop_result *zc_res = nullptr;     // mapped pinned: results out
    uint32_t *zc_fwd = nullptr;       // mapped pinned: forward list + count
    uint32_t zc_cap = 0;
    // asynchronous host batches (cop_host_batch_submit / _wait): slot s runs
    // on lane s % n_lanes with its own pinned and device staging
    struct HostSlot {
        uint8_t *h_stage = nullptr, *d_stage = nullptr;
        cop_result *h_res = nullptr, *d_res = nullptr;
        uint32_t cap = 0, n = 0;
        hipEvent_t done = nullptr;
        bool busy = false;
    } hs[COP_HOST_SLOTS];
    cop_pmd *pmd = nullptr;             // the poll-mode kernel serving this context, if any
    hipStream_t tele_stream = nullptr;  // cop_counters_snapshot
    uint64_t *tele_host = nullptr;
    unsigned long long *tele_dev = nullptr;   // exchange_words scratch
    size_t tele_words = 0;
    unsigned long long *ctr_snap = nullptr;   // cop_coll_reduce_counters(reset): exchanged words
    size_t ctr_snap_words = 0;
    // host-path op times ($COP_HOST_PROF=1, cop_debug_host_prof): gather,
    // launch, wait, copy-out ns; batches; packets
    bool hprof = false;
    uint64_t hp[6] = {0, 0, 0, 0, 0, 0};
};

static inline uint64_t hp_ns()
{
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

static int set_err(cop_ctx *c, int code, const char *fmt, ...)
{
    if (c) {
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(c->err, sizeof(c->err), fmt, ap);
        va_end(ap);
    }
    return code;
}

#define HIPCHK(c, expr)                                                                         \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess)                                                                   \
            return set_err((c), -EIO, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
                           __LINE__);                                                           \
    } while (0)

// Memsets and device copies outside the launch lanes complete before they
// return: the lanes are non-blocking streams, so a plain hipMemset (null
// stream, asynchronous to the host) could still be zeroing look-back words
// or counters while the next kernel on a lane uses them.
static hipError_t memset_sync(void *p, int v, size_t bytes, hipStream_t s)
{
    hipError_t e = hipMemsetAsync(p, v, bytes, s);
    return e == hipSuccess ? hipStreamSynchronize(s) : e;
}

static inline uint32_t next_pow2(uint32_t x)
{
    uint32_t m = 1;
    while (m < x) m <<= 1;
    return m;
}

extern "C" {

void cop_config_default(cop_config *cfg)
{
    memset(cfg, 0, sizeof(*cfg));
    cfg->device = 0;
    cfg->stages = COP_DEFAULT_STAGES;
    cfg->n_ports = COP_KNI_KTHREAD;
    cfg->max_batch = 262144;
    cfg->max_batches = COPK_MAXB;
    cfg->flags = 0;
    cfg->n_streams = 2;
    cfg->routing_table = nullptr;
}

int cop_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char *cop_last_error(cop_ctx *ctx) { return ctx ? ctx->err : "no context"; }

int cop_device_pci_bus_id(int device, char *buf, int len)
{
    if (!buf || len < 13) return -EINVAL;
    if (hipDeviceGetPCIBusId(buf, len, device) != hipSuccess) return -ENODEV;
    return 0;
}

static void free_lpm(DevLpm &t)
{
    if (t.starts) (void)hipFree(t.starts);
    if (t.vals) (void)hipFree(t.vals);
    if (t.tbl24) (void)hipFree(t.tbl24);
    if (t.tbl8) (void)hipFree(t.tbl8);
    if (t.tl0) (void)hipFree(t.tl0);
    if (t.tnodes) (void)hipFree(t.tnodes);
    if (t.tleaves) (void)hipFree(t.tleaves);
    if (t.bidx) (void)hipFree(t.bidx);
    if (t.bpairs) (void)hipFree(t.bpairs);
    t = DevLpm();
}

static void coll_destroy(cop_ctx *c);

void cop_destroy(cop_ctx *c)
{
    if (!c) return;
    if (c->pmd) (void)cop_pmd_stop(c->pmd);
    (void)hipSetDevice(c->device);
    for (int l = 0; l < MAX_LANES; l++)
        if (c->lane[l].s) (void)hipStreamSynchronize(c->lane[l].s);
    free_lpm(c->fw);
    free_lpm(c->lpm);
    if (c->rt_top) (void)hipFree(c->rt_top);
    if (c->rt_leaf) (void)hipFree(c->rt_leaf);
    if (c->stamps) (void)hipFree(c->stamps);
    if (c->counters) (void)hipFree(c->counters);
    if (c->ctr_sum) (void)hipFree(c->ctr_sum);
    if (c->ctr_snap) (void)hipFree(c->ctr_snap);
    coll_destroy(c);
    if (c->h_err) (void)hipHostFree(c->h_err);
    if (c->t0) (void)hipEventDestroy(c->t0);
    if (c->t1) (void)hipEventDestroy(c->t1);
    for (int l = 0; l < MAX_LANES; l++) {
        Lane &L = c->lane[l];
        for (int q = 0; q < 2; q++)
            if (L.tickets[q]) (void)hipFree(L.tickets[q]);
        if (L.look) (void)hipFree(L.look);
        if (L.hit_region) (void)hipFree(L.hit_region);
        if (L.hit_off) (void)hipFree(L.hit_off);
        for (int i = 0; i < L.ev_created; i++) {
            (void)hipEventDestroy(L.ev[i][0]);
            (void)hipEventDestroy(L.ev[i][1]);
        }
        if (L.join) (void)hipEventDestroy(L.join);
        if (L.done) (void)hipEventDestroy(L.done);
        if (L.h_stage) (void)hipHostFree(L.h_stage);
        if (L.h_res) (void)hipHostFree(L.h_res);
        if (L.d_stage) (void)hipFree(L.d_stage);
        if (L.d_res) (void)hipFree(L.d_res);
        if (L.s && L.s != c->stream) (void)hipStreamDestroy(L.s);
    }
    if (c->zc_stage) (void)hipHostFree(c->zc_stage);
    if (c->zc_res) (void)hipHostFree(c->zc_res);
    if (c->zc_fwd) (void)hipHostFree(c->zc_fwd);
    for (auto &h : c->hs) {
        if (h.h_stage) (void)hipHostFree(h.h_stage);   // mapped: d_* alias these
        if (h.h_res) (void)hipHostFree(h.h_res);
        if (h.done) (void)hipEventDestroy(h.done);
    }
    if (c->h_stage) (void)hipHostFree(c->h_stage);
    if (c->d_stage) (void)hipFree(c->d_stage);
    if (c->d_res) (void)hipFree(c->d_res);
    if (c->d_fwd) (void)hipFree(c->d_fwd);
    if (c->d_fwdn) (void)hipFree(c->d_fwdn);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->tele_stream) (void)hipStreamDestroy(c->tele_stream);
    if (c->tele_host) (void)hipHostFree(c->tele_host);
    if (c->tele_dev) (void)hipFree(c->tele_dev);
    delete c->gather;
    delete c;
}

static int upload_empty_ivt(cop_ctx *c, DevLpm &t)
{
    // empty table: m = 4 (the LDS copy works in uint4 units), every value 0
    // (miss), so whatever interval the search lands in reads nh 0, no hit;
    // a zero bucket index (ib 6) sends every address to interval 0
    free_lpm(t);
    t.ib = 6;
    t.lv = 0;
    t.iw = ((64u + 2u) / 2u + 3u) & ~3u;
    const std::vector<uint32_t> zeros(4 + t.iw, 0u);
    HIPCHK(c, hipMalloc(&t.starts, zeros.size() * 4));
    HIPCHK(c, hipMalloc(&t.vals, 16));
    HIPCHK(c, hipMemcpy(t.starts, zeros.data(), zeros.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(t.vals, zeros.data(), 16, hipMemcpyHostToDevice));
    t.m = 4;
    t.loaded = true;
    HIPCHK(c, hipDeviceSynchronize());   // the copies have landed before any lane reads them
    return 0;
}

static int sync_lanes(cop_ctx *c);

// Read and clear the device error words of the lanes in `mask`.
static int take_lane_errors(cop_ctx *c, uint32_t mask)
{
    bool bad = false;
    for (int l = 0; l < MAX_LANES; l++)
        if ((mask >> l) & 1u) {
            volatile uint32_t *w = c->h_err + 4 * l;
            if (*w) {
                *w = 0;
                bad = true;
            }
        }
    return bad ? set_err(c, -EIO, "device reported a look-back timeout") : 0;
}

int cop_set_routing_table(cop_ctx *c, const uint16_t *rt)
{
    if (!c || !rt) return -EINVAL;
    if (c->pmd) return set_err(c, -EBUSY, "a poll-mode kernel is serving this context (cop_pmd_stop first)");
    if (c->lane[0].s)
        if (int rc = sync_lanes(c)) return rc;
    HIPCHK(c, hipSetDevice(c->device));
    uint32_t top[256];
    std::vector<uint16_t> leaves;
    uint32_t nleaf = 0;
    for (uint32_t b = 0; b < 256; b++) {
        const uint16_t *blk = rt + b * 256;
        bool uni = true;
        for (int i = 1; i < 256 && uni; i++) uni = blk[i] == blk[0];
        if (uni) {
            top[b] = blk[0];
        } else {
            top[b] = 0x80000000u | nleaf;
            leaves.insert(leaves.end(), blk, blk + 256);
            nleaf++;
        }
    }
    if (c->rt_top) (void)hipFree(c->rt_top);
    if (c->rt_leaf) (void)hipFree(c->rt_leaf);
    c->rt_top = nullptr;
    c->rt_leaf = nullptr;
    HIPCHK(c, hipMalloc(&c->rt_top, sizeof(top)));
    HIPCHK(c, hipMemcpy(c->rt_top, top, sizeof(top), hipMemcpyHostToDevice));
    HIPCHK(c, hipMalloc(&c->rt_leaf, nleaf ? nleaf * 512 : 16));
    if (nleaf) HIPCHK(c, hipMemcpy(c->rt_leaf, leaves.data(), nleaf * 512, hipMemcpyHostToDevice));
    c->rt_nleaf = nleaf;
    HIPCHK(c, hipDeviceSynchronize());   // the copies have landed before any lane reads them
    return 0;
}

int cop_create(const cop_config *cfg_in, cop_ctx **out)
{
    if (!out) return -EINVAL;
    *out = nullptr;
    cop_config cfg;
    if (cfg_in) cfg = *cfg_in;
    else cop_config_default(&cfg);
    if (cfg.max_batches == 0 || cfg.max_batches > COPK_MAXB || cfg.max_batch == 0 ||
        cfg.max_batch > (1u << 30) || cfg.n_ports == 0 || cfg.n_ports > 0xFFFFu ||
        cfg.n_streams > MAX_LANES)
        return -EINVAL;
    if (cfg.n_streams == 0) cfg.n_streams = 1;
    if ((cfg.flags & (COP_CFG_DEMUX_PORTS | COP_CFG_PORT_STATS)) && cfg.n_ports > COP_MAX_DEMUX_PORTS)
        return -EINVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return -ENODEV;
    if (cfg.device < 0 || cfg.device >= ndev) return -ENODEV;

    cop_ctx *c = new (std::nothrow) cop_ctx();
    if (!c) return -ENOMEM;
    c->device = cfg.device;
    c->cfg = cfg;
    c->cfg.routing_table = nullptr;
    int rc = 0;
#define CREATE_CHK(expr)                                                                  \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "cop_create: %s: %s\n", #expr, hipGetErrorString(e_));        \
            cop_destroy(c);                                                               \
            return -EIO;                                                                  \
        }                                                                                 \
    } while (0)
    CREATE_CHK(hipSetDevice(c->device));
    hipDeviceProp_t prop;
    CREATE_CHK(hipGetDeviceProperties(&prop, c->device));
    c->ncu = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    if (const char *e = getenv("COP_PPT")) {
        int v = atoi(e);
        c->ppt_override = (v == 1 || v == 4 || v == 8) ? v : 0;
    }
    if (const char *e = getenv("COP_DBG")) c->dbg = (uint32_t)strtoul(e, nullptr, 0);
    if (const char *e = getenv("COP_LDS_PAD")) c->lds_pad = (uint32_t)strtoul(e, nullptr, 0) & ~15u;
    if (const char *e = getenv("COP_ZC_MAX")) c->zc_max = (uint32_t)strtoul(e, nullptr, 0);
    if (const char *e = getenv("COP_STREAM_ZC")) c->stream_zc = std::min(2, std::max(0, atoi(e)));
    if (const char *e = getenv("COP_STREAM_REC")) c->stream_rec = atoi(e) == 16 ? COP_HDR16_STRIDE : COP_HDR12_STRIDE;
    if (const char *e = getenv("COP_LOADS")) c->coalesced = strcmp(e, "strided") != 0;
    if (const char *e = getenv("COP_STAGE_LISTS")) c->stage_lists = atoi(e) != 0;
    if (const char *e = getenv("COP_HIT_BINS")) c->hit_bins = atoi(e) != 0;
    if (const char *e = getenv("COP_HOST_PROF")) c->hprof = atoi(e) != 0;
    if (const char *e = getenv("COP_STATIC_ORDER")) c->static_small = atoi(e) != 0;
    if (const char *e = getenv("COP_REC_PAIRED")) c->rec_paired = atoi(e) != 0;
    if (const char *e = getenv("COP_PROBE_NT")) c->probe_nt = atoi(e) != 0;
    if (const char *e = getenv("COP_BKT_XBITS")) c->bkt_xbits = (uint32_t)atoi(e) & 7u;
    // route-table form for tables too large for LDS (A/B runs): trie | dir
    if (const char *e = getenv("COP_LPM_FORM")) {
        if (!strcmp(e, "trie")) c->cfg.flags = (c->cfg.flags & ~COP_CFG_LPM_BKT) | COP_CFG_LPM_TRIE;
        else if (!strcmp(e, "bkt")) c->cfg.flags = (c->cfg.flags & ~COP_CFG_LPM_TRIE) | COP_CFG_LPM_BKT;
        else if (!strcmp(e, "dir")) c->cfg.flags &= ~(COP_CFG_LPM_TRIE | COP_CFG_LPM_BKT);
    }
    // firewall-table form for tables too large for LDS (A/B runs): bkt | dir
    if (const char *e = getenv("COP_FW_FORM")) {
        if (!strcmp(e, "bkt")) c->cfg.flags |= COP_CFG_FW_BKT;
        else if (!strcmp(e, "dir")) c->cfg.flags &= ~COP_CFG_FW_BKT;
    }
    if (const char *e = getenv("COP_STREAMS")) {
        int v = atoi(e);
        if (v >= 1 && v <= MAX_LANES) cfg.n_streams = (uint32_t)v;
    }
    c->n_lanes = (int)cfg.n_streams;
    c->cfg.n_streams = cfg.n_streams;
    if (c->dbg & 8u) CREATE_CHK(hipMalloc(&c->stamps, (size_t)COPK_STAMP_WG * 8 * 8));
    uint32_t tiles_per_batch = (cfg.max_batch + LOOK_TILE_MIN - 1) / LOOK_TILE_MIN;
    c->look_cap = tiles_per_batch * cfg.max_batches;
    for (int l = 0; l < c->n_lanes; l++) {
        Lane &L = c->lane[l];
        CREATE_CHK(hipStreamCreateWithFlags(&L.s, hipStreamNonBlocking));
        for (int q = 0; q < 2; q++) {
            CREATE_CHK(hipMalloc(&L.tickets[q], COPK_MAX_LAUNCH_BATCHES * 16 * sizeof(unsigned long long)));
            CREATE_CHK(memset_sync(L.tickets[q], 0, COPK_MAX_LAUNCH_BATCHES * 16 * sizeof(unsigned long long), L.s));
        }
        CREATE_CHK(hipMalloc(&L.look, (size_t)c->look_cap * 8));
        CREATE_CHK(memset_sync(L.look, 0, (size_t)c->look_cap * 8, L.s));
        L.look_cap = c->look_cap;
        CREATE_CHK(hipEventCreateWithFlags(&L.join, hipEventDisableTiming));
        CREATE_CHK(hipEventCreateWithFlags(&L.done, hipEventDisableTiming));
        for (int i = 0; i < TIMING_SLOTS; i++) {
            CREATE_CHK(hipEventCreate(&L.ev[i][0]));
            if (hipEventCreate(&L.ev[i][1]) != hipSuccess) {
                (void)hipEventDestroy(L.ev[i][0]);
                cop_destroy(c);
                return -EIO;
            }
            L.ev_created = i + 1;
        }
    }
    c->stream = c->lane[0].s;
    CREATE_CHK(hipMalloc(&c->counters, RULE_OFF * 8));
    CREATE_CHK(memset_sync(c->counters, 0, RULE_OFF * 8, c->stream));
    CREATE_CHK(hipHostMalloc(&c->h_err, 64, hipHostMallocMapped));
    memset(c->h_err, 0, 64);
    CREATE_CHK(hipHostGetDevicePointer((void **)&c->d_err, c->h_err, 0));
    CREATE_CHK(hipEventCreate(&c->t0));
    CREATE_CHK(hipEventCreate(&c->t1));
#undef CREATE_CHK
    uint16_t *rt = (uint16_t *)malloc(COP_ROUTING_TBL_SZ * sizeof(uint16_t));
    if (!rt) {
        cop_destroy(c);
        return -ENOMEM;
    }
    if (cfg_in && cfg_in->routing_table) memcpy(rt, cfg_in->routing_table, COP_ROUTING_TBL_SZ * 2);
    else cop_route_table_default(rt, cfg.n_ports);
    rc = cop_set_routing_table(c, rt);
    free(rt);
    if (!rc) rc = upload_empty_ivt(c, c->fw);
    if (!rc) rc = upload_empty_ivt(c, c->lpm);
    if (rc) {
        fprintf(stderr, "cop_create: %s\n", c->err);
        cop_destroy(c);
        return rc;
    }
    *out = c;
    return 0;
}

static int sync_lanes(cop_ctx *c)
{
    HIPCHK(c, hipSetDevice(c->device));
    for (int l = 0; l < c->n_lanes; l++) HIPCHK(c, hipStreamSynchronize(c->lane[l].s));
    return 0;
}

// form: COP_FORM_RULE for the firewall (entries carry the matching rule id
// and the drop bit), COP_FORM_NH for the route stage (entries carry nh)
// Packed tbl8 groups ($COP_TBL8=packed|plain; default: packed once the
// groups pass 16 MiB, i.e. large tables whose groups would crowd the
// Infinity Cache). The form is described at COPK_TBL_DIR in cop_kernels.h.
static bool tbl8_pack_wanted(uint32_t n_ext)
{
    if (const char *e = getenv("COP_TBL8")) {
        if (!strcmp(e, "packed")) return n_ext > 0;
        if (!strcmp(e, "plain")) return false;
    }
    return n_ext >= 16384;
}

// Rewrite a DIR-24-8 image's groups as packed run blocks: h8 becomes the
// block array (u32 words, 64-byte blocks), and every extended tbl24 entry's
// payload the offset of its block in 64-byte units.
static void pack_tbl8(std::vector<uint32_t> &h24, std::vector<uint32_t> &h8)
{
    const size_t n_grp = h8.size() / 256;
    std::vector<uint32_t> blk;
    std::vector<uint32_t> off(n_grp);
    blk.reserve(n_grp * 32);
    for (size_t g = 0; g < n_grp; g++) {
        const uint32_t *e = &h8[g * 256];
        uint32_t words[8] = {0}, runs = 0, pre[8];
        std::vector<uint32_t> vals;
        for (uint32_t w = 0; w < 8; w++) {
            pre[w] = runs;
            for (uint32_t b = 0; b < 32; b++) {
                const uint32_t i = w * 32 + b;
                if (i == 0 || e[i] != e[i - 1]) {
                    words[w] |= 1u << b;
                    vals.push_back(e[i]);
                    runs++;
                }
            }
        }
        off[g] = (uint32_t)(blk.size() / 16);
        for (uint32_t w = 0; w < 8; w++) {
            blk.push_back(words[w]);   // little-endian u64: low word = bitmap
            blk.push_back(pre[w]);
        }
        blk.insert(blk.end(), vals.begin(), vals.end());
        blk.resize((blk.size() + 15) & ~(size_t)15, 0u);
    }
    for (auto &x : h24)
        if ((x & 0x03000000u) == 0x03000000u) x = (x & 0xFF000000u) | off[x & 0x00FFFFFFu];
    if (blk.empty()) blk.resize(16, 0u);
    h8.swap(blk);
}

// the multibit-trie form of intervals (s, v, m) into t (COP_CFG_LPM_TRIE)
static int upload_trie(cop_ctx *c, DevLpm &t, const uint32_t *s, const uint32_t *v, uint32_t m)
{
    cop_lpm_trie tr;
    int rc = cop_lpm_trie_build(s, v, m, &tr);
    if (rc) return set_err(c, rc, "trie build failed: %d", rc);
    const size_t nb = (size_t)std::max(tr.n_nodes, 1u) * COP_TRIE_NODE_WORDS * 4, lb = (size_t)std::max(tr.n_leaves, 1u) * 4;
    hipError_t e = hipMalloc(&t.tl0, COP_TRIE_L0 * 4);
    if (e == hipSuccess) e = hipMalloc(&t.tnodes, nb);
    if (e == hipSuccess) e = hipMalloc(&t.tleaves, lb);
    if (e == hipSuccess) e = hipMemcpy(t.tl0, tr.l0, COP_TRIE_L0 * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(t.tnodes, tr.nodes, nb, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(t.tleaves, tr.leaves, lb, hipMemcpyHostToDevice);
    t.t_nodes = tr.n_nodes;
    t.t_leaves = tr.n_leaves;
    cop_lpm_trie_free(&tr);
    if (e != hipSuccess) return set_err(c, -ENOMEM, "trie upload: %s", hipGetErrorString(e));
    return 0;
}

// the bucketed global form of intervals (s, v, m) into t (COP_CFG_LPM_BKT;
// lpm_bkt.c)
static int upload_bkt(cop_ctx *c, DevLpm &t, const uint32_t *s, const uint32_t *v, uint32_t m)
{
    cop_lpm_bkt bk;
    int rc = cop_lpm_bkt_build(s, v, m, c->bkt_xbits, &bk);
    if (rc) return set_err(c, rc, "bucketed route form build failed: %d", rc);
    const size_t idx_bytes = ((size_t)(1u << bk.ib) + 1) * 4, pair_bytes = 2 * ((size_t)m + COP_BKT_PADS) * 4;
    hipError_t e = hipMalloc(&t.bidx, idx_bytes);
    if (e == hipSuccess) e = hipMalloc(&t.bpairs, pair_bytes);
    if (e == hipSuccess) e = hipMemcpy(t.bidx, bk.idx, idx_bytes, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(t.bpairs, bk.pairs, pair_bytes, hipMemcpyHostToDevice);
    t.ib = bk.ib;
    t.lv = bk.lv;
    t.b_m = m;
    cop_lpm_bkt_free(&bk);
    if (e != hipSuccess) return set_err(c, -ENOMEM, "bucketed route form upload: %s", hipGetErrorString(e));
    return 0;
}

static int upload_lpm(cop_ctx *c, DevLpm &t, const cop_lpm_table *tab, bool want_ivt, int form, bool want_trie = false,
                      bool want_bkt = false)
{
    if (int rc = sync_lanes(c)) return rc;
    free_lpm(t);
    // interval form for LDS
    uint32_t *s = nullptr, *v = nullptr;
    uint32_t m = cop_lpm_form_intervals(tab, form, &s, &v);
    if (!s) return set_err(c, -ENOMEM, "interval export failed");
    if (want_ivt && m <= IVT_MAX) {
        // Bucketed form for LDS: the sorted starts (padded with 0xFFFFFFFF,
        // which only ip 0xFFFFFFFF reaches: its value, the last real
        // interval's, is repeated in the pads) and, per bucket of the top ib
        // bits, the position of its first candidate (R(bucket start), R(x) =
        // the last k with sorted[k] <= x); a lookup reads the bucket's two
        // index entries, then binary-lifts over at most lv levels inside the
        // bucket: 2 + lv dependent LDS reads instead of log2(M) + 1.
        const uint32_t M = next_pow2(m < 4 ? 4 : m);
        std::vector<uint32_t> sorted(M), hv(M);
        for (uint32_t k = 0; k < M; k++) {
            sorted[k] = k < m ? s[k] : 0xFFFFFFFFu;
            hv[k] = k < m ? v[k] : v[m - 1];
        }
        uint32_t ib = 0;
        while ((1u << ib) < m && ib < 12) ib++;
        if (ib < 6) ib = 6;
        const uint32_t nb = 1u << ib, iw = ((nb + 2) / 2 + 3) & ~3u;
        std::vector<uint32_t> img(M + iw, 0);
        std::copy(sorted.begin(), sorted.end(), img.begin());
        std::vector<uint16_t> idx(nb + 1);
        uint32_t k = 0, widest = 0;
        for (uint32_t b = 0; b <= nb; b++) {
            // R(b << (32 - ib)); the end sentinel is R(0xFFFFFFFF) = M - 1
            const uint64_t x = b == nb ? 0xFFFFFFFFull : (uint64_t)b << (32 - ib);
            while (k + 1 < M && sorted[k + 1] <= x) k++;
            idx[b] = (uint16_t)k;
            if (b) widest = std::max<uint32_t>(widest, idx[b] - idx[b - 1]);
        }
        memcpy(img.data() + M, idx.data(), idx.size() * sizeof(uint16_t));   // the index words (LE u16 pairs)
        uint32_t lv = 0;
        while ((1u << lv) <= widest) lv++;
        HIPCHK(c, hipMalloc(&t.starts, (size_t)(M + iw) * 4));
        HIPCHK(c, hipMalloc(&t.vals, M * 4));
        HIPCHK(c, hipMemcpy(t.starts, img.data(), (size_t)(M + iw) * 4, hipMemcpyHostToDevice));
        HIPCHK(c, hipMemcpy(t.vals, hv.data(), M * 4, hipMemcpyHostToDevice));
        t.m = M;
        t.ib = ib;
        t.lv = lv;
        t.iw = iw;
    }
    int trc = 0;
    if (want_bkt && !t.m) trc = upload_bkt(c, t, s, v, m);     // too large for the LDS interval form
    else if (want_trie && !t.m) trc = upload_trie(c, t, s, v, m);
    free(s);
    free(v);
    if (trc) return trc;
    // DIR-24-8 image (always: FORCE_DIR24 and the large-table path)
    const uint32_t n_ext = cop_lpm_form_n_ext(tab, form);
    std::vector<uint32_t> h24((size_t)1 << 24);
    std::vector<uint32_t> h8((size_t)(n_ext ? n_ext : 1) * 256);
    cop_lpm_form_fill_dir24(tab, form, h24.data(), h8.data());
    const bool packed = tbl8_pack_wanted(n_ext);
    if (packed) pack_tbl8(h24, h8);
    HIPCHK(c, hipMalloc(&t.tbl24, h24.size() * 4));
    HIPCHK(c, hipMalloc(&t.tbl8, h8.size() * 4));
    HIPCHK(c, hipMemcpy(t.tbl24, h24.data(), h24.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(t.tbl8, h8.data(), h8.size() * 4, hipMemcpyHostToDevice));
    t.n_ext = n_ext;
    t.tbl8_packed = packed;
    t.tbl8_bytes = h8.size() * 4;
    t.loaded = true;
    HIPCHK(c, hipDeviceSynchronize());   // the copies have landed before any lane reads them
    return 0;
}

// counter buffer = shards (COPK_COUNTER_SHARDS x 16) followed by n_rules
// per-rule words; the shard words are carried over, the rule words zeroed
static int resize_counters(cop_ctx *c, uint32_t n_rules)
{
    unsigned long long *nb = nullptr;
    HIPCHK(c, hipMalloc(&nb, (RULE_OFF + n_rules) * 8));
    hipError_t e = hipMemcpyAsync(nb, c->counters, RULE_OFF * 8, hipMemcpyDeviceToDevice, c->stream);
    if (e == hipSuccess && n_rules) e = hipMemsetAsync(nb + RULE_OFF, 0, (size_t)n_rules * 8, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) {
        (void)hipFree(nb);
        return set_err(c, -EIO, "counter resize: %s", hipGetErrorString(e));
    }
    (void)hipFree(c->counters);
    c->counters = nb;
    c->n_rule_ctr = n_rules;
    return 0;
}

int cop_set_fw_table(cop_ctx *c, const cop_lpm_table *t)
{
    if (!c || !t) return -EINVAL;
    if (c->pmd) return set_err(c, -EBUSY, "a poll-mode kernel is serving this context (cop_pmd_stop first)");
    if (t->n_rules > COP_LPM_NH_MASK) return set_err(c, -EINVAL, "rule ids exceed 24 bits");
    int rc = upload_lpm(c, c->fw, t, !(c->cfg.flags & COP_CFG_FW_FORCE_DIR24), COP_FORM_RULE, false,
                        (c->cfg.flags & COP_CFG_FW_BKT) != 0);
    if (rc) {
        // a failed upload leaves the stage with the empty table (every lookup
        // misses), never with a partial image a launch could read
        (void)upload_empty_ivt(c, c->fw);
        return rc;
    }
    if (c->cfg.flags & COP_CFG_RULE_COUNTERS) rc = resize_counters(c, t->n_rules);
    return rc;
}

int cop_set_route_lpm(cop_ctx *c, const cop_lpm_table *t)
{
    if (!c || !t) return -EINVAL;
    if (c->pmd) return set_err(c, -EBUSY, "a poll-mode kernel is serving this context (cop_pmd_stop first)");
    const int rc = upload_lpm(c, c->lpm, t, !(c->cfg.flags & COP_CFG_LPM_FORCE_DIR24), COP_FORM_NH,
                              (c->cfg.flags & COP_CFG_LPM_TRIE) != 0, (c->cfg.flags & COP_CFG_LPM_BKT) != 0);
    if (rc) (void)upload_empty_ivt(c, c->lpm);   // as cop_set_fw_table
    return rc;
}

int cop_load_fw_rules_file(cop_ctx *c, const char *path, const cop_lpm_config *cfg,
                           cop_lpm_report *report)
{
    cop_prefix *rules = nullptr;
    uint32_t n = 0;
    int rc = cop_rules_load_json(path, &rules, &n);
    if (rc) return set_err(c, rc, "rules file %s: error %d", path ? path : "(null)", rc);
    cop_lpm_table *t = nullptr;
    rc = cop_lpm_build(rules, n, cfg, &t, report);
    cop_rules_free(rules);
    if (rc) return set_err(c, rc, "lpm build failed: %d", rc);
    rc = cop_set_fw_table(c, t);
    cop_lpm_free(t);
    return rc;
}

static int pick_mode(const cop_ctx *c, const DevLpm &t, bool enabled, bool force_dir)
{
    if (!enabled) return COPK_TBL_OFF;
    if (!force_dir && t.m) return COPK_TBL_IVT;
    if (!force_dir && t.tl0) return COPK_TBL_TRIE;
    if (!force_dir && t.bidx) return COPK_TBL_BKT;
    if (t.tbl24) return COPK_TBL_DIR;
    return COPK_TBL_IVT;  // empty table (m = 4)
}

// tests: the route stage's table form a launch would use (COPK_TBL_*)
int cop_debug_route_form(cop_ctx *c)
{
    if (!c) return -EINVAL;
    return pick_mode(c, c->lpm, true, (c->cfg.flags & COP_CFG_LPM_FORCE_DIR24) != 0);
}

static void harvest_one(cop_ctx *c, Lane &L)
{
    int idx = (L.ev_head - L.ev_count + TIMING_SLOTS) % TIMING_SLOTS;
    float ms = 0;
    if (hipEventSynchronize(L.ev[idx][1]) == hipSuccess &&
        hipEventElapsedTime(&ms, L.ev[idx][0], L.ev[idx][1]) == hipSuccess) {
        c->ev_sum_ms += ms;
        c->ev_n++;
    }
    L.ev_count--;
}

static int submit_on(cop_ctx *c, Lane &L, const cop_batch *batches, uint32_t nb, bool demux, uint32_t stages);
static int pick_mode(const cop_ctx *c, const DevLpm &t, bool enabled, bool force_dir);

int cop_submit(cop_ctx *c, const cop_batch *batches, uint32_t nb)
{
    if (!c || (!batches && nb)) return -EINVAL;
    if (nb == 0) return 0;
    Lane &L = c->lane[c->next_lane];
    c->next_lane = (c->next_lane + 1) % c->n_lanes;
    return submit_on(c, L, batches, nb, true, c->cfg.stages);
}

static int choose_ppt(const cop_ctx *c, uint64_t total, bool imix)
{
    // tile size: the largest of 256 * {8, 4, 1} packets that still gives at
    // least one tile per CU (fewer tiles = fewer ticket / look-back steps).
    // IMIX stops at 4: its per-lane offset + header loads hold fewer
    // registers per packet in flight, so more resident workgroups pay
    // (533 vs 554 us at 384 x 64k)
    int ppt = 1;
    if (total >= (uint64_t)COPK_BLOCK * 8 * c->ncu) ppt = imix ? 4 : 8;
    else if (total >= (uint64_t)COPK_BLOCK * 4 * c->ncu) ppt = 4;
    // the bucketed forms read 64 bytes of pairs per packet in one round: at
    // 8 packets per lane that needs 195 VGPRs (2 waves per SIMD), at 4, 98
    // (4 waves); the firewall's bucketed form (COP_CFG_FW_BKT) the same
    if ((c->lpm.bidx || c->fw.bidx) && ppt > 4) ppt = 4;
    if (c->ppt_override) ppt = c->ppt_override;
    return ppt;
}

// The launch's tile size (256 * ppt packets) and packet layout.
struct Plan {
    int ppt;
    int layout;   // COPK_LAY_*
};

static Plan plan_launch(const cop_ctx *c, uint64_t total, bool imix, uint32_t min_stride)
{
    const bool wide = !imix && min_stride >= COPK_COALESCED_MIN_STRIDE;
    const bool hdr16 = !imix && (min_stride == COP_HDR16_STRIDE || min_stride == COP_HDR12_STRIDE);
    return Plan{choose_ppt(c, total, imix),
                imix    ? COPK_LAY_IMIX
                : hdr16 ? COPK_LAY_HDR16
                : (wide && c->coalesced) ? COPK_LAY_COALESCED
                                         : COPK_LAY_SLOTS};
}

// The table / counter / option part of a launch's parameters: table modes
// (LDS interval form or HBM DIR-24-8, falling back to DIR-24-8 when LDS
// would overflow), table pointers, the LDS carve, counters and options.
// p.stages, p.compact and p.demux are set by the caller.
static int fill_launch(cop_ctx *c, CopKParams &p, int ppt, int *fw_mode_out, int *lpm_mode_out, uint32_t *lds_out,
                       bool stage_records = false)
{
    const uint32_t stages = p.stages;
    int fw_mode = pick_mode(c, c->fw, (stages & COP_STAGE_FW) != 0, (c->cfg.flags & COP_CFG_FW_FORCE_DIR24) != 0);
    int lpm_mode =
        pick_mode(c, c->lpm, (stages & COP_STAGE_LPM) != 0, (c->cfg.flags & COP_CFG_LPM_FORCE_DIR24) != 0);
    p.n_ports = c->cfg.n_ports;
    p.dbg = c->dbg;
    p.rt_top = c->rt_top;
    p.rt_leaf = c->rt_leaf;
    p.rt_nleaf = c->rt_nleaf;
    // LDS carve (u32 words): rt_top 256 | leaves nleaf*128 | fw 2m | lpm 2m | misc | list stage
    const uint32_t misc_words =
        (p.demux || (c->cfg.flags & COP_CFG_PORT_STATS)) ? COPK_LDS_MISC_EXT_WORDS : COPK_LDS_MISC_WORDS;
    const bool stage_list = p.compact && !p.demux && (c->stage_lists || p.seg);
    auto lds_need = [&](int fwm, int lpmm) {
        return (256u + c->rt_nleaf * 128u + (fwm == COPK_TBL_IVT ? 2u * c->fw.m + c->fw.iw : 0u) +
                (lpmm == COPK_TBL_IVT ? 2u * c->lpm.m + c->lpm.iw : lpmm == COPK_TBL_TRIE ? COPK_TRIE_L0 : 0u) +
                misc_words +
                (stage_list ? COPK_BLOCK * ppt : 0u) +
                (stage_records ? 2u * COPK_BLOCK * ppt : 0u)) *
                   4u +
               c->lds_pad;
    };
    // Too much for LDS (a dense custom routing table beside large interval
    // tables): look the interval tables up in their DIR-24-8 images in HBM
    // instead, the route stage's first. Results are identical.
    while (lds_need(fw_mode, lpm_mode) > 160u * 1024u) {
        if ((lpm_mode == COPK_TBL_IVT || lpm_mode == COPK_TBL_TRIE) && c->lpm.tbl24) lpm_mode = COPK_TBL_DIR;
        else if (fw_mode == COPK_TBL_IVT && c->fw.tbl24) fw_mode = COPK_TBL_DIR;
        else return set_err(c, -E2BIG, "tables exceed LDS (%u bytes)", lds_need(fw_mode, lpm_mode));
    }
    // The bucketed firewall's kernel parts are built for the route forms that
    // large tables take (DIR-24-8, bucketed) and for no route stage: a route
    // table small enough for LDS, or in the trie form, is looked up in its
    // DIR-24-8 image beside it (same results). Only the empty route table has
    // no image.
    if (fw_mode == COPK_TBL_BKT && (lpm_mode == COPK_TBL_IVT || lpm_mode == COPK_TBL_TRIE)) {
        if (!c->lpm.tbl24)
            return set_err(c, -EINVAL,
                           "bucketed firewall (COP_CFG_FW_BKT) with the route stage on needs a route table "
                           "(cop_set_route_lpm)");
        lpm_mode = COPK_TBL_DIR;
    }
    p.fw_m = fw_mode == COPK_TBL_IVT ? c->fw.m : 0;
    p.fw_ib = c->fw.ib;
    p.fw_lv = c->fw.lv;
    p.fw_iw = fw_mode == COPK_TBL_IVT ? c->fw.iw : 0;
    p.fw_starts = c->fw.starts;
    p.fw_vals = c->fw.vals;
    p.fw_tbl24 = c->fw.tbl24;
    p.fw_tbl8 = c->fw.tbl8;
    p.fw_tbl8_packed = c->fw.tbl8_packed ? 1u : 0u;
    p.lpm_m = lpm_mode == COPK_TBL_IVT ? c->lpm.m : 0;
    p.lpm_ib = c->lpm.ib;
    p.lpm_lv = c->lpm.lv;
    p.lpm_iw = lpm_mode == COPK_TBL_IVT ? c->lpm.iw : 0;
    p.lpm_starts = c->lpm.starts;
    p.lpm_vals = c->lpm.vals;
    p.lpm_tbl24 = c->lpm.tbl24;
    p.lpm_tbl8 = c->lpm.tbl8;
    p.lpm_tbl8_packed = c->lpm.tbl8_packed ? 1u : 0u;
    p.probe_nt = c->probe_nt ? 1u : 0u;
    p.lpm_tl0 = c->lpm.tl0;
    p.lpm_tnodes = c->lpm.tnodes;
    p.lpm_tleaves = c->lpm.tleaves;
    p.lpm_bidx = c->lpm.bidx;
    p.lpm_bpairs = c->lpm.bpairs;
    p.fw_bidx = c->fw.bidx;
    p.fw_bpairs = c->fw.bpairs;
    uint32_t off = 256 + c->rt_nleaf * 128;
    p.lds_fw_off = off;
    off += 2 * p.fw_m + p.fw_iw;
    p.lds_lpm_off = off;
    off += lpm_mode == COPK_TBL_TRIE ? COPK_TRIE_L0 : 2 * p.lpm_m + p.lpm_iw;
    p.lds_misc_off = off;
    off += misc_words;
    p.lds_stage_off = 0;
    if (stage_list) {
        p.lds_stage_off = off;   // the tile's forward list, written out in 16-byte stores
        off += COPK_BLOCK * ppt;
    }
    p.lds_rec_off = 0;
    if (stage_records) {
        p.lds_rec_off = off;     // the tile's records, written out in 16-byte stores
        off += 2 * COPK_BLOCK * ppt;
    }
    p.counters = c->counters;
    p.rule_hits = (fw_mode != COPK_TBL_OFF && c->n_rule_ctr) ? c->counters + RULE_OFF : nullptr;
    p.port_ctr = c->counters + SHARD_WORDS;
    p.port_stats = (c->cfg.flags & COP_CFG_PORT_STATS) ? c->cfg.n_ports : 0u;
    p.stamps = c->stamps;
    *fw_mode_out = fw_mode;
    *lpm_mode_out = lpm_mode;
    *lds_out = off * 4 + c->lds_pad;
    return 0;
}

// Launch the one-shot kernel on lane L: its look-back words and epoch, its
// ticket buffers, then the table part (fill_launch).
// p.b / p.rg, p.nb, p.ntiles, p.uniform_ntiles, p.compact, p.demux and
// p.stages are set by the caller.
static int launch_on(cop_ctx *c, Lane &L, CopKParams &p, bool imix, Plan pl, uint32_t nb_used)
{
    const int ppt = pl.ppt;
    HIPCHK(c, hipSetDevice(c->device));
    // one chain per port (demux)
    const uint32_t look_need = p.ntiles * (p.demux ? p.demux : 1u);
    if (look_need > L.look_cap) {
        // grow this lane's look-back words (stream order: free after its work)
        HIPCHK(c, hipStreamSynchronize(L.s));
        HIPCHK(c, hipFree(L.look));
        L.look = nullptr;
        L.look_cap = 0;
        HIPCHK(c, hipMalloc(&L.look, (size_t)look_need * 8));
        HIPCHK(c, memset_sync(L.look, 0, (size_t)look_need * 8, L.s));
        L.look_cap = look_need;
        L.epoch = 0;
    }
    int fw_mode = 0, lpm_mode = 0;
    uint32_t lds_bytes = 0;
    if (int rc = fill_launch(c, p, ppt, &fw_mode, &lpm_mode, &lds_bytes)) return rc;
    // records as 16-byte stores from lane pairs ($COP_REC_PAIRED=1): every
    // batch's records must start 16-byte aligned
    p.rec_paired = 0;
    if (c->rec_paired) {
        bool al = true;
        if (p.ring) al = ((uintptr_t)p.rg.results & 15) == 0 && (p.rg.results_slot & 1) == 0;
        else
            for (uint32_t i = 0; i < p.nb; i++) al = al && ((uintptr_t)p.b[i].results & 15) == 0;
        p.rec_paired = al ? 1u : 0u;
    }
    if (++L.epoch == 0) {
        HIPCHK(c, hipMemsetAsync(L.look, 0, (size_t)L.look_cap * 8, L.s));
        L.epoch = 1;
    }
    p.epoch = L.epoch;
    // tickets: draw from buffer `parity`, zero the other buffer's dirty lines
    const int q = L.parity;
    p.tickets = L.tickets[q];
    p.zero_tickets = L.tickets[q ^ 1];
    p.zero_lines = L.dirty[q ^ 1];
    p.look = L.look;
    p.err = c->d_err + 4 * (&L - c->lane);
    if ((c->dbg & 8u) && p.ntiles > COPK_STAMP_WG) p.dbg &= ~8u;
    const uint32_t grid = p.ntiles;   // one tile per workgroup
    // Small launches (at most 4 workgroups per CU) take tile j of a batch in
    // blockIdx order: a look-back then waits only on workgroups dispatched
    // before it, as with tickets, without the ticket atomics that one batch's
    // workgroups would all issue on one counter (~3 us for 256 of them).
    // Large launches keep tickets. ($COP_STATIC_ORDER=0: always tickets)
    p.static_order = (grid <= 4u * (uint32_t)c->ncu && c->static_small) ? 1u : 0u;
    // per-rule hit counters by binning: each tile sorts its hits' rule ids by
    // bucket into its region, cop_hit_count adds them up after the launch
    p.hit_region = nullptr;
    p.hit_off = nullptr;
    p.hit_nb = 0;
    if (p.rule_hits && c->hit_bins) {
        const uint32_t nb = (c->n_rule_ctr + (1u << COPK_HIT_SHIFT) - 1) >> COPK_HIT_SHIFT;
        const uint32_t reg = COPK_BLOCK * (uint32_t)ppt + 4u * nb;
        const uint32_t base = (lds_bytes / 4u + 3u) & ~3u;
        const uint32_t words = ((3u * nb + 5u + 3u) & ~3u) + COPK_BLOCK * (uint32_t)ppt + reg;
        if (nb >= 1 && nb <= COPK_HIT_MAX_BUCKETS && (base + words) * 4u <= 160u * 1024u) {
            const size_t need_reg = (size_t)grid * reg * 4, need_off = (size_t)grid * (nb + 1) * 4;
            if (need_reg > L.hit_region_cap || need_off > L.hit_off_cap) {
                HIPCHK(c, hipStreamSynchronize(L.s));   // the lane's earlier launches are done with them
                if (need_reg > L.hit_region_cap) {
                    HIPCHK(c, hipFree(L.hit_region));
                    L.hit_region = nullptr;
                    L.hit_region_cap = 0;
                    HIPCHK(c, hipMalloc(&L.hit_region, need_reg));
                    L.hit_region_cap = need_reg;
                }
                if (need_off > L.hit_off_cap) {
                    HIPCHK(c, hipFree(L.hit_off));
                    L.hit_off = nullptr;
                    L.hit_off_cap = 0;
                    HIPCHK(c, hipMalloc(&L.hit_off, need_off));
                    L.hit_off_cap = need_off;
                }
            }
            p.hit_region = L.hit_region;
            p.hit_off = L.hit_off;
            p.hit_nb = nb;
            p.hit_reg_words = reg;
            p.lds_hit_off = base;
            lds_bytes = (base + words) * 4u;
        }
    }

    if (c->timing) {
        if (L.ev_count == TIMING_SLOTS) harvest_one(c, L);
        HIPCHK(c, hipEventRecord(L.ev[L.ev_head][0], L.s));
    }
    hipError_t e = copk_launch(&p, fw_mode, lpm_mode, pl.layout, ppt, grid, lds_bytes, L.s);
    if (e != hipSuccess) return set_err(c, -EIO, "launch: %s", hipGetErrorString(e));
    if (p.hit_region && (e = copk_hit_count(&p, grid, COPK_BLOCK * (uint32_t)ppt, L.s)) != hipSuccess)
        return set_err(c, -EIO, "hit count launch: %s", hipGetErrorString(e));
    L.dirty[q ^ 1] = 0;
    L.dirty[q] = (p.compact && !p.seg && !(c->dbg & 2u) && !p.static_order) ? nb_used : 0;
    L.parity = q ^ 1;
    if (c->timing) {
        HIPCHK(c, hipEventRecord(L.ev[L.ev_head][1], L.s));
        L.ev_head = (L.ev_head + 1) % TIMING_SLOTS;
        L.ev_count++;
    }
    return 0;
}

// demux: the caller's forward lists follow the COP_CFG_DEMUX_PORTS layout
// (public submits); the library's own host paths use one list per batch.
// stages: the context's mask, or the drop-in path's NF chain.
static int submit_on(cop_ctx *c, Lane &L, const cop_batch *batches, uint32_t nb, bool demux, uint32_t stages)
{
    if (c->inject_submit) {
        c->inject_submit--;
        return set_err(c, -EIO, "injected submit failure");
    }
    if (nb > c->cfg.max_batches) return set_err(c, -EINVAL, "nb %u > max_batches", nb);
    CopKParams p;
    memset(&p, 0, sizeof(p));
    uint64_t total = 0;
    bool imix = batches[0].offsets != nullptr;
    bool compact = false;
    for (uint32_t i = 0; i < nb; i++) {
        const cop_batch &b = batches[i];
        if ((b.offsets != nullptr) != imix)
            return set_err(c, -EINVAL, "batches in one submit must all be slot or all IMIX");
        if (b.n > c->cfg.max_batch) return set_err(c, -EINVAL, "batch %u: n %u > max_batch", i, b.n);
        if (b.n && (!b.pkts || !b.results)) return set_err(c, -EINVAL, "batch %u: null pointer", i);
        // (12-byte records are read as dwords: 4-byte aligned starts suffice)
        const bool rec12 = !imix && b.stride == COP_HDR12_STRIDE;
        if (((uintptr_t)b.pkts & (rec12 ? 3 : 15)) || (b.data_off & 15) || (!imix && !rec12 && (b.stride & 15)) ||
            (!imix && !rec12 && b.stride < 36 && b.stride != COP_HDR16_STRIDE))
            return set_err(c, -EINVAL, "batch %u: packet starts must be 16-byte aligned", i);
        if (!imix && b.n && b.stride != batches[0].stride &&
            (b.stride <= COP_HDR16_STRIDE || batches[0].stride <= COP_HDR16_STRIDE))
            return set_err(c, -EINVAL, "batches in one submit must all be 16-byte records, 12-byte records or frames");
        if ((uintptr_t)b.results & 7) return set_err(c, -EINVAL, "batch %u: results misaligned", i);
        total += b.n;
        if (b.fwd_idx || b.fwd_count) compact = true;
    }
    if (c->cfg.flags & COP_CFG_NO_COMPACT) compact = false;
    // segmented lists: public submits only (the library's own host paths
    // read one dense list per batch)
    const bool seg = demux && compact && (c->cfg.flags & COP_CFG_SEG_LISTS);
    if (seg && (c->cfg.flags & COP_CFG_DEMUX_PORTS)) return set_err(c, -EINVAL, "SEG_LISTS with DEMUX_PORTS");
    for (uint32_t i = 0; seg && i < nb; i++)
        if ((uintptr_t)batches[i].fwd_idx & 15) return set_err(c, -EINVAL, "batch %u: fwd_idx not 16-byte aligned", i);
    uint32_t min_stride = 0xFFFFFFFFu;
    for (uint32_t i = 0; i < nb; i++)
        if (batches[i].n) min_stride = std::min(min_stride, batches[i].stride);
    const Plan pl = plan_launch(c, total, imix, min_stride);
    const uint32_t tile = COPK_BLOCK * pl.ppt;
    uint32_t ntiles = 0;
    for (uint32_t i = 0; i < nb; i++) {
        const cop_batch &b = batches[i];
        CopKBatch &d = p.b[i];
        d.pkts = (const uint8_t *)b.pkts;
        d.offsets = b.offsets;
        d.results = b.results;
        d.fwd_idx = compact ? b.fwd_idx : nullptr;
        d.fwd_count = compact ? b.fwd_count : nullptr;
        d.n = b.n;
        d.stride = b.stride;
        d.data_off = b.data_off;
        d.ntiles = b.n ? (b.n + tile - 1) / tile : 1;   // an empty batch still reports count 0
        p.tile_begin[i] = ntiles;
        p.look_begin[i] = ntiles;
        ntiles += d.ntiles;
    }
    p.ring = 0;
    p.nb = nb;
    p.ntiles = ntiles;
    p.uniform_ntiles = p.b[0].ntiles;
    for (uint32_t i = 1; i < nb; i++)
        if (p.b[i].ntiles != p.b[0].ntiles) p.uniform_ntiles = 0;
    p.compact = compact ? 1u : 0u;
    p.seg = seg ? 1u : 0u;
    p.stages = stages;
    p.demux = (demux && compact && (c->cfg.flags & COP_CFG_DEMUX_PORTS)) ? c->cfg.n_ports : 0u;
    return launch_on(c, L, p, imix, pl, nb);
}

// COP_CFG_SEG_LISTS rings: no demux, 16-byte aligned segments
static int check_seg_ring(cop_ctx *c, const cop_batch_ring *r, bool seg)
{
    if (!seg) return 0;
    if (c->cfg.flags & COP_CFG_DEMUX_PORTS) return set_err(c, -EINVAL, "SEG_LISTS with DEMUX_PORTS");
    if (r->fwd_idx && (((uintptr_t)r->fwd_idx & 15) || (r->fwd_slot & 3)))
        return set_err(c, -EINVAL, "ring: segmented lists need a 16-byte aligned fwd_idx and fwd_slot %% 4 == 0");
    return 0;
}

int cop_submit_ring(cop_ctx *c, const cop_batch_ring *r, uint32_t first_slot, uint32_t count)
{
    if (!c || !r) return -EINVAL;
    if (count == 0) return 0;
    if (count > COPK_MAX_LAUNCH_BATCHES || r->n_slots == 0 || first_slot >= r->n_slots)
        return set_err(c, -EINVAL, "ring: count %u / first %u / n_slots %u", count, first_slot, r->n_slots);
    if (r->n > c->cfg.max_batch) return set_err(c, -EINVAL, "ring: n %u > max_batch", r->n);
    const bool imix = r->offsets != nullptr;
    if (r->n && (!r->pkts || !r->results)) return set_err(c, -EINVAL, "ring: null pointer");
    if (((uintptr_t)r->pkts & 15) || (r->pkts_slot_bytes & 15) || (r->data_off & 15) ||
        (!imix && ((r->stride & 15) || (r->stride < 36 && r->stride != COP_HDR16_STRIDE))))
        return set_err(c, -EINVAL, "ring: packet starts must be 16-byte aligned");
    bool compact = (r->fwd_idx || r->fwd_count) && !(c->cfg.flags & COP_CFG_NO_COMPACT);
    const uint32_t lists = (compact && (c->cfg.flags & COP_CFG_DEMUX_PORTS)) ? c->cfg.n_ports : 1u;
    if (r->results_slot < r->n || (r->fwd_idx && r->fwd_slot < (uint64_t)r->n * lists))
        return set_err(c, -EINVAL, "ring: slot sizes smaller than n (x ports with demux)");
    const bool seg = compact && (c->cfg.flags & COP_CFG_SEG_LISTS);
    if (int rc = check_seg_ring(c, r, seg)) return rc;
    const Plan pl = plan_launch(c, (uint64_t)r->n * count, imix, r->stride);
    const uint32_t tile = COPK_BLOCK * pl.ppt;
    const uint32_t tpb = r->n ? (r->n + tile - 1) / tile : 1;
    CopKParams p;
    memset(&p, 0, sizeof(p));
    p.ring = 1;
    p.rg.pkts = (const uint8_t *)r->pkts;
    p.rg.offsets = r->offsets;
    p.rg.results = r->results;
    p.rg.fwd_idx = compact ? r->fwd_idx : nullptr;
    p.rg.fwd_count = compact ? r->fwd_count : nullptr;
    p.rg.pkts_slot_bytes = r->pkts_slot_bytes;
    p.rg.offsets_slot_words = r->offsets_slot_words;
    p.rg.results_slot = r->results_slot;
    p.rg.fwd_slot = r->fwd_slot;
    p.rg.n_slots = r->n_slots;
    p.rg.first = first_slot;
    p.rg.n = r->n;
    p.rg.stride = r->stride;
    p.rg.data_off = r->data_off;
    p.nb = count;
    p.ntiles = tpb * count;
    p.uniform_ntiles = tpb;
    p.compact = compact ? 1u : 0u;
    p.seg = seg ? 1u : 0u;
    p.stages = c->cfg.stages;
    p.demux = lists > 1 || (compact && (c->cfg.flags & COP_CFG_DEMUX_PORTS)) ? lists : 0u;
    Lane &L = c->lane[c->next_lane];
    c->next_lane = (c->next_lane + 1) % c->n_lanes;
    return launch_on(c, L, p, imix, pl, count);
}

int cop_sync(cop_ctx *c)
{
    if (!c) return -EINVAL;
    if (int rc = sync_lanes(c)) return rc;
    if (int rc = take_lane_errors(c, 0xFu)) return rc;
    return 0;
}

int cop_poll(cop_ctx *c)
{
    if (!c) return -EINVAL;
    for (int l = 0; l < c->n_lanes; l++) {
        hipError_t e = hipStreamQuery(c->lane[l].s);
        if (e == hipErrorNotReady) return -EAGAIN;
        if (e != hipSuccess) return set_err(c, -EIO, "stream: %s", hipGetErrorString(e));
    }
    if (int rc = take_lane_errors(c, 0xFu)) return rc;
    return 0;
}

void cop_pack_headers(const void *const *pkt_data, uint32_t n, uint8_t *out)
{
    GatherPool::slice(pkt_data, out, n, 1, 0);
}

void cop_pack_headers12(const void *const *pkt_data, uint32_t n, uint8_t *out)
{
    GatherPool::slice(pkt_data, out, n, 1, 0, COP_HDR12_STRIDE);
}

static void host_gather(cop_ctx *c, const void *const *src, uint8_t *dst, uint32_t n)
{
    if (c->gather) c->gather->gather(src, dst, n);
    else GatherPool::slice(src, dst, n, 1, 0);
}

// Small batches: the kernel reads the records from mapped pinned memory and
// writes records and forward list there (one launch and one sync per call,
// no copy-engine round trips); the CPU then copies the records out.
static int process_host_zc(cop_ctx *c, uint32_t stages, const void *const *pkt_data, uint32_t n,
                           cop_result *results, uint32_t *fwd_idx, uint32_t *fwd_count)
{
    if (c->zc_cap < n || !c->zc_stage) {
        const uint32_t cap = n < 1024 ? 1024 : n;
        if (c->zc_stage) (void)hipHostFree(c->zc_stage);
        if (c->zc_res) (void)hipHostFree(c->zc_res);
        if (c->zc_fwd) (void)hipHostFree(c->zc_fwd);
        c->zc_stage = nullptr;
        c->zc_res = nullptr;
        c->zc_fwd = nullptr;
        c->zc_cap = 0;
        HIPCHK(c, hipHostMalloc(&c->zc_stage, (size_t)cap * COP_HDR16_STRIDE, hipHostMallocMapped));
        HIPCHK(c, hipHostMalloc(&c->zc_res, (size_t)cap * sizeof(cop_result), hipHostMallocMapped));
        HIPCHK(c, hipHostMalloc(&c->zc_fwd, (size_t)(cap + 4) * 4, hipHostMallocMapped));
        c->zc_cap = cap;
    }
    if (int rc0 = sync_lanes(c)) return rc0;   // the mapped buffers may still be in use
    uint64_t t0 = c->hprof ? hp_ns() : 0;
    host_gather(c, pkt_data, c->zc_stage, n);
    if (c->hprof) {
        const uint64_t t1 = hp_ns();
        c->hp[0] += t1 - t0;
        t0 = t1;
    }
    void *d_stage = nullptr, *d_res = nullptr, *d_fwd = nullptr;
    HIPCHK(c, hipHostGetDevicePointer(&d_stage, c->zc_stage, 0));
    HIPCHK(c, hipHostGetDevicePointer(&d_res, c->zc_res, 0));
    HIPCHK(c, hipHostGetDevicePointer(&d_fwd, c->zc_fwd, 0));
    cop_batch b;
    memset(&b, 0, sizeof(b));
    b.pkts = d_stage;
    b.n = n;
    b.stride = COP_HDR16_STRIDE;
    b.results = (cop_result *)d_res;
    b.fwd_idx = fwd_idx ? (uint32_t *)d_fwd + 4 : nullptr;
    b.fwd_count = (fwd_idx || fwd_count) ? (uint32_t *)d_fwd : nullptr;
    if (int rc = submit_on(c, c->lane[0], &b, 1, false, stages)) return rc;
    if (c->hprof) {
        const uint64_t t1 = hp_ns();
        c->hp[1] += t1 - t0;
        t0 = t1;
    }
    if (int rc = cop_sync(c)) return rc;
    if (c->hprof) {
        const uint64_t t1 = hp_ns();
        c->hp[2] += t1 - t0;
        t0 = t1;
    }
    memcpy(results, c->zc_res, (size_t)n * sizeof(cop_result));
    const uint32_t cnt = b.fwd_count ? c->zc_fwd[0] : 0u;
    if (fwd_idx && cnt) memcpy(fwd_idx, c->zc_fwd + 4, (size_t)cnt * 4);
    if (fwd_count) *fwd_count = cnt;
    if (c->hprof) {
        c->hp[3] += hp_ns() - t0;
        c->hp[4]++;
        c->hp[5] += n;
    }
    return 0;
}

int cop_process_host(cop_ctx *c, const void *const *pkt_data, uint32_t n, cop_result *results,
                     uint32_t *fwd_idx, uint32_t *fwd_count)
{
    return cop_process_host_stages(c, c ? c->cfg.stages : 0u, pkt_data, n, results, fwd_idx, fwd_count);
}

int cop_process_host_stages(cop_ctx *c, uint32_t stages, const void *const *pkt_data, uint32_t n,
                            cop_result *results, uint32_t *fwd_idx, uint32_t *fwd_count)
{
    if (!c || (n && (!pkt_data || !results))) return -EINVAL;
    if (n > c->cfg.max_batch) return set_err(c, -EINVAL, "n %u > max_batch", n);
    HIPCHK(c, hipSetDevice(c->device));
    if (n <= c->zc_max) return process_host_zc(c, stages, pkt_data, n, results, fwd_idx, fwd_count);
    if (c->stage_cap < n || !c->h_stage) {
        uint32_t cap = n < 1024 ? 1024 : n;
        if (c->h_stage) (void)hipHostFree(c->h_stage);
        if (c->d_stage) (void)hipFree(c->d_stage);
        if (c->d_res) (void)hipFree(c->d_res);
        if (c->d_fwd) (void)hipFree(c->d_fwd);
        if (c->d_fwdn) (void)hipFree(c->d_fwdn);
        c->h_stage = nullptr;
        c->d_stage = nullptr;
        c->d_res = nullptr;
        c->d_fwd = nullptr;
        c->d_fwdn = nullptr;
        c->stage_cap = 0;
        HIPCHK(c, hipHostMalloc(&c->h_stage, (size_t)cap * COP_HDR16_STRIDE, hipHostMallocDefault));
        HIPCHK(c, hipMalloc(&c->d_stage, (size_t)cap * COP_HDR16_STRIDE));
        HIPCHK(c, hipMalloc(&c->d_res, (size_t)cap * 8));
        HIPCHK(c, hipMalloc(&c->d_fwd, (size_t)cap * 4));
        HIPCHK(c, hipMalloc(&c->d_fwdn, 16));
        c->stage_cap = cap;
    }
    if (int rc0 = sync_lanes(c)) return rc0;   // the staging buffers may still be in use
    // gather the 16 header bytes of every packet the pipeline reads
    host_gather(c, pkt_data, c->h_stage, n);
    HIPCHK(c, hipMemcpyAsync(c->d_stage, c->h_stage, (size_t)n * COP_HDR16_STRIDE, hipMemcpyHostToDevice, c->stream));
    cop_batch b;
    memset(&b, 0, sizeof(b));
    b.pkts = c->d_stage;
    b.n = n;
    b.stride = COP_HDR16_STRIDE;
    b.results = c->d_res;
    b.fwd_idx = fwd_idx ? c->d_fwd : nullptr;
    b.fwd_count = (fwd_idx || fwd_count) ? c->d_fwdn : nullptr;
    int rc = submit_on(c, c->lane[0], &b, 1, false, stages);
    if (rc) return rc;
    HIPCHK(c, hipMemcpyAsync(results, c->d_res, (size_t)n * 8, hipMemcpyDeviceToHost, c->stream));
    uint32_t cnt = 0;
    if (b.fwd_count) {
        HIPCHK(c, hipMemcpyAsync(&cnt, c->d_fwdn, 4, hipMemcpyDeviceToHost, c->stream));
    }
    rc = cop_sync(c);
    if (rc) return rc;
    if (fwd_idx && cnt) HIPCHK(c, hipMemcpy(fwd_idx, c->d_fwd, (size_t)cnt * 4, hipMemcpyDeviceToHost));
    if (fwd_count) *fwd_count = cnt;
    return 0;
}

int cop_set_host_threads(cop_ctx *c, uint32_t n)
{
    if (!c || n == 0 || n > 256) return -EINVAL;
    delete c->gather;
    c->gather = nullptr;
    if (n > 1) {
        c->gather = new (std::nothrow) GatherPool();
        if (!c->gather) return -ENOMEM;
        c->gather->start((int)n);
    }
    return 0;
}

uint32_t cop_ctx_max_batch(const cop_ctx *c) { return c ? c->cfg.max_batch : 0u; }

int cop_host_batch_submit(cop_ctx *c, uint32_t slot, const void *const *pkt_data, uint32_t n)
{
    return cop_host_batch_submit_stages(c, c ? c->cfg.stages : 0u, slot, pkt_data, n);
}

int cop_host_batch_submit_stages(cop_ctx *c, uint32_t stages, uint32_t slot, const void *const *pkt_data, uint32_t n)
{
    if (!c || slot >= COP_HOST_SLOTS || (n && !pkt_data)) return -EINVAL;
    if (n > c->cfg.max_batch) return set_err(c, -EINVAL, "n %u > max_batch", n);
    auto &h = c->hs[slot];
    if (h.busy) return set_err(c, -EBUSY, "host slot %u still in flight", slot);
    Lane &L = c->lane[slot % (uint32_t)c->n_lanes];
    HIPCHK(c, hipSetDevice(c->device));
    if (h.cap < n || !h.h_stage) {
        const uint32_t cap = n < 1024 ? 1024 : n;
        if (h.h_stage) (void)hipHostFree(h.h_stage);
        if (h.h_res) (void)hipHostFree(h.h_res);
        h.h_stage = h.d_stage = nullptr;
        h.h_res = h.d_res = nullptr;
        h.cap = 0;
        // mapped pinned memory: the kernel reads the records and writes the
        // results in host memory (no copy-engine round trips); d_* are the
        // device's addresses of the same buffers
        HIPCHK(c, hipHostMalloc(&h.h_stage, (size_t)cap * COP_HDR16_STRIDE, hipHostMallocMapped));
        HIPCHK(c, hipHostMalloc(&h.h_res, (size_t)cap * sizeof(cop_result), hipHostMallocMapped));
        void *ds = nullptr, *dr = nullptr;
        HIPCHK(c, hipHostGetDevicePointer(&ds, h.h_stage, 0));
        HIPCHK(c, hipHostGetDevicePointer(&dr, h.h_res, 0));
        h.d_stage = (uint8_t *)ds;
        h.d_res = (cop_result *)dr;
        h.cap = cap;
    }
    if (!h.done) HIPCHK(c, hipEventCreateWithFlags(&h.done, hipEventDisableTiming));
    h.n = n;
    if (n) {
        // the 16-byte header records into mapped memory, then the pipeline
        uint64_t t0 = c->hprof ? hp_ns() : 0;
        host_gather(c, pkt_data, h.h_stage, n);
        if (c->hprof) {
            const uint64_t t1 = hp_ns();
            c->hp[0] += t1 - t0;
            t0 = t1;
        }
        cop_batch b;
        memset(&b, 0, sizeof(b));
        b.pkts = h.d_stage;
        b.n = n;
        b.stride = COP_HDR16_STRIDE;
        b.results = h.d_res;
        if (int rc = submit_on(c, L, &b, 1, false, stages)) return rc;
        if (c->hprof) {
            c->hp[1] += hp_ns() - t0;
            c->hp[4]++;
            c->hp[5] += n;
        }
    }
    HIPCHK(c, hipEventRecord(h.done, L.s));
    h.busy = true;
    return 0;
}

int cop_host_batch_wait(cop_ctx *c, uint32_t slot, const cop_result **results, uint32_t *n)
{
    if (!c || slot >= COP_HOST_SLOTS) return -EINVAL;
    auto &h = c->hs[slot];
    if (!h.busy) return set_err(c, -EINVAL, "host slot %u has no batch", slot);
    const uint64_t t0 = c->hprof ? hp_ns() : 0;
    hipError_t e = hipEventSynchronize(h.done);
    if (c->hprof) c->hp[2] += hp_ns() - t0;
    if (c->inject_wait) {
        c->inject_wait--;
        e = hipErrorUnknown;
    }
    h.busy = false;   // on every path: a failed wait must not wedge the slot
    if (e != hipSuccess) return set_err(c, -EIO, "host slot %u: %s", slot, hipGetErrorString(e));
    // only this slot's lane: another lane's timeout does not void these results
    if (int rc = take_lane_errors(c, 1u << (slot % (uint32_t)c->n_lanes))) return rc;
    if (results) *results = h.h_res;
    if (n) *n = h.n;
    return 0;
}

static int lane_finish(cop_ctx *c, Lane &L, cop_result *results)
{
    if (!L.busy) return 0;
    HIPCHK(c, hipEventSynchronize(L.done));
    memcpy(results + L.first, L.h_res, (size_t)L.n * sizeof(cop_result));
    L.busy = false;
    return 0;
}

int cop_process_host_stream(cop_ctx *c, const void *const *pkt_data, uint64_t n, uint32_t batch,
                            cop_result *results)
{
    if (!c || (n && (!pkt_data || !results)) || batch == 0) return -EINVAL;
    if (batch > c->cfg.max_batch) return set_err(c, -EINVAL, "batch %u > max_batch", batch);
    if (int rc = sync_lanes(c)) return rc;
    // zc 1: staging and records mapped; 2: records mapped, staging copied.
    // rec: the staged header record, 12 bytes (default) or 16
    const int zc = c->stream_zc;
    const bool zc_in = zc == 1, zc_out = zc != 0;
    const uint32_t rec = c->stream_rec;
    for (int l = 0; l < c->n_lanes; l++) {
        Lane &L = c->lane[l];
        if (L.cap >= batch && L.zc == zc) continue;
        if (L.h_stage) (void)hipHostFree(L.h_stage);
        if (L.h_res) (void)hipHostFree(L.h_res);
        if (L.d_stage) (void)hipFree(L.d_stage);
        if (L.d_res) (void)hipFree(L.d_res);
        L.h_stage = L.d_stage = L.m_stage = nullptr;
        L.h_res = L.d_res = L.m_res = nullptr;
        L.cap = 0;
        L.zc = zc;
        if (zc_in) {
            HIPCHK(c, hipHostMalloc(&L.h_stage, (size_t)batch * COP_HDR16_STRIDE, hipHostMallocMapped));
            void *ds = nullptr;
            HIPCHK(c, hipHostGetDevicePointer(&ds, L.h_stage, 0));
            L.m_stage = (uint8_t *)ds;
        } else {
            HIPCHK(c, hipHostMalloc(&L.h_stage, (size_t)batch * COP_HDR16_STRIDE, hipHostMallocDefault));
            HIPCHK(c, hipMalloc(&L.d_stage, (size_t)batch * COP_HDR16_STRIDE));
        }
        if (zc_out) {
            HIPCHK(c, hipHostMalloc(&L.h_res, (size_t)batch * 8, hipHostMallocMapped));
            void *dr = nullptr;
            HIPCHK(c, hipHostGetDevicePointer(&dr, L.h_res, 0));
            L.m_res = (cop_result *)dr;
        } else {
            HIPCHK(c, hipHostMalloc(&L.h_res, (size_t)batch * 8, hipHostMallocDefault));
            HIPCHK(c, hipMalloc(&L.d_res, (size_t)batch * 8));
        }
        L.cap = batch;
    }
    // Batch bi runs on lane bi % n_lanes. Preparing it waits for that lane's
    // previous batch, copies that batch's records out and gathers bi's
    // header records into the lane's staging. With two or more lanes and a
    // gather pool, batch bi + 1 is prepared by the pool's workers while the
    // caller issues batch bi's copy and launch (whose API calls would
    // otherwise sit between two gathers); one lane reuses one staging, so it
    // prepares in line.
    const uint64_t nb = (n + batch - 1) / batch;
    const bool overlap = c->gather && c->gather->th.size() > 0 && c->n_lanes > 1;
    auto prepare = [&](uint64_t bi, bool async) -> int {
        Lane &L = c->lane[bi % (uint64_t)c->n_lanes];
        const uint64_t first = bi * batch;
        const uint32_t k = (uint32_t)std::min<uint64_t>(batch, n - first);
        const cop_result *prev = nullptr;
        uint32_t prev_n = 0;
        uint64_t prev_first = 0;
        if (L.busy) {
            HIPCHK(c, hipEventSynchronize(L.done));
            L.busy = false;
            prev = L.h_res;
            prev_n = L.n;
            prev_first = L.first;
        }
        cop_result *prev_dst = prev ? results + prev_first : nullptr;
        const size_t prev_bytes = (size_t)prev_n * sizeof(cop_result);
        if (c->gather && async) {
            c->gather->start_async(pkt_data + first, L.h_stage, k, prev, prev_dst, prev_bytes, rec);
        } else if (c->gather) {
            c->gather->run(pkt_data + first, L.h_stage, k, prev, prev_dst, prev_bytes, rec);
        } else {
            if (prev_n) memcpy(prev_dst, prev, prev_bytes);
            GatherPool::slice(pkt_data + first, L.h_stage, k, 1, 0, rec);
        }
        return 0;
    };
    auto issue = [&](uint64_t bi) -> int {
        Lane &L = c->lane[bi % (uint64_t)c->n_lanes];
        const uint64_t first = bi * batch;
        const uint32_t k = (uint32_t)std::min<uint64_t>(batch, n - first);
        // (c->dbg & 0x100: timing ablation, the H2D copy skipped; results wrong)
        if (!zc_in && !(c->dbg & 0x100u))
            HIPCHK(c, hipMemcpyAsync(L.d_stage, L.h_stage, (size_t)k * rec, hipMemcpyHostToDevice, L.s));
        cop_batch b;
        memset(&b, 0, sizeof(b));
        b.pkts = zc_in ? L.m_stage : L.d_stage;
        b.n = k;
        b.stride = rec;
        b.results = zc_out ? L.m_res : L.d_res;
        if (int rc = submit_on(c, L, &b, 1, false, c->cfg.stages)) return rc;
        if (!zc_out) HIPCHK(c, hipMemcpyAsync(L.h_res, L.d_res, (size_t)k * 8, hipMemcpyDeviceToHost, L.s));
        HIPCHK(c, hipEventRecord(L.done, L.s));
        L.busy = true;
        L.first = first;
        L.n = k;
        return 0;
    };
    if (nb)
        if (int rc = prepare(0, false)) return rc;
    for (uint64_t bi = 0; bi < nb; bi++) {
        const bool pre = overlap && bi + 1 < nb;
        if (pre)
            if (int rc = prepare(bi + 1, true)) return rc;
        const int rc = issue(bi);
        if (pre) c->gather->wait();   // (also on an error: the workers are done with the staging)
        if (rc) return rc;
        if (!overlap && bi + 1 < nb)
            if (int rc2 = prepare(bi + 1, false)) return rc2;
    }
    for (int l = 0; l < c->n_lanes; l++)
        if (int rc = lane_finish(c, c->lane[l], results)) return rc;
    if (int rc = take_lane_errors(c, 0xFu)) return rc;
    return 0;
}

static int pmd_hits_flush(cop_ctx *c);
static int pmd_pause(cop_ctx *c);
static int pmd_resume(cop_ctx *c);

// The telemetry scratch: every counter word (shards, port shards, rules),
// so a snapshot never reallocates it (hipFree synchronises the whole
// device: it would wait for launches in flight and for a poll-mode kernel)
static int tele_scratch(cop_ctx *c)
{
    HIPCHK(c, hipSetDevice(c->device));
    if (!c->tele_stream) HIPCHK(c, hipStreamCreateWithFlags(&c->tele_stream, hipStreamNonBlocking));
    const size_t n = RULE_OFF + c->n_rule_ctr;
    if (c->tele_words < n) {
        if (c->tele_dev) (void)hipFree(c->tele_dev);
        c->tele_dev = nullptr;
        c->tele_words = 0;
        HIPCHK(c, hipMalloc(&c->tele_dev, n * 8));
        c->tele_words = n;
    }
    return 0;
}

// Counter words [off, off + n) of the counter block into host memory `out`,
// read — or atomically exchanged with 0 when reset — by a small kernel on
// the telemetry stream: an increment lands before the exchange (this read)
// or after it (the next), none is lost or counted twice. Beside one-shot
// launches it does not wait for them. A poll-mode kernel is paused for it
// (pmd_pause: a kernel of another stream is not guaranteed a place beside
// it) and relaunched after.
static int exchange_words(cop_ctx *c, size_t off, size_t n, uint64_t *out, int reset)
{
    if (int rc = tele_scratch(c)) return rc;
    if (int rc = pmd_pause(c)) return rc;
    int rc = 0;
    for (size_t done = 0; done < n && !rc;) {
        const uint32_t k = (uint32_t)std::min<size_t>(n - done, (size_t)1 << 30);
        hipError_t e = copk_snapshot(c->counters + off + done, k, c->tele_dev + done, reset ? 1 : 0, c->tele_stream);
        if (e != hipSuccess) rc = set_err(c, -EIO, "snapshot: %s", hipGetErrorString(e));
        done += k;
    }
    if (!rc && hipMemcpyAsync(out, c->tele_dev, n * 8, hipMemcpyDeviceToHost, c->tele_stream) != hipSuccess)
        rc = set_err(c, -EIO, "snapshot copy");
    if (!rc && hipStreamSynchronize(c->tele_stream) != hipSuccess) rc = set_err(c, -EIO, "snapshot sync");
    const int rrc = pmd_resume(c);
    return rc ? rc : rrc;
}

int cop_counters_read(cop_ctx *c, cop_counters *out, int reset)
{
    if (!c || !out) return -EINVAL;
    if (int rc = sync_lanes(c)) return rc;
    std::vector<uint64_t> sh(SHARD_WORDS);
    if (c->pmd) {
        // the poll-mode kernel may be adding: read (and zero) atomically
        if (int rc = exchange_words(c, 0, SHARD_WORDS, sh.data(), reset)) return rc;
    } else {
        HIPCHK(c, hipMemcpy(sh.data(), c->counters, sh.size() * 8, hipMemcpyDeviceToHost));
        if (reset) HIPCHK(c, memset_sync(c->counters, 0, sh.size() * 8, c->stream));
    }
    uint64_t sum[COP_N_COUNTERS] = {0};
    for (int s = 0; s < COPK_COUNTER_SHARDS; s++)
        for (int k = 0; k < COP_N_COUNTERS; k++) sum[k] += sh[(size_t)s * COP_N_COUNTERS + k];
    memcpy(out, sum, sizeof(cop_counters));
    return 0;
}

void *cop_counters_device_ptr(cop_ctx *c) { return c ? (void *)c->counters : nullptr; }

// fold the port shards into per-port coprocessor_stats
static void fold_ports(const uint64_t *sh, cop_port_stats *out, uint32_t n)
{
    for (uint32_t q = 0; q < n; q++) {
        uint64_t rx = 0, tx = 0;
        for (int s = 0; s < COPK_COUNTER_SHARDS; s++) {
            rx += sh[(size_t)s * COPK_PORT_WORDS + 2 * q];
            tx += sh[(size_t)s * COPK_PORT_WORDS + 2 * q + 1];
        }
        memset(&out[q], 0, sizeof(out[q]));
        out[q].rx_packets = rx;
        out[q].tx_packets = tx;
        out[q].nf_dropped = rx - tx;
    }
}

static void fold_shards(const uint64_t *sh, cop_counters *out)
{
    uint64_t sum[COP_N_COUNTERS] = {0};
    for (int s = 0; s < COPK_COUNTER_SHARDS; s++)
        for (int k = 0; k < COP_N_COUNTERS; k++) sum[k] += sh[(size_t)s * COP_N_COUNTERS + k];
    memcpy(out, sum, sizeof(cop_counters));
}

int cop_port_stats_read(cop_ctx *c, cop_port_stats *out, uint32_t n, int reset)
{
    if (!c || (n && !out)) return -EINVAL;
    if (!(c->cfg.flags & COP_CFG_PORT_STATS)) return set_err(c, -EINVAL, "port stats not enabled");
    if (n > c->cfg.n_ports) n = c->cfg.n_ports;
    if (int rc = sync_lanes(c)) return rc;
    std::vector<uint64_t> sh(PORT_WORDS);
    if (c->pmd) {
        if (int rc = exchange_words(c, SHARD_WORDS, PORT_WORDS, sh.data(), reset)) return rc;
    } else {
        HIPCHK(c, hipMemcpy(sh.data(), c->counters + SHARD_WORDS, PORT_WORDS * 8, hipMemcpyDeviceToHost));
        if (reset) HIPCHK(c, memset_sync(c->counters + SHARD_WORDS, 0, PORT_WORDS * 8, c->stream));
    }
    fold_ports(sh.data(), out, n);
    return (int)c->cfg.n_ports;
}

// Live read(-and-zero) while launches are in flight or a poll-mode kernel
// runs (exchange_words): the print_stats read-and-zero (switch.c:33-90).
int cop_counters_snapshot(cop_ctx *c, cop_counters *total, cop_port_stats *ports, uint32_t n_ports, int reset)
{
    if (!c || (n_ports && !ports)) return -EINVAL;
    if (!c->tele_host) {
        HIPCHK(c, hipSetDevice(c->device));
        HIPCHK(c, hipHostMalloc(&c->tele_host, RULE_OFF * 8, hipHostMallocDefault));
    }
    if (int rc = exchange_words(c, 0, RULE_OFF, c->tele_host, reset)) return rc;
    if (total) fold_shards(c->tele_host, total);
    if (n_ports) {
        if (n_ports > c->cfg.n_ports) n_ports = c->cfg.n_ports;
        fold_ports(c->tele_host + SHARD_WORDS, ports, n_ports);
    }
    return 0;
}

int cop_rule_counters_read(cop_ctx *c, uint64_t *out, uint32_t cap, int reset)
{
    if (!c || (cap && !out)) return -EINVAL;
    if (!(c->cfg.flags & COP_CFG_RULE_COUNTERS)) return set_err(c, -EINVAL, "rule counters not enabled");
    if (int rc = sync_lanes(c)) return rc;
    if (int rc = pmd_hits_flush(c)) return rc;   // poll mode: count the binned hits of completed batches
    unsigned long long *d = c->counters + RULE_OFF;
    const uint32_t k = cap < c->n_rule_ctr ? cap : c->n_rule_ctr;
    if (c->pmd && reset) {
        // read-and-zero of every rule word at once, beside the running kernel
        std::vector<uint64_t> all(c->n_rule_ctr);
        if (c->n_rule_ctr)
            if (int rc = exchange_words(c, RULE_OFF, c->n_rule_ctr, all.data(), 1)) return rc;
        if (k) memcpy(out, all.data(), (size_t)k * 8);
        return (int)c->n_rule_ctr;
    }
    if (k) HIPCHK(c, hipMemcpy(out, d, (size_t)k * 8, hipMemcpyDeviceToHost));
    if (reset && c->n_rule_ctr) HIPCHK(c, memset_sync(d, 0, (size_t)c->n_rule_ctr * 8, c->stream));
    return (int)c->n_rule_ctr;
}

int cop_rule_counters_device_ptr(cop_ctx *c, void **dptr, uint32_t *n_rules)
{
    if (!c || !dptr) return -EINVAL;
    if (!(c->cfg.flags & COP_CFG_RULE_COUNTERS)) return set_err(c, -EINVAL, "rule counters not enabled");
    *dptr = c->counters + RULE_OFF;
    if (n_rules) *n_rules = c->n_rule_ctr;
    return 0;
}

// ---- RCCL (xGMI) counter reduction ----------------------------------------
// librccl is opened lazily so that the library (and every single-GPU path)
// works on hosts without it.
namespace {
struct Rccl {
    bool tried = false, ok = false;
    ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*all_reduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                               hipStream_t) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    const char *(*error_string)(ncclResult_t) = nullptr;
};
Rccl g_rccl;
}  // namespace

static bool rccl_load()
{
    Rccl &r = g_rccl;
    if (r.tried) return r.ok;
    r.tried = true;
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) return false;
    r.get_unique_id = (decltype(r.get_unique_id))dlsym(h, "ncclGetUniqueId");
    r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(h, "ncclCommInitRank");
    r.all_reduce = (decltype(r.all_reduce))dlsym(h, "ncclAllReduce");
    r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
    r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
    r.ok = r.get_unique_id && r.comm_init_rank && r.all_reduce && r.comm_destroy && r.error_string;
    return r.ok;
}

static void coll_destroy(cop_ctx *c)
{
    if (c->comm && g_rccl.ok) (void)g_rccl.comm_destroy(c->comm);
    c->comm = nullptr;
}

int cop_coll_unique_id(uint8_t id[COP_COLL_ID_BYTES])
{
    if (!id) return -EINVAL;
    if (!rccl_load()) return -ENOSYS;
    ncclUniqueId u;
    if (g_rccl.get_unique_id(&u) != ncclSuccess) return -EIO;
    memcpy(id, u.internal, COP_COLL_ID_BYTES);
    return 0;
}

static int coll_init_free(cop_ctx *c, const uint8_t id[COP_COLL_ID_BYTES], int rank, int nranks);

int cop_coll_init(cop_ctx *c, const uint8_t id[COP_COLL_ID_BYTES], int rank, int nranks)
{
    if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks) return -EINVAL;
    if (!rccl_load()) return set_err(c, -ENOSYS, "librccl not available");
    HIPCHK(c, hipSetDevice(c->device));
    // the communicator's set-up, its buffers (hipFree synchronises the
    // device) and the prewarm all-reduce run with the GPU free, as every
    // reduce does: a poll-mode kernel serving this context is paused around
    // them (it holds every workgroup slot it could get)
    if (int rc = pmd_pause(c)) return rc;
    const int rc = coll_init_free(c, id, rank, nranks);
    const int rrc = pmd_resume(c);
    return rc ? rc : rrc;
}

// cop_coll_init with no poll-mode kernel on the GPU
static int coll_init_free(cop_ctx *c, const uint8_t id[COP_COLL_ID_BYTES], int rank, int nranks)
{
    coll_destroy(c);
    ncclUniqueId u;
    memcpy(u.internal, id, COP_COLL_ID_BYTES);
    ncclResult_t r = g_rccl.comm_init_rank(&c->comm, nranks, u, rank);
    if (r != ncclSuccess) {
        c->comm = nullptr;
        return set_err(c, -EIO, "ncclCommInitRank: %s", g_rccl.error_string(r));
    }
    // one all-reduce of a single word now (every rank is in this call): the
    // communicator's lazy set-up and its kernels' first dispatch happen here,
    // not in the first reporting interval beside a running poll-mode kernel
    // ($COP_COLL_PREWARM=0: off, experiments)
    const char *pw = getenv("COP_COLL_PREWARM");
    if (pw && !atoi(pw)) return 0;
    // the reduce's buffers at their full size now (every counter word), so
    // a reporting interval allocates nothing
    const size_t words = RULE_OFF + c->n_rule_ctr;
    if (c->ctr_sum_words < words) {
        if (c->ctr_sum) (void)hipFree(c->ctr_sum);
        c->ctr_sum = nullptr;
        c->ctr_sum_words = 0;
        HIPCHK(c, hipMalloc(&c->ctr_sum, words * 8));
        c->ctr_sum_words = words;
    }
    if (c->ctr_snap_words < words) {
        if (c->ctr_snap) (void)hipFree(c->ctr_snap);
        c->ctr_snap = nullptr;
        c->ctr_snap_words = 0;
        HIPCHK(c, hipMalloc(&c->ctr_snap, words * 8));
        c->ctr_snap_words = words;
    }
    r = g_rccl.all_reduce(c->counters, c->ctr_sum, 1, ncclUint64, ncclSum, c->comm, c->stream);
    if (r != ncclSuccess) return set_err(c, -EIO, "ncclAllReduce: %s", g_rccl.error_string(r));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return 0;
}

static int coll_reduce_free(cop_ctx *c, cop_counters *total, uint64_t *rule_hits, uint32_t cap, int reset);
static int pmd_hits_sync(cop_pmd *m, uint64_t upto);
static uint64_t pmd_refresh(cop_pmd *m, uint32_t r);

int cop_coll_reduce_counters(cop_ctx *c, cop_counters *total, uint64_t *rule_hits, uint32_t cap, int reset)
{
    if (!c || (cap && !rule_hits)) return -EINVAL;
    if (!c->comm) return set_err(c, -EINVAL, "cop_coll_init not called");
    if (int rc = sync_lanes(c)) return rc;
    // the snapshot and the all-reduce run with the GPU free (pmd_pause):
    // RCCL's kernels need room on every rank's GPU
    if (int rc = pmd_pause(c)) return rc;
    int rc = coll_reduce_free(c, total, rule_hits, cap, reset);
    const int rrc = pmd_resume(c);
    return rc ? rc : rrc;
}

// cop_coll_reduce_counters with no poll-mode kernel on the GPU
static int coll_reduce_free(cop_ctx *c, cop_counters *total, uint64_t *rule_hits, uint32_t cap, int reset)
{
    if (c->pmd) {
        if (int rc = pmd_hits_sync(c->pmd, pmd_refresh(c->pmd, 0))) return rc;
    }
    const size_t shard_words = SHARD_WORDS;
    const size_t words = RULE_OFF + c->n_rule_ctr;
    if (c->ctr_sum_words < words) {
        if (c->ctr_sum) (void)hipFree(c->ctr_sum);
        c->ctr_sum = nullptr;
        c->ctr_sum_words = 0;
        HIPCHK(c, hipMalloc(&c->ctr_sum, words * 8));
        c->ctr_sum_words = words;
    }
    // reset: read-and-zero every word first (an atomic exchange, so adds of
    // a poll-mode kernel running beside it land in this interval or the
    // next), then reduce that snapshot
    const unsigned long long *src = c->counters;
    if (reset) {
        if (c->ctr_snap_words < words) {
            if (c->ctr_snap) (void)hipFree(c->ctr_snap);
            c->ctr_snap = nullptr;
            c->ctr_snap_words = 0;
            HIPCHK(c, hipMalloc(&c->ctr_snap, words * 8));
            c->ctr_snap_words = words;
        }
        hipError_t e = copk_snapshot(c->counters, (uint32_t)words, c->ctr_snap, 1, c->stream);
        if (e != hipSuccess) return set_err(c, -EIO, "snapshot: %s", hipGetErrorString(e));
        src = c->ctr_snap;
    }
    // ranks hold the same rule table, so the per-rule ranges line up
    ncclResult_t r = g_rccl.all_reduce(src, c->ctr_sum, words, ncclUint64, ncclSum, c->comm, c->stream);
    if (r != ncclSuccess) return set_err(c, -EIO, "ncclAllReduce: %s", g_rccl.error_string(r));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (total) {
        std::vector<uint64_t> sh(shard_words);
        HIPCHK(c, hipMemcpy(sh.data(), c->ctr_sum, shard_words * 8, hipMemcpyDeviceToHost));
        uint64_t sum[COP_N_COUNTERS] = {0};
        for (int s = 0; s < COPK_COUNTER_SHARDS; s++)
            for (int k = 0; k < COP_N_COUNTERS; k++) sum[k] += sh[(size_t)s * COP_N_COUNTERS + k];
        memcpy(total, sum, sizeof(cop_counters));
    }
    const uint32_t k = cap < c->n_rule_ctr ? cap : c->n_rule_ctr;
    if (k) HIPCHK(c, hipMemcpy(rule_hits, c->ctr_sum + RULE_OFF, (size_t)k * 8, hipMemcpyDeviceToHost));
    return (int)c->n_rule_ctr;
}

int cop_dev_alloc(cop_ctx *c, size_t bytes, void **dptr)
{
    if (!c || !dptr) return -EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMalloc(dptr, bytes ? bytes : 16));
    return 0;
}

int cop_dev_alloc_ex(cop_ctx *c, size_t bytes, uint32_t flags, void **dptr)
{
    if (!c || !dptr || (flags != 0 && flags != COP_ALLOC_UNCACHED && flags != COP_ALLOC_FINEGRAINED)) return -EINVAL;
    if (!flags) return cop_dev_alloc(c, bytes, dptr);
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipExtMallocWithFlags(dptr, bytes ? bytes : 16,
                                    flags == COP_ALLOC_UNCACHED ? hipDeviceMallocUncached : hipDeviceMallocFinegrained));
    return 0;
}

int cop_dev_free(cop_ctx *c, void *dptr)
{
    if (!c) return -EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipFree(dptr));
    return 0;
}

int cop_host_alloc_pinned(cop_ctx *c, size_t bytes, void **hptr)
{
    if (!c || !hptr) return -EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipHostMalloc(hptr, bytes ? bytes : 16, hipHostMallocDefault));
    return 0;
}

int cop_host_alloc_mapped(cop_ctx *c, size_t bytes, void **hptr, void **dptr)
{
    if (!c || !hptr || !dptr) return -EINVAL;
    HIPCHK(c, hipSetDevice(c->device));
    // coherent (fine-grained): a poll-mode kernel never ends, so its stores
    // must reach host memory without the kernel-end write-back of the L2
    HIPCHK(c, hipHostMalloc(hptr, bytes ? bytes : 16, hipHostMallocMapped | hipHostMallocCoherent));
    hipError_t e = hipHostGetDevicePointer(dptr, *hptr, 0);
    if (e != hipSuccess) {
        (void)hipHostFree(*hptr);
        *hptr = nullptr;
        return set_err(c, -EIO, "mapping: %s", hipGetErrorString(e));
    }
    return 0;
}

int cop_host_free_pinned(cop_ctx *c, void *hptr)
{
    if (!c) return -EINVAL;
    HIPCHK(c, hipHostFree(hptr));
    return 0;
}

int cop_memcpy_h2d(cop_ctx *c, void *dst, const void *src, size_t bytes)
{
    if (!c) return -EINVAL;
    if (int rc = sync_lanes(c)) return rc;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return 0;
}

int cop_memcpy_d2h(cop_ctx *c, void *dst, const void *src, size_t bytes)
{
    if (!c) return -EINVAL;
    if (int rc = sync_lanes(c)) return rc;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return 0;
}

int cop_memcpy_d2d(cop_ctx *c, void *dst, const void *src, size_t bytes)
{
    if (!c) return -EINVAL;
    if (int rc = sync_lanes(c)) return rc;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return 0;
}

int cop_memset_d(cop_ctx *c, void *dst, int value, size_t bytes)
{
    if (!c) return -EINVAL;
    if (int rc = sync_lanes(c)) return rc;
    HIPCHK(c, hipSetDevice(c->device));
    HIPCHK(c, hipMemsetAsync(dst, value, bytes, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return 0;
}

int cop_timer_start(cop_ctx *c)
{
    if (!c) return -EINVAL;
    HIPCHK(c, hipEventRecord(c->t0, c->stream));
    for (int l = 1; l < c->n_lanes; l++) HIPCHK(c, hipStreamWaitEvent(c->lane[l].s, c->t0, 0));
    return 0;
}

int cop_timer_stop(cop_ctx *c, double *ms)
{
    if (!c || !ms) return -EINVAL;
    for (int l = 1; l < c->n_lanes; l++) {
        HIPCHK(c, hipEventRecord(c->lane[l].join, c->lane[l].s));
        HIPCHK(c, hipStreamWaitEvent(c->stream, c->lane[l].join, 0));
    }
    HIPCHK(c, hipEventRecord(c->t1, c->stream));
    HIPCHK(c, hipEventSynchronize(c->t1));
    float f = 0;
    HIPCHK(c, hipEventElapsedTime(&f, c->t0, c->t1));
    *ms = f;
    return 0;
}


// ---- poll-mode kernel (cop_pmd.hip) ---------------------------------------
// A persistent kernel serving one or several batch rings: the host posts a
// ring's batches by bumping its counter in mapped host memory and reads
// their completion from per-slot words the kernel writes there. No launch,
// no per-launch ramp, tables staged into LDS once per worker.

struct PmdRing {
    std::atomic<uint64_t> posted{0};      // batches posted (written by the ring's thread)
    std::atomic<uint64_t> completed{0};   // first batch not known complete (the ring's thread)
};

struct cop_pmd {
    cop_ctx *c = nullptr;
    hipStream_t s = nullptr;
    CopKPmd P{};
    int fw_mode = 0, lpm_mode = 0, layout = 0, ppt = 0, ext = 0;
    uint32_t lds_bytes = 0;
    uint8_t *ctl = nullptr;                 // mapped host control block
    volatile uint32_t *h_stop = nullptr;
    volatile uint32_t *h_state = nullptr;
    volatile uint64_t *h_done = nullptr;    // [r * n_slots + slot]: sequence + 1 of its last completed batch
    volatile uint32_t *h_n = nullptr;       // [r * n_slots + slot]: packets of the posted batch (variable n)
    uint8_t *dev = nullptr;                 // device words: ctl, gates, relays, slot tile counts, look-back
    size_t dev_bytes = 0;
    uint32_t n_rings = 1, n_slots = 0, tpb = 0, per_cu = 0, ring_n = 0;
    uint32_t acquire = 4;       // CopKPmd::sys_acquire: 4 coherent loads on slot reuse (default), 3 on every tile, 0 never
    bool dyn = false;           // CopKPmd::dyn: dynamic tiles
    bool pf = false;            // CopKPmd::dyn 2: the static order with the next tile prefetched
    std::atomic<uint32_t> launches{0};
    uint32_t pauses = 0;                    // pmd_pause calls that stopped a running kernel
    bool was_live = false;                  // pmd_pause found it running (pmd_resume relaunches)
    bool live = false;                      // a launch may still be running
    std::mutex mu;                          // relaunch after an idle exit, from any ring's thread
    PmdRing ring[COPK_PMD_MAX_RINGS];
    // per-rule hits by binning (one ring only): tile (slot, j) parks its
    // sorted hit ids in region slot*tpb + j; cop_hit_count adds them up on
    // stream hs, over runs of completed batches, before their slots are
    // posted again
    bool bins = false;
    hipStream_t hs = nullptr;
    uint64_t counted = 0;                   // batches < counted have their count launched
    uint64_t count_synced = 0;              // ... and completed
    volatile uint64_t *h_posted(uint32_t r) const { return (volatile uint64_t *)(ctl + 64 * (size_t)r); }
};

// host control block: [64 r] ring r's posted count, [512] stop, [516] state
// words, [576] the completion words, then the batch sizes (variable n)
constexpr size_t PMD_H_STOP = 512, PMD_H_STATE = 516, PMD_H_DONE = 576;
// device words: [8] d_ctl, [64] d_act, [1024 + 128 r] ring r's gate,
// [2048 + 128 (8 r + x)] its relays, [PMD_TICKET_OFF + 128 r] its tile
// ticket (dynamic tiles), then the slot tile counts, then the look-back
// chains (dense lists)
constexpr size_t PMD_ACT_OFF = 64;
constexpr size_t PMD_GATE_OFF = 1024;
constexpr size_t PMD_RELAY_OFF = 2048;
constexpr size_t PMD_TICKET_OFF = PMD_RELAY_OFF + 128 * COPK_PMD_RELAYS * COPK_PMD_MAX_RINGS;   // dynamic tiles
constexpr size_t PMD_CTL_BYTES = PMD_TICKET_OFF + 128 * COPK_PMD_TK_LANES * COPK_PMD_MAX_RINGS;
static_assert(PMD_GATE_OFF + 128 * COPK_PMD_MAX_RINGS <= PMD_RELAY_OFF, "gates overlap relays");
static_assert(64 * COPK_PMD_MAX_RINGS <= PMD_H_STOP, "posted words overlap the stop word");

// the first batch of ring r not complete, from the completion words (a scan
// from what the ring's thread last saw; it never passes a batch not posted)
static uint64_t pmd_scan(const cop_pmd *m, uint32_t r)
{
    uint64_t c = m->ring[r].completed.load(std::memory_order_relaxed);
    const volatile uint64_t *d = m->h_done + (size_t)r * m->n_slots;
    while (d[c % m->n_slots] == c + 1) c++;
    return c;
}

static int pmd_launch(cop_pmd *m)
{
    cop_ctx *c = m->c;
    HIPCHK(c, hipSetDevice(c->device));
    // every device word restarts at zero: the gates, relays, exit and census
    // words, the slot tile counts and the look-back chains. An idle exit
    // leaves no batch half done (the gates: every batch a worker may have
    // started is finished before the workers leave, so each tile's counter
    // and per-rule adds happen exactly once); this launch serves each ring
    // from its first batch not completed.
    HIPCHK(c, hipMemsetAsync(m->dev, 0, m->dev_bytes, m->s));
    m->h_state[0] = 0;
    m->h_state[1] = 0;
    *m->h_stop = 0;
    for (uint32_t r = 0; r < m->n_rings; r++) m->P.seq0r[r] = pmd_scan(m, r);
    std::atomic_thread_fence(std::memory_order_seq_cst);
    hipError_t e = copk_pmd_launch(&m->P, m->fw_mode, m->lpm_mode, m->layout, m->ppt, m->ext, m->lds_bytes, m->s);
    if (e != hipSuccess) return set_err(c, -EIO, "pmd launch: %s", hipGetErrorString(e));
    m->launches++;
    m->live = true;
    return 0;
}

// wait until the launch has left the GPU (bounded: it leaves by itself on
// stop, idle or abort)
static int pmd_join(cop_pmd *m, double timeout_s)
{
    if (!m->live) return 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        hipError_t e = hipStreamQuery(m->s);
        if (e == hipSuccess) break;
        if (e != hipErrorNotReady) return set_err(m->c, -EIO, "pmd: %s", hipGetErrorString(e));
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
            return set_err(m->c, -ETIMEDOUT, "pmd: kernel did not leave within %.0f s", timeout_s);
        std::this_thread::sleep_for(std::chrono::microseconds(5));
    }
    m->live = false;
    return 0;
}

// advance ring r's completed count over its completion words. Any thread
// may call it (the ring's own, a counter reader, cop_pmd_completed_ring):
// the count only ever rises. A caller descheduled between its load and its
// store must not move it back below a count the ring's thread has since
// raised past a reposted slot: the scan from a lower count would stop at
// that slot (its word then holds the newer sequence) for good.
static uint64_t pmd_refresh(cop_pmd *m, uint32_t r)
{
    PmdRing &g = m->ring[r];
    const uint64_t posted = g.posted.load(std::memory_order_relaxed);
    const uint64_t c0 = g.completed.load(std::memory_order_relaxed);
    uint64_t c = c0;
    const volatile uint64_t *d = m->h_done + (size_t)r * m->n_slots;
    while (c < posted && d[c % m->n_slots] == c + 1) c++;
    uint64_t cur = c0;
    while (c > cur && !g.completed.compare_exchange_weak(cur, c, std::memory_order_relaxed)) {
    }
    return std::max(c, cur);
}

// count the binned rule hits of every completed batch not yet counted
// (cop_hit_count over runs of consecutive slots, on stream hs, beside the
// running kernel; one ring)
static int pmd_hits_launch(cop_pmd *m)
{
    if (!m->bins) return 0;
    const CopKParams &p = m->P.k;
    const uint64_t completed = m->ring[0].completed.load(std::memory_order_relaxed);
    while (m->counted < completed) {
        const uint32_t s0 = (uint32_t)(m->counted % m->n_slots);
        const uint32_t k = (uint32_t)std::min<uint64_t>(completed - m->counted, m->n_slots - s0);
        CopKParams q = p;
        q.hit_region = p.hit_region + (size_t)s0 * m->tpb * p.hit_reg_words;
        q.hit_off = p.hit_off + (size_t)s0 * m->tpb * (p.hit_nb + 1);
        hipError_t e = copk_hit_count(&q, k * m->tpb, COPK_BLOCK * (uint32_t)m->ppt, m->hs);
        if (e != hipSuccess) return set_err(m->c, -EIO, "pmd hit count: %s", hipGetErrorString(e));
        m->counted += k;
    }
    return 0;
}

// batches < upto counted and their count kernels done (their slots may be
// rewritten, their hits are in the rule counters)
static int pmd_hits_sync(cop_pmd *m, uint64_t upto)
{
    if (!m->bins || m->count_synced >= upto) return 0;
    if (int rc = pmd_hits_launch(m)) return rc;
    HIPCHK(m->c, hipStreamSynchronize(m->hs));
    m->count_synced = m->counted;
    return 0;
}

// count every completed batch's binned hits, with the GPU free (pmd_pause)
static int pmd_hits_flush(cop_ctx *c)
{
    cop_pmd *m = c->pmd;
    if (!m || !m->bins) return 0;
    if (m->count_synced >= pmd_refresh(m, 0) && m->ring[0].posted.load() == m->count_synced) return 0;
    if (int rc = pmd_pause(c)) return rc;
    int rc = pmd_hits_sync(m, pmd_refresh(m, 0));
    const int rrc = pmd_resume(c);
    return rc ? rc : rrc;
}

// every worker must be resident at once (static tile order): all of the
// GPU's workgroup slots for this kernel; other kernels on the device wait
// until the poll-mode kernel stops or leaves idle
static void pmd_size(cop_pmd *m)
{
    m->P.n_work = (uint32_t)m->c->ncu * m->per_cu;
    // 5 doorbell readers over PCIe: 20 (stride 64) took 17.7 us per one-batch
    // post against 16.1; 80 (stride 16) flood the link (56.8 us).
    // Stride 257, not 256: workgroups go round-robin over the XCDs and their
    // CUs, so every multiple of 256 lands on the same CU of XCD 0; 257 puts
    // the five readers on five XCDs (the driver's command +2 % / +6 % in two
    // A/B pairs on one box, noise on another; 16 batches in flight +15 %:
    // profiles/r03/lead*/). With several rings each ring's worker 0 reads
    // its ring's doorbell (one reader per ring).
    m->P.relay_stride = 257;
    if (const char *e = getenv("COP_PMD_RELAY_STRIDE")) m->P.relay_stride = std::max(1u, (uint32_t)atoi(e));
    m->P.poll_backoff = 3;
    m->P.stepwise = getenv("COP_PMD_STEPWISE") && !atoi(getenv("COP_PMD_STEPWISE")) ? 0u : 1u;
    m->P.dyn = m->dyn ? 1u : m->pf ? 2u : 0u;
    // ticket lanes of dynamic tiles: 8 unless $COP_PMD_TK_LANES says 1
    m->P.tk_lanes = COPK_PMD_TK_LANES;
    if (const char *e = getenv("COP_PMD_TK_LANES")) m->P.tk_lanes = atoi(e) == 1 ? 1u : (uint32_t)COPK_PMD_TK_LANES;
    if (const char *e = getenv("COP_PMD_BACKOFF")) m->P.poll_backoff = std::min(64u, (uint32_t)atoi(e));
    // Slot reuse (switch.c:463-470: the fast path refills the rings
    // forever): a ring slot may be rewritten by another agent between its
    // batches, and a persistent kernel gets no dispatch-time invalidation, so
    // by default a tile reads its slot with system-coherent loads once its
    // ring has wrapped in this launch (mode 4; a slot's first read in a
    // launch is fresh). Rings whose packets live in host memory (mapped
    // pinned: the drop-in's header records) do so on every tile (mode 3,
    // also COP_PMD_SYS_ACQUIRE); COP_PMD_STATIC_SLOTS declares the slots
    // written once before the start (mode 0: plain loads).
    m->P.sys_acquire = m->acquire;
    if (m->acquire == 4u) {
        for (uint32_t q = 0; q < m->n_rings; q++) {
            hipPointerAttribute_t at;
            if (hipPointerGetAttributes(&at, m->P.rings[q].pkts) == hipSuccess && at.type == hipMemoryTypeHost)
                m->P.sys_acquire = 3;
        }
        (void)hipGetLastError();   // (an unregistered pointer leaves an error behind)
        // Mode 4 trusts a slot's first read in a launch, which holds only if
        // no read of another slot brought one of its cache lines in earlier:
        // slots (and IMIX offset arrays) must start on 128-byte L2 lines. A
        // ring whose slots share lines (e.g. 4097 packets 64 bytes apart per
        // slot) takes coherent loads on every tile (mode 3).
        for (uint32_t q = 0; q < m->n_rings && m->P.sys_acquire == 4u; q++) {
            const CopKRing &r = m->P.rings[q];
            bool lined = (uintptr_t)r.pkts % 128u == 0 && r.pkts_slot_bytes % 128u == 0;
            if (r.offsets) lined = lined && (uintptr_t)r.offsets % 128u == 0 && (r.offsets_slot_words * 4u) % 128u == 0;
            if (!lined) m->P.sys_acquire = 3;
        }
    }
    if (const char *e = getenv("COP_PMD_ACQUIRE")) m->P.sys_acquire = std::min(4u, (uint32_t)atoi(e));   // A/B runs
    // tests: a tile that never runs, so its successors' look-back gives up
    m->P.test_skip = getenv("COP_PMD_TEST_SKIP_TILE") ? (uint32_t)atoi(getenv("COP_PMD_TEST_SKIP_TILE")) + 1u : 0u;
}

// wait for the launch's census: 0 = every worker resident, 1 = aborted
// (some could not be), or -errno
static int pmd_census(cop_pmd *m)
{
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        if (m->h_state[1] == m->P.n_work) return 0;
        if (m->h_state[0] == COPK_PMD_ABORT) return 1;
        if (m->h_state[0] != COPK_PMD_RUNNING) return set_err(m->c, -EIO, "pmd: left during the census");
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > 5.0)
            return set_err(m->c, -ETIMEDOUT, "pmd: no census after 5 s");
        std::this_thread::sleep_for(std::chrono::microseconds(5));
    }
}

// Dispatch every side kernel that may have to run beside the persistent
// kernel once on its own stream, before the persistent kernel holds the CUs:
// the binned hit count (stream hs) and the counter snapshot (telemetry and
// context streams). Their code objects are then loaded and their queues set
// up while the GPU is free. ($COP_PMD_PREWARM=0: off, experiments)
static int pmd_prewarm(cop_pmd *m)
{
    cop_ctx *c = m->c;
    const char *env = getenv("COP_PMD_PREWARM");
    if (env && !atoi(env)) return 0;
    HIPCHK(c, hipSetDevice(c->device));
    if (m->bins) {
        hipError_t e = copk_hit_count(&m->P.k, 0, COPK_BLOCK * (uint32_t)m->ppt, m->hs);
        if (e != hipSuccess) return set_err(c, -EIO, "pmd prewarm: %s", hipGetErrorString(e));
        HIPCHK(c, hipStreamSynchronize(m->hs));
    }
    if (int rc = tele_scratch(c)) return rc;
    for (hipStream_t s : {c->tele_stream, c->stream}) {
        hipError_t e = copk_snapshot(c->counters, 1, c->tele_dev, 0, s);
        if (e != hipSuccess) return set_err(c, -EIO, "pmd prewarm: %s", hipGetErrorString(e));
        HIPCHK(c, hipStreamSynchronize(s));
    }
    return 0;
}

// Launch with every worker resident: when the census finds workers that
// could not become resident (another kernel, context or process holds CUs,
// likely after an idle exit), retry with one worker fewer per CU.
static int pmd_launch_resident(cop_pmd *m)
{
    for (;;) {
        if (int rc = pmd_launch(m)) return rc;
        const int st = pmd_census(m);
        if (st == 0) return 0;
        if (st < 0) return st;
        if (int rc = pmd_join(m, 10.0)) return rc;
        if (m->per_cu <= 1 || m->c->ncu * (m->per_cu - 1) < m->n_rings)
            return set_err(m->c, -EIO, "pmd: workers never co-resident");
        m->per_cu--;
        pmd_size(m);
    }
}

// the kernel left: relaunch after an idle exit (every batch it completed
// stays complete; the rest, posted before or after the exit, are served by
// the new launch from each ring's first incomplete one), else fail. Any
// ring's thread may call it; one relaunches, the others find it running.
static int pmd_revive(cop_pmd *m)
{
    if (m->h_state[0] == COPK_PMD_RUNNING) return 0;
    std::lock_guard<std::mutex> lk(m->mu);
    const uint32_t why = m->h_state[0];
    if (why == COPK_PMD_RUNNING) return 0;   // another ring's thread relaunched it
    if (why != COPK_PMD_IDLE && why != COPK_PMD_PAUSED)
        return set_err(m->c, -EIO, "pmd kernel left (%s)", why == COPK_PMD_ABORT ?
                       "abort: workers not co-resident, or a look-back timed out" : "stopped");
    if (int rc = pmd_join(m, 10.0)) return rc;
    return pmd_launch_resident(m);
}

// Make the GPU free for kernels the host must see finish while a poll-mode
// kernel serves the context: the binned hit count and the RCCL all-reduce
// of the counters. The poll-mode kernel holds every workgroup slot it may
// use, and a kernel of another stream beside it is not guaranteed to run
// (round 3's config-5 record: cop_hit_count waited 1 s for the idle exit;
// DESIGN.md §14.1). So the host asks it to leave (h_stop = 2: it closes its
// gates and finishes every batch below them, as an idle exit does), waits
// until it has left, runs the side work, and relaunches it (pmd_resume).
// Holds the relaunch lock in between: a ring's post or wait meanwhile
// blocks in pmd_revive until the relaunch.
static int pmd_pause(cop_ctx *c)
{
    cop_pmd *m = c->pmd;
    if (!m) return 0;
    m->mu.lock();
    m->was_live = m->live && m->h_state[0] == COPK_PMD_RUNNING;
    if (m->was_live) {
        *m->h_stop = 2u;
        std::atomic_thread_fence(std::memory_order_seq_cst);
    }
    const int rc = pmd_join(m, 10.0);
    if (rc) m->mu.unlock();
    else m->pauses += m->was_live ? 1u : 0u;
    return rc;
}

// relaunch after pmd_pause (only if it was running then: a kernel that had
// left idle is relaunched by the next post, as always)
static int pmd_resume(cop_ctx *c)
{
    cop_pmd *m = c->pmd;
    if (!m) return 0;
    int rc = 0;
    if (m->was_live && !m->live && m->h_state[0] == COPK_PMD_PAUSED) rc = pmd_launch_resident(m);
    m->mu.unlock();
    return rc;
}

// ring geometry every ring of one kernel shares (the kernel is instantiated
// once: one layout, tile size and slot count)
static bool pmd_same_geometry(const cop_batch_ring *a, const cop_batch_ring *b)
{
    return a->n_slots == b->n_slots && a->n == b->n && a->stride == b->stride && a->data_off == b->data_off &&
           (a->offsets != nullptr) == (b->offsets != nullptr) && (a->fwd_idx != nullptr) == (b->fwd_idx != nullptr) &&
           (a->fwd_count != nullptr) == (b->fwd_count != nullptr) && a->results_slot == b->results_slot &&
           a->fwd_slot == b->fwd_slot;
}

int cop_pmd_start(cop_ctx *c, const cop_batch_ring *r, cop_pmd **out)
{
    return cop_pmd_start_rings(c, r, 1, 0u, out);
}

int cop_pmd_start_rings(cop_ctx *c, const cop_batch_ring *rings, uint32_t n_rings, uint32_t flags, cop_pmd **out)
{
    return cop_pmd_start_rings_stages(c, rings, n_rings, flags, c ? c->cfg.stages : 0u, out);
}

int cop_pmd_start_rings_stages(cop_ctx *c, const cop_batch_ring *rings, uint32_t n_rings, uint32_t flags,
                               uint32_t stages, cop_pmd **out)
{
    if (!c || !rings || !out || n_rings < 1) return -EINVAL;
    *out = nullptr;
    if (n_rings > COPK_PMD_MAX_RINGS) return set_err(c, -EINVAL, "pmd: %u rings > %d", n_rings, COPK_PMD_MAX_RINGS);
    if (flags & ~(COP_PMD_VARIABLE_N | COP_PMD_SYS_ACQUIRE | COP_PMD_STATIC_SLOTS | COP_PMD_DYNAMIC_TILES))
        return set_err(c, -EINVAL, "pmd: unknown flags %#x", flags);
    if ((flags & COP_PMD_SYS_ACQUIRE) && (flags & COP_PMD_STATIC_SLOTS))
        return set_err(c, -EINVAL, "pmd: COP_PMD_SYS_ACQUIRE and COP_PMD_STATIC_SLOTS contradict");
    if (c->pmd) return set_err(c, -EBUSY, "this context already has a poll-mode kernel");
    const cop_batch_ring *r = &rings[0];
    for (uint32_t q = 0; q < n_rings; q++) {
        const cop_batch_ring *x = &rings[q];
        if (x->n_slots == 0 || x->n == 0 || !x->pkts || !x->results) return set_err(c, -EINVAL, "pmd: empty ring");
        if (q && !pmd_same_geometry(r, x))
            return set_err(c, -EINVAL, "pmd: ring %u's geometry differs from ring 0's (n, slots, stride, layout)", q);
    }
    if (r->n > c->cfg.max_batch) return set_err(c, -EINVAL, "pmd: n %u > max_batch", r->n);
    const bool imix = r->offsets != nullptr;
    const bool compact = (r->fwd_idx || r->fwd_count) && !(c->cfg.flags & COP_CFG_NO_COMPACT);
    const uint32_t lists = (compact && (c->cfg.flags & COP_CFG_DEMUX_PORTS)) ? c->cfg.n_ports : 1u;
    const bool seg = compact && (c->cfg.flags & COP_CFG_SEG_LISTS);
    bool wide = true;   // every slot's records 16-byte aligned (lane-pair record stores)
    for (uint32_t q = 0; q < n_rings; q++) {
        const cop_batch_ring *x = &rings[q];
        if (((uintptr_t)x->pkts & 15) || (x->pkts_slot_bytes & 15) || (x->data_off & 15) ||
            (!imix && ((x->stride & 15) || (x->stride < 36 && x->stride != COP_HDR16_STRIDE))))
            return set_err(c, -EINVAL, "pmd: packet starts must be 16-byte aligned");
        if (x->results_slot < x->n || (x->fwd_idx && x->fwd_slot < (uint64_t)x->n * lists))
            return set_err(c, -EINVAL, "pmd: slot sizes smaller than n (x ports with demux)");
        if (int rc = check_seg_ring(c, x, seg)) return rc;
        // the coherent slot loads (every mode but COP_PMD_STATIC_SLOTS) take
        // 31-bit byte offsets from the slot's base (a buffer resource,
        // cop_device.h sys_rsrc): a slot's packets must lie within its first
        // 2 GiB, where an IMIX offset can reach anywhere in the slot
        const uint64_t span = imix ? x->pkts_slot_bytes + x->data_off + 64u
                                   : (uint64_t)x->n * x->stride + x->data_off + 64u;
        if (!(flags & COP_PMD_STATIC_SLOTS) && span > 0x7FFFFFFFull)
            return set_err(c, -EINVAL,
                           "pmd: slots span %llu bytes; coherent slot loads reach 2 GiB (COP_PMD_STATIC_SLOTS for "
                           "slots written once)",
                           (unsigned long long)span);
        wide = wide && ((uintptr_t)x->results & 15) == 0 && (x->results_slot & 1) == 0;
    }
    if (int rc = sync_lanes(c)) return rc;

    cop_pmd *m = new (std::nothrow) cop_pmd();
    if (!m) return -ENOMEM;
    m->c = c;
    m->n_rings = n_rings;
    m->ring_n = r->n;
    m->acquire = (flags & COP_PMD_SYS_ACQUIRE) ? 3u : (flags & COP_PMD_STATIC_SLOTS) ? 0u : 4u;
    Plan pl = plan_launch(c, (uint64_t)r->n * r->n_slots, imix, r->stride);
    // tile size: 1024-packet tiles (five workers per CU, so a 20-batch burst
    // of 64k packets is one tile per worker), 256-packet tiles for small
    // batches
    int ppt = r->n >= 4u * COPK_BLOCK * 4 ? 4 : 1;
    // dynamic tiles (COP_PMD_DYNAMIC_TILES; segmented lists, step-by-step
    // tiles): the next tile's first two steps' loads in flight during the
    // current one (COPK_PMD_WIN 2). A/B runs: $COP_PMD_DYN=1 256-packet
    // dynamic tiles, 4 the flag's 1024-packet tiles, 0 off
    const char *dyn_env = getenv("COP_PMD_DYN");
    m->dyn = seg && (dyn_env ? atoi(dyn_env) != 0 : (flags & COP_PMD_DYNAMIC_TILES) != 0);
    if (m->dyn && dyn_env && atoi(dyn_env) == 1) ppt = 1;
    // A/B runs: $COP_PMD_PF=1 the static order with the next tile's first
    // step prefetched during the current one (segmented lists)
    m->pf = seg && !m->dyn && getenv("COP_PMD_PF") && atoi(getenv("COP_PMD_PF")) != 0;
    if (c->ppt_override) ppt = c->ppt_override;
    pl.ppt = ppt;
    m->ppt = ppt;
    m->layout = pl.layout;
    m->tpb = (r->n + COPK_BLOCK * ppt - 1) / (COPK_BLOCK * ppt);
    m->n_slots = r->n_slots;
    CopKParams &p = m->P.k;
    memset(&p, 0, sizeof(p));
    p.ring = 1;
    for (uint32_t q = 0; q < n_rings; q++) {
        const cop_batch_ring *x = &rings[q];
        CopKRing &g = m->P.rings[q];
        g.pkts = (const uint8_t *)x->pkts;
        g.offsets = x->offsets;
        g.results = x->results;
        g.fwd_idx = compact ? x->fwd_idx : nullptr;
        g.fwd_count = compact ? x->fwd_count : nullptr;
        g.pkts_slot_bytes = x->pkts_slot_bytes;
        g.offsets_slot_words = x->offsets_slot_words;
        g.results_slot = x->results_slot;
        g.fwd_slot = x->fwd_slot;
        g.n_slots = x->n_slots;
        g.first = 0;
        g.n = x->n;
        g.stride = x->stride;
        g.data_off = x->data_off;
    }
    p.rg = m->P.rings[0];
    m->P.n_rings = n_rings;
    p.nb = 1;
    p.ntiles = m->tpb;
    p.uniform_ntiles = m->tpb;
    p.compact = compact ? 1u : 0u;
    p.seg = seg ? 1u : 0u;
    p.stages = stages;
    p.demux = (compact && (c->cfg.flags & COP_CFG_DEMUX_PORTS)) ? c->cfg.n_ports : 0u;
    int rc = 0;
#define PMD_FAIL(code)       \
    do {                     \
        rc = (code);         \
        goto fail;           \
    } while (0)
    {
        // records as 16-byte write-through stores: every slot's records
        // 16-byte aligned
        // ($COP_PMD_REC: paired = from lane pairs in registers, the default;
        // stage = through an LDS stage after the compaction; 8 = 8-byte stores)
        const char *rec_env = getenv("COP_PMD_REC");
        wide = wide && !(rec_env && !strcmp(rec_env, "8"));
        const bool stage_rec = wide && rec_env && !strcmp(rec_env, "stage");
        if ((rc = fill_launch(c, p, ppt, &m->fw_mode, &m->lpm_mode, &m->lds_bytes, stage_rec))) goto fail;
        p.rec_paired = wide && !stage_rec ? 1u : 0u;
        p.dbg = 0;   // no ablations in the persistent kernel
        p.stamps = nullptr;
        const char *stamps_env = getenv("COP_PMD_STAMPS");
        if (stamps_env && atoi(stamps_env) >= 2) {   // diagnostic: the tile body's phase stamps too
            if (hipMalloc(&p.stamps, (size_t)c->ncu * 8 * 8 * 8) != hipSuccess)
                PMD_FAIL(set_err(c, -ENOMEM, "pmd: stamps"));
            // 2: through the EXT kernel (dbg bit 8); 3: the production kernel
            // of a -DCOPK_PHASE_STAMPS=1 experiment build
            if (atoi(stamps_env) == 2) p.dbg = 8;
        }
        // per-rule hits by binning, as in the one-shot kernel: one region per
        // (slot, tile), counted by cop_hit_count beside the running kernel
        // (one ring; with several, one atomic per hit)
        if (p.rule_hits && c->hit_bins && n_rings == 1) {
            const uint32_t nb = (c->n_rule_ctr + (1u << COPK_HIT_SHIFT) - 1) >> COPK_HIT_SHIFT;
            const uint32_t reg = COPK_BLOCK * (uint32_t)ppt + 4u * nb;
            const uint32_t base = (m->lds_bytes / 4u + 3u) & ~3u;
            const uint32_t words = ((3u * nb + 5u + 3u) & ~3u) + COPK_BLOCK * (uint32_t)ppt + reg;
            if (nb >= 1 && nb <= COPK_HIT_MAX_BUCKETS && (base + words) * 4u <= 160u * 1024u) {
                const size_t tiles = (size_t)m->n_slots * m->tpb;
                if (hipMalloc(&p.hit_region, tiles * reg * 4) != hipSuccess ||
                    hipMalloc(&p.hit_off, tiles * (nb + 1) * 4) != hipSuccess)
                    PMD_FAIL(set_err(c, -ENOMEM, "pmd: hit regions"));
                if (hipStreamCreateWithFlags(&m->hs, hipStreamNonBlocking) != hipSuccess)
                    PMD_FAIL(set_err(c, -EIO, "pmd: hit stream"));
                p.hit_nb = nb;
                p.hit_reg_words = reg;
                p.lds_hit_off = base;
                m->lds_bytes = (base + words) * 4u;
                m->bins = true;
            }
        }
        m->ext = (p.demux || p.port_stats || p.rule_hits || p.dbg) ? 1 : 0;
        int occ = 0;
        hipError_t e = copk_pmd_occupancy(m->fw_mode, m->lpm_mode, m->layout, ppt, m->ext, m->lds_bytes, &occ);
        if (e != hipSuccess || occ < 1) PMD_FAIL(set_err(c, -EIO, "pmd occupancy: %s (%d)", hipGetErrorString(e), occ));
        // the hardware admits at most 800 / (roundup16(sgprs) + 16) 256-thread
        // workgroups per CU (MI355X_MICROARCH.md, Residency): 6 at the
        // pipeline kernels' ~106 SGPRs, below what the API may answer; the
        // start-up census confirms, else one fewer per CU is tried
        occ = std::min(occ, 6);
        if (p.dbg) occ = std::min(occ, 4);   // the EXT diagnostic kernel holds more registers
        // binned hits: leave room beside the workers for the count kernel
        // (64 KiB of LDS and a workgroup per CU)
        if (m->bins) occ = std::min(occ, 4);
        // dynamic tiles: leave a workgroup slot per CU free (at six workers
        // per CU a pageable cop_memcpy_h2d beside the kernel waited for its
        // idle exit: profiles/r05/check1/pytest_dyn.log, relaunches per post)
        if (m->dyn) occ = std::min(occ, 5);
        if (const char *env = getenv("COP_PMD_PER_CU")) occ = std::min(occ, std::max(1, atoi(env)));
        m->per_cu = (uint32_t)occ;
        pmd_size(m);
        m->P.idle_ticks = 100000000ull;   // 1 s at 100 MHz
        if (const char *env = getenv("COP_PMD_IDLE_MS")) {
            // ms -> ticks in 64 bits, clamped to a day
            const unsigned long long ms = std::min<unsigned long long>(strtoull(env, nullptr, 0), 86400000ull);
            m->P.idle_ticks = std::max<unsigned long long>(ms, 1ull) * 100000ull;
        }
        // control block in mapped host memory: posted words, stop, state,
        // then the completion words (and the batch sizes) of every ring slot
        const size_t words = (size_t)n_rings * m->n_slots;
        const bool var_n = (flags & COP_PMD_VARIABLE_N) != 0;
        const size_t ctl_bytes = PMD_H_DONE + words * 8 + (var_n ? words * 4 : 0);
        HIPCHK(c, hipSetDevice(c->device));
        if (hipHostMalloc(&m->ctl, ctl_bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
            PMD_FAIL(set_err(c, -ENOMEM, "pmd: host control block"));
        memset(m->ctl, 0, ctl_bytes);
        void *dctl = nullptr;
        if (hipHostGetDevicePointer(&dctl, m->ctl, 0) != hipSuccess) PMD_FAIL(set_err(c, -EIO, "pmd: mapping"));
        m->h_stop = (volatile uint32_t *)(m->ctl + PMD_H_STOP);
        m->h_state = (volatile uint32_t *)(m->ctl + PMD_H_STATE);
        m->h_done = (volatile uint64_t *)(m->ctl + PMD_H_DONE);
        m->P.h_posted = (const unsigned long long *)dctl;
        m->P.h_stop = (const uint32_t *)((uint8_t *)dctl + PMD_H_STOP);
        m->P.h_state = (uint32_t *)((uint8_t *)dctl + PMD_H_STATE);
        m->P.h_done = (unsigned long long *)((uint8_t *)dctl + PMD_H_DONE);
        if (var_n) {
            m->h_n = (volatile uint32_t *)(m->ctl + PMD_H_DONE + words * 8);
            m->P.h_n = (const uint32_t *)((uint8_t *)dctl + PMD_H_DONE + words * 8);
        }
        // device words: control, gates and relays, slot tile counts, then the
        // look-back chains (dense lists only)
        // one slot counter per 4160 bytes: 64 returning adds per batch on
        // counters packed 16 to a line held a 20-batch burst up ~3 us
        // (tools/burst modes 15/16, profiles/r03/burst/burst7)
        m->P.slot_stride = 520;
        if (const char *e = getenv("COP_PMD_SLOT_STRIDE")) m->P.slot_stride = std::max(1u, (uint32_t)atoi(e));
        const size_t look_off = (PMD_CTL_BYTES + words * m->P.slot_stride * 8 + 255) & ~(size_t)255;
        const size_t look_words = (compact && !seg) ? words * m->tpb * (p.demux ? p.demux : 1u) : 0;
        m->dev_bytes = look_off + look_words * 8;
        if (getenv("COP_PMD_STAMPS")) {   // diagnostic phase stamps (cop_debug_pmd_stamps)
            if (hipMalloc(&m->P.stamps, ((size_t)m->P.n_work * 8 + 128) * 8) != hipSuccess)
                PMD_FAIL(set_err(c, -ENOMEM, "pmd: stamps"));
            (void)hipMemset(m->P.stamps, 0, ((size_t)m->P.n_work * 8 + 128) * 8);
            (void)hipDeviceSynchronize();
        }
        if (hipMalloc(&m->dev, m->dev_bytes) != hipSuccess) PMD_FAIL(set_err(c, -ENOMEM, "pmd: device words"));
        if (hipStreamCreateWithFlags(&m->s, hipStreamNonBlocking) != hipSuccess)
            PMD_FAIL(set_err(c, -EIO, "pmd: stream"));
        m->P.d_ctl = (uint32_t *)(m->dev + 8);
        m->P.d_act = (unsigned long long *)(m->dev + PMD_ACT_OFF);
        m->P.d_gate = (unsigned long long *)(m->dev + PMD_GATE_OFF);
        m->P.d_posted = (unsigned long long *)(m->dev + PMD_RELAY_OFF);
        m->P.d_ticket = (unsigned long long *)(m->dev + PMD_TICKET_OFF);
        m->P.slot_tiles = (unsigned long long *)(m->dev + PMD_CTL_BYTES);
        p.look = look_words ? (unsigned long long *)(m->dev + look_off) : nullptr;
        p.err = nullptr;   // the look-back reports through d_ctl[2] (LookCtx)
        p.epoch = 0;
        if ((rc = pmd_prewarm(m))) goto fail;
        if ((rc = pmd_launch_resident(m))) {
            (void)pmd_join(m, 10.0);
            goto fail;
        }
    }
#undef PMD_FAIL
    c->pmd = m;
    *out = m;
    return 0;
fail:
    if (m->P.stamps) (void)hipFree(m->P.stamps);
    if (m->P.k.stamps) (void)hipFree(m->P.k.stamps);
    if (m->P.k.hit_region) (void)hipFree(m->P.k.hit_region);
    if (m->P.k.hit_off) (void)hipFree(m->P.k.hit_off);
    if (m->hs) (void)hipStreamDestroy(m->hs);
    if (m->s) (void)hipStreamDestroy(m->s);
    if (m->dev) (void)hipFree(m->dev);
    if (m->ctl) (void)hipHostFree(m->ctl);
    delete m;
    return rc;
}

int cop_pmd_wait_ring(cop_pmd *m, uint32_t ring, uint64_t seq)
{
    if (!m || ring >= m->n_rings) return -EINVAL;
    PmdRing &g = m->ring[ring];
    const uint64_t posted = g.posted.load(std::memory_order_relaxed);
    if (seq > posted)
        return set_err(m->c, -EINVAL, "pmd: ring %u: wait for %llu > %llu posted", ring, (unsigned long long)seq,
                       (unsigned long long)posted);
    const auto t0 = std::chrono::steady_clock::now();
    uint32_t spins = 0;
    for (;;) {
        if (pmd_refresh(m, ring) >= seq) break;
        if (m->h_state[0] != COPK_PMD_RUNNING) {
            if (pmd_refresh(m, ring) >= seq) break;   // its last completion may have landed just before it left
            if (int rc = pmd_revive(m)) return rc;
        }
        if ((++spins & 1023u) == 0 &&
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > 30.0)
            return set_err(m->c, -ETIMEDOUT, "pmd: ring %u: batch %llu not complete after 30 s", ring,
                           (unsigned long long)g.completed.load());
    }
    std::atomic_thread_fence(std::memory_order_seq_cst);
    return 0;
}

int cop_pmd_wait(cop_pmd *m, uint64_t seq) { return cop_pmd_wait_ring(m, 0, seq); }

// Post `count` batches to ring r; n_each: their packets (variable-n rings),
// 0 = the ring's n
static int pmd_post(cop_pmd *m, uint32_t r, uint32_t count, uint32_t n_each)
{
    if (count == 0) return 0;
    if (count > m->n_slots) return set_err(m->c, -EINVAL, "pmd: post of %u > %u ring slots", count, m->n_slots);
    PmdRing &g = m->ring[r];
    const uint64_t posted = g.posted.load(std::memory_order_relaxed);
    // a slot is reposted only after its previous batch completed
    const uint64_t need = posted + count;
    if (need - g.completed.load(std::memory_order_relaxed) > m->n_slots)
        if (int rc = cop_pmd_wait_ring(m, r, need - m->n_slots)) return rc;
    if (r == 0 && m->bins && need > m->n_slots && m->count_synced < need - m->n_slots) {
        // the reused slots' binned hits are counted first, with the GPU free
        if (int rc = pmd_pause(m->c)) return rc;
        int rc = pmd_hits_sync(m, need - m->n_slots);
        const int rrc = pmd_resume(m->c);
        if (rc || rrc) return rc ? rc : rrc;
    }
    if (int rc = pmd_revive(m)) return rc;
    if (m->h_n)
        for (uint64_t b = posted; b < need; b++)
            m->h_n[(size_t)r * m->n_slots + b % m->n_slots] = n_each ? n_each : m->ring_n;
    std::atomic_thread_fence(std::memory_order_seq_cst);   // ring slots (and sizes) written before the doorbell
    *m->h_posted(r) = need;
    g.posted.store(need, std::memory_order_relaxed);
    return 0;
}

int cop_pmd_post_ring(cop_pmd *m, uint32_t ring, uint32_t count)
{
    if (!m || ring >= m->n_rings) return -EINVAL;
    return pmd_post(m, ring, count, 0);
}

int cop_pmd_post(cop_pmd *m, uint32_t count) { return cop_pmd_post_ring(m, 0, count); }

int cop_pmd_post_batch(cop_pmd *m, uint32_t ring, uint32_t n)
{
    if (!m || ring >= m->n_rings) return -EINVAL;
    if (!m->h_n) return set_err(m->c, -EINVAL, "pmd: started without COP_PMD_VARIABLE_N");
    if (n == 0 || n > m->ring_n) return set_err(m->c, -EINVAL, "pmd: batch of %u packets (1..%u)", n, m->ring_n);
    return pmd_post(m, ring, 1, n);
}

uint64_t cop_pmd_posted(const cop_pmd *m) { return m ? m->ring[0].posted.load() : 0; }

uint64_t cop_pmd_posted_ring(const cop_pmd *m, uint32_t ring)
{
    return m && ring < m->n_rings ? m->ring[ring].posted.load() : 0;
}

uint64_t cop_pmd_completed_ring(cop_pmd *m, uint32_t ring)
{
    return m && ring < m->n_rings ? pmd_refresh(m, ring) : 0;
}

int cop_pmd_run(cop_pmd *m, uint64_t count)
{
    if (!m) return -EINVAL;
    const uint32_t chunk = std::max(1u, m->n_slots / 4);   // a quarter ring per post: the ring never drains
    for (uint64_t done = 0; done < count;) {
        const uint32_t k = (uint32_t)std::min<uint64_t>(chunk, count - done);
        if (int rc = cop_pmd_post(m, k)) return rc;
        done += k;
    }
    return cop_pmd_wait(m, m->ring[0].posted.load());
}

static uint64_t mono_ns()
{
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

int cop_pmd_run_timed(cop_pmd *m, uint64_t count, uint64_t *t_post_ns, uint64_t *t_done_ns)
{
    if (!m) return -EINVAL;
    const uint64_t t0 = mono_ns();
    const int rc = cop_pmd_run(m, count);
    const uint64_t t1 = mono_ns();
    if (t_post_ns) *t_post_ns = t0;
    if (t_done_ns) *t_done_ns = t1;
    return rc;
}

int cop_pmd_info(const cop_pmd *m, cop_pmd_info_t *out)
{
    if (!m || !out) return -EINVAL;
    out->workers = m->P.n_work;
    out->workers_per_cu = m->per_cu;
    out->tiles_per_batch = m->tpb;
    out->packets_per_tile = COPK_BLOCK * (uint32_t)m->ppt;
    out->launches = m->launches.load();
    out->state = m->h_state[0];
    out->slot_loads = m->P.sys_acquire;
    out->kernel = (uint32_t)m->fw_mode | (uint32_t)m->lpm_mode << 4 | (uint32_t)m->layout << 8 |
                  (uint32_t)(m->ext ? 1 : 0) << 12;
    out->posted = out->completed = 0;
    for (uint32_t r = 0; r < m->n_rings; r++) {   // every ring's batches
        out->posted += m->ring[r].posted.load();
        out->completed += m->ring[r].completed.load();
    }
    return 0;
}

int cop_pmd_stop(cop_pmd *m)
{
    if (!m) return -EINVAL;
    cop_ctx *c = m->c;
    int rc = 0;
    for (uint32_t r = 0; r < m->n_rings && !rc; r++) rc = cop_pmd_wait_ring(m, r, m->ring[r].posted.load());
    *m->h_stop = 1;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    const int jrc = pmd_join(m, 10.0);
    if (!rc) rc = jrc;
    if (!rc) rc = pmd_hits_sync(m, m->ring[0].completed.load());   // the GPU is free now
    if (m->hs) (void)hipStreamSynchronize(m->hs);
    if (!jrc) {
        if (m->s) (void)hipStreamDestroy(m->s);
        if (m->hs) (void)hipStreamDestroy(m->hs);
        if (m->dev) (void)hipFree(m->dev);
        if (m->ctl) (void)hipHostFree(m->ctl);
        if (m->P.stamps) (void)hipFree(m->P.stamps);
        if (m->P.k.stamps) (void)hipFree(m->P.k.stamps);
        if (m->P.k.hit_region) (void)hipFree(m->P.k.hit_region);
        if (m->P.k.hit_off) (void)hipFree(m->P.k.hit_off);
    }   // else: the kernel may still touch them; leak rather than free under it
    if (c->pmd == m) c->pmd = nullptr;
    delete m;
    return rc;
}

/* diagnostic (not in the public header): the poll-mode kernel's phase
 * stamps ($COP_PMD_STAMPS): per worker 8 u64 {tile start, batch seen,
 * body done, counted, batch, last-of-batch, -, -}, then 64 doorbell relays
 * {posted, time}; s_memrealtime ticks (100 MHz). Returns words copied. */
int cop_debug_pmd_stamps(cop_pmd *m, uint64_t *out, uint32_t max_words)
{
    if (!m || !m->P.stamps || !out) return -EINVAL;
    const uint32_t n = std::min<uint32_t>(max_words, m->P.n_work * 8 + 128);
    HIPCHK(m->c, hipMemcpy(out, m->P.stamps, (size_t)n * 8, hipMemcpyDeviceToHost));
    // then the tile body's stamps (cop_tile.h STAMP: 2 pass 1, 3 pass 2, 5 compaction, 6 counters)
    const uint32_t n2 = std::min<uint32_t>(max_words - n, m->P.n_work * 8);
    if (n2 && m->P.k.stamps) HIPCHK(m->c, hipMemcpy(out + n, m->P.k.stamps, (size_t)n2 * 8, hipMemcpyDeviceToHost));
    return (int)(n + (m->P.k.stamps ? n2 : 0));
}

/* test hook (not in the public header): make the next `count` launches
 * (what = 1) or host batch waits (what = 2) fail as a HIP error would, so
 * the drop-in loops' error paths can be exercised */
int cop_debug_inject(cop_ctx *c, int what, uint32_t count)
{
    if (!c || (what != 1 && what != 2)) return -EINVAL;
    if (what == 1) c->inject_submit = count;
    else c->inject_wait = count;
    return 0;
}

/* diagnostic (not in the public header): copy the phase stamps of the last
 * launch made with $COP_DBG bit 8; returns the number of u64 copied */
int cop_debug_stamps(cop_ctx *c, uint64_t *out, uint32_t max_words)
{
    if (!c || !c->stamps) return -EINVAL;
    uint32_t n = max_words < COPK_STAMP_WG * 8 ? max_words : COPK_STAMP_WG * 8;
    if (int rc = sync_lanes(c)) return rc;
    HIPCHK(c, hipMemcpy(out, c->stamps, (size_t)n * 8, hipMemcpyDeviceToHost));
    return (int)n;
}

int cop_debug_host_prof(cop_ctx *c, uint64_t *out, uint32_t n, int reset)
{
    if (!c || !out) return -EINVAL;
    for (uint32_t i = 0; i < n && i < 6; i++) out[i] = c->hp[i];
    if (reset) memset(c->hp, 0, sizeof(c->hp));
    return 6;
}

int cop_launch_timing(cop_ctx *c, int enable)
{
    if (!c) return -EINVAL;
    c->timing = enable != 0;
    return 0;
}

int cop_launch_timing_read(cop_ctx *c, double *mean_ms, uint64_t *n, int reset)
{
    if (!c) return -EINVAL;
    for (int l = 0; l < c->n_lanes; l++)
        while (c->lane[l].ev_count) harvest_one(c, c->lane[l]);
    if (mean_ms) *mean_ms = c->ev_n ? c->ev_sum_ms / (double)c->ev_n : 0.0;
    if (n) *n = c->ev_n;
    if (reset) {
        c->ev_sum_ms = 0;
        c->ev_n = 0;
    }
    return 0;
}

}  // extern "C"
