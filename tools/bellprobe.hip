// bellprobe.hip — doorbell latency probe (experiment tool, not the product).
// Can the host write a poll-mode kernel's doorbell straight into device
// memory, and how soon do polling workers see it? A ping-pong: the host
// writes sequence i into the bell word(s); workgroup 0 of the grid, on
// seeing it, writes i into a host-mapped ack word; the host times bell
// write -> ack seen. Modes:
//   host: bell in mapped pinned host memory, read over PCIe by the pollers
//         (one poller: the round-5 leader's read; many: every workgroup)
//   dev:  bell in fine-grained / uncached device memory written by the CPU
//         through the BAR, replicated over 8 lines, polled with
//         system-scope loads
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/_bellprobe tools/bellprobe.hip
#include <hip/hip_runtime.h>
#include <setjmp.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

// every workgroup's lane 0 waits for sequence i and stamps when it saw it;
// workgroup 0 acks i into host memory (write -> ack: workgroup 0's
// detection plus one PCIe store; the stamps give every other poller's lag
// behind workgroup 0). relay 0: each polls its replica line (bell + 16 *
// (wg % reps)) at system scope; relay 1: workgroup 0 polls the bell and
// raises 8 device relay lines (agent-scope atomic max), the others poll
// their relay line at agent scope (the round-5 doorbell). A poller that
// waits ~0.5 s gives up, so the grid always drains.
__global__ void pingpong(unsigned long long *bell, unsigned reps, unsigned long long *relays, int relay,
                         unsigned long long *cnt, unsigned long long *h_ack, unsigned n, unsigned *err)
{
    if (threadIdx.x) return;
    unsigned long long *mine = bell + 16 * (blockIdx.x % reps);
    unsigned long long *rl = relays + 16 * (blockIdx.x % 8);
    const bool lead = relay && blockIdx.x == 0;
    for (unsigned i = 1; i <= n; i++) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        for (;;) {
            const unsigned long long v = (!relay || lead)
                                             ? __hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                                             : __hip_atomic_load(rl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (v >= i) {
                if (lead)
                    for (int x = 0; x < 8; x++) atomicMax(relays + 16 * x, v);
                break;
            }
            if (__builtin_amdgcn_s_memrealtime() - t0 > 50000000ull) {   // 0.5 s at 100 MHz
                atomicAdd(err, 1u);
                return;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        // when this poller saw i (GPU clock; the host reads the spread)
        cnt[(size_t)(i - 1) * gridDim.x + blockIdx.x] = __builtin_amdgcn_s_memrealtime();
        if (blockIdx.x == 0)
            __hip_atomic_store(h_ack, (unsigned long long)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static sigjmp_buf jb;
static void on_segv(int) { siglongjmp(jb, 1); }

static double now_us()
{
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

static unsigned long long *g_relays, *g_cnt;
static int g_relay;

static void run(const char *name, unsigned long long *bell_host, unsigned long long *bell_dev, unsigned reps,
                unsigned grid, unsigned long long *h_ack, unsigned long long *d_ack, unsigned *d_err)
{
    const unsigned n = 2000;
    for (unsigned r = 0; r < reps; r++) __atomic_store_n(&bell_host[16 * r], 0ull, __ATOMIC_SEQ_CST);
    __atomic_store_n(h_ack, 0ull, __ATOMIC_SEQ_CST);
    CK(hipMemset(d_err, 0, 4));
    CK(hipMemset(g_relays, 0, 8 * 128));
    CK(hipMemset(g_cnt, 0, (size_t)n * grid * 8));
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(pingpong, dim3(grid), dim3(64), 0, 0, bell_dev, reps, g_relays, g_relay, g_cnt, d_ack, n, d_err);
    std::vector<double> dt;
    bool lost = false;
    for (unsigned i = 1; i <= n && !lost; i++) {
        const double t0 = now_us();
        for (unsigned r = 0; r < reps; r++) __atomic_store_n(&bell_host[16 * r], (unsigned long long)i, __ATOMIC_RELEASE);
        __builtin_ia32_sfence();   // out of the write-combining buffers (device memory through the BAR)
        while (__atomic_load_n(h_ack, __ATOMIC_ACQUIRE) < i) {
            if (now_us() - t0 > 1e6) {
                lost = true;
                break;
            }
        }
        dt.push_back(now_us() - t0);
        const double t1 = now_us();
        while (now_us() - t1 < 30.0) {   // every poller has seen i before i + 1
        }
    }
    if (lost)   // release every poller so the grid drains
        for (unsigned r = 0; r < reps; r++) __atomic_store_n(&bell_host[16 * r], (unsigned long long)n, __ATOMIC_RELEASE);
    CK(hipDeviceSynchronize());
    unsigned err = 0;
    CK(hipMemcpy(&err, d_err, 4, hipMemcpyDeviceToHost));
    // lag of the last poller behind workgroup 0 (10 ns clock ticks), per i
    std::vector<unsigned long long> st((size_t)n * grid);
    CK(hipMemcpy(st.data(), g_cnt, st.size() * 8, hipMemcpyDeviceToHost));
    std::vector<double> lag;
    for (unsigned i = 100; i < n; i++) {
        const unsigned long long *r = &st[(size_t)i * grid];
        unsigned long long mx = r[0];
        for (unsigned w = 0; w < grid; w++) mx = std::max(mx, r[w]);
        if (r[0]) lag.push_back((mx - r[0]) * 0.01);
    }
    std::sort(lag.begin(), lag.end());
    std::sort(dt.begin() + std::min<size_t>(dt.size(), 100), dt.end());
    const size_t k = dt.size() > 100 ? 100 : 0;
    const size_t m = dt.size() - k;
    printf("%-34s%s grid %5u reps %u: write -> ack median %.2f us, p10 %.2f, p90 %.2f, max %.2f; last poller after wg 0: median %.2f us, p90 %.2f%s%s\n", name, g_relay ? " +relay" : "", grid,
           reps, m ? dt[k + m / 2] : -1.0, m ? dt[k + m / 10] : -1.0, m ? dt[k + m * 9 / 10] : -1.0,
           m ? dt.back() : -1.0, lag.empty() ? -1.0 : lag[lag.size() / 2],
           lag.empty() ? -1.0 : lag[lag.size() * 9 / 10], lost ? "  LOST" : "", err ? "  (poller timeouts)" : "");
    fflush(stdout);
}

int main()
{
    CK(hipSetDevice(0));
    unsigned *d_err = nullptr;
    CK(hipMalloc(&d_err, 4));
    CK(hipMalloc(&g_relays, 8 * 128));
    CK(hipMalloc(&g_cnt, (size_t)2000 * 1280 * 8));
    void *ack = nullptr, *dack = nullptr;
    CK(hipHostMalloc(&ack, 4096, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer(&dack, ack, 0));
    // bell in host memory
    void *hb = nullptr, *db = nullptr;
    CK(hipHostMalloc(&hb, 8 * 128, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer(&db, hb, 0));
    run("host bell, one poller", (unsigned long long *)hb, (unsigned long long *)db, 1, 1, (unsigned long long *)ack,
        (unsigned long long *)dack, d_err);
    g_relay = 1;   // the round-5 doorbell: one PCIe poller, device relays
    run("host bell, 1280 workers", (unsigned long long *)hb, (unsigned long long *)db, 1, 1280,
        (unsigned long long *)ack, (unsigned long long *)dack, d_err);
    g_relay = 0;
    // bell in device memory, written by the CPU
    const struct {
        unsigned flag;
        const char *name;
    } kinds[] = {{hipDeviceMallocFinegrained, "fine-grained"}, {hipDeviceMallocUncached, "uncached"}};
    for (const auto &kd : kinds) {
        void *p = nullptr;
        if (hipExtMallocWithFlags(&p, 8 * 128, kd.flag) != hipSuccess) {
            printf("%s device memory: allocation failed\n", kd.name);
            continue;
        }
        hipPointerAttribute_t a;
        memset(&a, 0, sizeof(a));
        if (hipPointerGetAttributes(&a, p) == hipSuccess)
            printf("%s: type %d device %p host %p\n", kd.name, (int)a.type, a.devicePointer, a.hostPointer);
        unsigned long long *hp = (unsigned long long *)(a.hostPointer ? a.hostPointer : p);
        struct sigaction sa, old;
        memset(&sa, 0, sizeof(sa));
        sa.sa_handler = on_segv;
        struct sigaction oldb;
        sigaction(SIGSEGV, &sa, &old);
        sigaction(SIGBUS, &sa, &oldb);
        bool ok = false;
        if (!sigsetjmp(jb, 1)) {
            __atomic_store_n(hp, 7ull, __ATOMIC_SEQ_CST);
            ok = __atomic_load_n(hp, __ATOMIC_SEQ_CST) == 7ull;
        }
        sigaction(SIGSEGV, &old, nullptr);
        sigaction(SIGBUS, &oldb, nullptr);
        printf("%s device memory: CPU store %s\n", kd.name, ok ? "ok" : "FAULTS");
        fflush(stdout);
        if (!ok) continue;
        char nm[64];
        snprintf(nm, sizeof nm, "dev bell (%s), one poller", kd.name);
        run(nm, hp, (unsigned long long *)p, 1, 1, (unsigned long long *)ack, (unsigned long long *)dack, d_err);
        snprintf(nm, sizeof nm, "dev bell (%s), 1280 workers", kd.name);
        run(nm, hp, (unsigned long long *)p, 8, 1280, (unsigned long long *)ack, (unsigned long long *)dack, d_err);
        run(nm, hp, (unsigned long long *)p, 1, 1280, (unsigned long long *)ack, (unsigned long long *)dack, d_err);
        g_relay = 1;
        run(nm, hp, (unsigned long long *)p, 1, 1280, (unsigned long long *)ack, (unsigned long long *)dack, d_err);
        g_relay = 0;
    }
    g_relay = 1;
    run("host bell, 1280 workers", (unsigned long long *)hb, (unsigned long long *)db, 1, 1280,
        (unsigned long long *)ack, (unsigned long long *)dack, d_err);
    return 0;
}
