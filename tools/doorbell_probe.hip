// doorbell_probe.hip — diagnostic: host -> GPU -> host ping-pong latency of
// the doorbell forms a poll-mode kernel can use (not the product).
//   host-mem : the host bumps a word in mapped pinned host memory; one GPU
//              lane polls it over PCIe (system-scope loads) and answers in
//              another mapped host word.
//   dev-mem  : the host bumps a word in fine-grained DEVICE memory through
//              its host mapping (if the platform maps it: large BAR); the
//              lane polls it locally.
// One workgroup of one wave; every spin bounded; the kernel leaves on a
// stop value or after ~2 s without progress.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <sys/wait.h>
#include <unistd.h>
#include <algorithm>
#include <vector>

#define CHK(x)                                                                            \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                       \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

__global__ void pong(unsigned long long *bell, int system_scope, unsigned long long *ack, unsigned long long n)
{
    if (threadIdx.x != 0) return;
    unsigned long long want = 1, t_last = __builtin_amdgcn_s_memrealtime();
    while (want <= n) {
        const unsigned long long v = system_scope
                                         ? __hip_atomic_load(bell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                                         : __hip_atomic_load(bell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long now = __builtin_amdgcn_s_memrealtime();
        if (v >= want) {
            __hip_atomic_store(ack, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            want = v + 1;
            t_last = now;
        } else if (now - t_last > 200000000ull) {   // 2 s without a ping: leave
            return;
        }
    }
}

static double run(unsigned long long *bell_host, unsigned long long *bell_dev, int system_scope,
                  volatile unsigned long long *ack_host, unsigned long long *ack_dev, int n)
{
    *(volatile unsigned long long *)bell_host = 0;
    *ack_host = 0;
    hipLaunchKernelGGL(pong, dim3(1), dim3(64), 0, 0, bell_dev, system_scope, ack_dev, (unsigned long long)n);
    std::vector<double> us;
    for (int i = 1; i <= n; i++) {
        const auto t0 = std::chrono::steady_clock::now();
        __atomic_store_n((unsigned long long *)bell_host, (unsigned long long)i, __ATOMIC_SEQ_CST);
        for (long spin = 0; *ack_host < (unsigned long long)i; spin++)
            if (spin > 2000000000L) {
                fprintf(stderr, "no ack\n");
                exit(2);
            }
        us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    CHK(hipDeviceSynchronize());
    std::sort(us.begin(), us.end());
    return us[us.size() / 2];
}

int main()
{
    const int n = 2000;
    unsigned long long *ack = nullptr, *ack_dev = nullptr;
    CHK(hipHostMalloc(&ack, 64, hipHostMallocMapped | hipHostMallocCoherent));
    CHK(hipHostGetDevicePointer((void **)&ack_dev, ack, 0));
    // host-memory doorbell
    unsigned long long *hb = nullptr, *hb_dev = nullptr;
    CHK(hipHostMalloc(&hb, 64, hipHostMallocMapped | hipHostMallocCoherent));
    CHK(hipHostGetDevicePointer((void **)&hb_dev, hb, 0));
    printf("host-mem doorbell: ping-pong median %.2f us\n", run(hb, hb_dev, 1, ack, ack_dev, n));
    // device-memory doorbell, written by the host through its mapping
    unsigned long long *db = nullptr;
    CHK(hipExtMallocWithFlags((void **)&db, 4096, hipDeviceMallocFinegrained));
    hipPointerAttribute_t attr;
    CHK(hipPointerGetAttributes(&attr, db));
    printf("fine-grained device memory: device %p host %p\n", attr.devicePointer, attr.hostPointer);
    // is it host-writable? try in a child first (a fault kills only the child)
    fflush(stdout);
    pid_t pid = fork();
    if (pid == 0) {
        *(volatile unsigned long long *)db = 0;
        _exit(0);
    }
    int st = 0;
    waitpid(pid, &st, 0);
    if (!(WIFEXITED(st) && WEXITSTATUS(st) == 0)) {
        printf("dev-mem doorbell: not host-writable here (child status %d)\n", st);
        return 0;
    }
    printf("dev-mem doorbell: ping-pong median %.2f us\n", run(db, db, 0, ack, ack_dev, n));
    return 0;
}
