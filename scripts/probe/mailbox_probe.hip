// Probe: round-trip latency of a resident (persistent) kernel served through a mailbox in
// fine-grained pinned host memory -- the transport of the per-sample Filterbank engine.
// Host posts (x, seq); one workgroup polls seq (system-scope acquire loads), computes, writes
// y and done (system-scope release stores).  The kernel leaves on a STOP request or after
// `idle_ticks` of the 100 MHz real-time counter without a request (exit flag = its epoch), so
// every wave always reaches the end.  Prints p50 / p99 / mean round trip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <cstdio>
#include <thread>
#include <vector>

struct Mailbox {
    double x;
    long long cmd;        // 0 compute, 1 stop
    long long req;        // written last by the host
    long long pad0[5];
    double y;
    long long done;       // written last by the device
    long long exited;     // epoch of the instance that left
    long long pad1[5];
};

__device__ __forceinline__ long long ld_sys(const long long* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(long long* p, long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(256) void resident(Mailbox* mb, long long epoch, long long idle_ticks, double* state) {
    __shared__ long long s_req;
    __shared__ double s_x;
    __shared__ double s_part[4];
    double acc = state[threadIdx.x];
    long long seen = mb->done;   // requests <= done are served
    long long last = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        if (threadIdx.x == 0) {
            long long r;
            for (;;) {
                r = ld_sys(&mb->req);
                if (r != seen) break;
                const long long now = __builtin_amdgcn_s_memrealtime();
                if (now - last > idle_ticks) {
                    r = -1;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            if (r > 0) {
                const long long c = __hip_atomic_load(&mb->cmd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                s_x = __hip_atomic_load(&mb->x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if (c == 1) r = -1;
            }
            s_req = r;
        }
        __syncthreads();
        const long long r = s_req;
        if (r < 0) break;
        acc = 0.999 * acc + s_x * (threadIdx.x + 1);
        double v = acc;
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6] = v;
        __syncthreads();
        if (threadIdx.x == 0) {
            __hip_atomic_store(&mb->y, s_part[0] + s_part[1] + s_part[2] + s_part[3], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
            st_sys(&mb->done, r);
        }
        seen = r;
        last = __builtin_amdgcn_s_memrealtime();
    }
    state[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x == 0) st_sys(&mb->exited, epoch);
}

#define CHECK(e)                                                               \
    do {                                                                       \
        hipError_t r_ = (e);                                                   \
        if (r_ != hipSuccess) {                                                \
            std::printf("%s: %s\n", #e, hipGetErrorString(r_));                \
            return 1;                                                          \
        }                                                                      \
    } while (0)

static long long vload(const long long* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }

int main() {
    Mailbox* mb = nullptr;
    CHECK(hipHostMalloc((void**)&mb, sizeof(Mailbox), hipHostMallocCoherent | hipHostMallocMapped));
    std::memset((void*)mb, 0, sizeof(Mailbox));
    Mailbox* dmb = nullptr;
    CHECK(hipHostGetDevicePointer((void**)&dmb, mb, 0));
    double* state = nullptr;
    CHECK(hipMalloc(&state, 256 * sizeof(double)));
    CHECK(hipMemset(state, 0, 256 * sizeof(double)));
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const long long idle = 5000000;   // 50 ms at 100 MHz
    long long epoch = 1, seq = 0;
    hipLaunchKernelGGL(resident, dim3(1), dim3(256), 0, s, dmb, epoch, idle, state);
    CHECK(hipGetLastError());
    auto post = [&](double x, long long cmd) {
        mb->x = x;
        mb->cmd = cmd;
        __atomic_store_n(&mb->req, ++seq, __ATOMIC_RELEASE);
    };
    auto wait_done = [&](long long want) -> int {
        const auto t0 = std::chrono::steady_clock::now();
        for (;;) {
            if (vload(&mb->done) >= want) return 0;
            if (vload(&mb->exited) == epoch) return 2;
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) return 1;
        }
    };
    std::vector<double> us;
    for (int pass = 0; pass < 2; ++pass) {
        us.clear();
        for (int i = 0; i < 20000; ++i) {
            const auto t0 = std::chrono::steady_clock::now();
            post(1e-3 * (i % 7), 0);
            const int w = wait_done(seq);
            const auto t1 = std::chrono::steady_clock::now();
            if (w == 1) {
                std::printf("timeout at request %lld\n", seq);
                post(0, 1);
                (void)hipStreamSynchronize(s);
                return 1;
            }
            if (w == 2) {   // the instance left before serving: relaunch, it serves the pending request
                ++epoch;
                hipLaunchKernelGGL(resident, dim3(1), dim3(256), 0, s, dmb, epoch, idle, state);
                if (wait_done(seq) != 0) {
                    std::printf("relaunch failed\n");
                    return 1;
                }
            }
            us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
        }
        std::sort(us.begin(), us.end());
        double mean = 0;
        for (double v : us) mean += v;
        mean /= us.size();
        std::printf("pass %d: round trip p50 %.2f us, p99 %.2f us, max %.2f us, mean %.2f us (y=%g)\n", pass,
                    us[us.size() / 2], us[us.size() * 99 / 100], us.back(), mean, mb->y);
        if (pass == 0) {   // idle exit, then the relaunch path
            std::this_thread::sleep_for(std::chrono::milliseconds(200));
            std::printf("exited flag after idle: %lld (epoch %lld)\n", vload(&mb->exited), epoch);
            CHECK(hipStreamSynchronize(s));
            ++epoch;
            hipLaunchKernelGGL(resident, dim3(1), dim3(256), 0, s, dmb, epoch, idle, state);
        }
    }
    post(0, 1);
    CHECK(hipStreamSynchronize(s));
    std::printf("stopped: exited flag %lld (epoch %lld)\n", vload(&mb->exited), epoch);
    return 0;
}
