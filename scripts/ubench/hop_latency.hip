// Cross-queue dependency latency on MI355X: the time from the last block of
// kernel A finishing to kernel B starting, when B is ordered after A
//   S  on the same stream,
//   T  on the same stream after A launched with a stop event (as K2 is),
//   E  on another stream by hipStreamWaitEvent on an event recorded after A,
//   X  on another stream by hipStreamWaitEvent on A's own completion event
//      (hipExtLaunchKernelGGL stop event: what libmbots uses),
//   V  on another stream by hipStreamWaitValue32 on a flag A's last block sets.
// Times are s_memrealtime ticks (100 MHz) read inside the kernels.
//   hipcc --offload-arch=gfx950 -O3 -o hop_latency hop_latency.hip && ./hop_latency
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__device__ __forceinline__ unsigned long long rt() { return __builtin_amdgcn_s_memrealtime(); }

// ~busy work per block, then the last block to finish stamps the end time and
// (optionally) raises the flag
__global__ void kern_a(unsigned *count, unsigned long long *t_end, unsigned *flag, unsigned epoch, int iters)
{
    float v = threadIdx.x;
    for (int i = 0; i < iters; ++i) v = __builtin_fmaf(v, 0.999f, 0.5f);
    if (v == 12345.0f) t_end[1] = 1;   // keep the loop
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        const unsigned done = atomicAdd(count, 1u) + 1u;
        if (done == gridDim.x) {
            t_end[0] = rt();
            *count = 0u;
            if (flag) {
                __threadfence_system();
                __hip_atomic_store(flag, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
}

__global__ void kern_b(unsigned long long *t_start)
{
    if (threadIdx.x == 0 && blockIdx.x == 0) t_start[0] = rt();
}

// coherence check: A' writes `val` into data[] (plain stores, every block a
// slice), releases (agent fence) and counts itself; the last block raises the
// flag.  B' (after the value wait, on another queue) reads all of data[] in
// every block and counts the words that are not `val` (stale lines in its
// XCD's L2 would show up here: every block read the whole array last round).
__global__ void kern_a2(unsigned *data, int n, unsigned val, unsigned *count, unsigned *flag, unsigned epoch)
{
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) data[i] = val;
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        if (atomicAdd(count, 1u) == gridDim.x - 1u) {
            atomicExch(count, 0u);
            __hip_atomic_store(flag, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}
__global__ void kern_b2(const unsigned *data, int n, unsigned val, unsigned *bad)
{
    unsigned c = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) c += data[i] != val;
    if (c) atomicAdd(bad, c);
}

int main()
{
    hipStream_t s1, s2;
    int lo, hi;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    CK(hipStreamCreateWithPriority(&s1, hipStreamNonBlocking, hi));
    CK(hipStreamCreateWithPriority(&s2, hipStreamNonBlocking, hi));
    unsigned *count, *flag;
    unsigned long long *t;
    CK(hipMalloc(&count, 4));
    CK(hipMemset(count, 0, 4));
    CK(hipMalloc(&t, 64));
    if (hipExtMallocWithFlags((void **)&flag, 8, hipMallocSignalMemory) != hipSuccess) {
        (void)hipGetLastError();
        CK(hipMalloc(&flag, 64));   // plain device memory
        printf("(flag in plain device memory)\n");
    }
    CK(hipMemset(flag, 0, 4));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming | hipEventReleaseToDevice));
    const int blocks = 2048, iters = 20000, reps = 200;
    const char *names[5] = {"S same stream", "E event after A", "X A's own stop event", "V wait value",
                            "T same stream, A with a stop event"};
    unsigned epoch = 0;
    for (int mode = 0; mode < 5; ++mode) {
        std::vector<double> gaps;
        for (int r = 0; r < reps + 10; ++r) {
            ++epoch;
            unsigned *fl = mode == 3 ? flag : nullptr;
            if (mode == 2 || mode == 4) {
                hipExtLaunchKernelGGL(kern_a, dim3(blocks), dim3(256), 0, s1, nullptr, ev, 0u, count, t, fl, epoch,
                                      iters);
            } else {
                hipLaunchKernelGGL(kern_a, dim3(blocks), dim3(256), 0, s1, count, t, fl, epoch, iters);
            }
            if (mode == 0 || mode == 4) {
                hipLaunchKernelGGL(kern_b, dim3(1), dim3(64), 0, s1, t + 2);
            } else {
                if (mode == 1) CK(hipEventRecord(ev, s1));
                if (mode == 3) CK(hipStreamWaitValue32(s2, flag, epoch, hipStreamWaitValueGte, 0xFFFFFFFFu));
                else CK(hipStreamWaitEvent(s2, ev, 0));
                hipLaunchKernelGGL(kern_b, dim3(1), dim3(64), 0, s2, t + 2);
            }
            CK(hipDeviceSynchronize());
            unsigned long long h[3];
            CK(hipMemcpy(h, t, 24, hipMemcpyDeviceToHost));
            if (r >= 10) gaps.push_back(((double)h[2] - (double)h[0]) / 100.0);   // us (100 MHz)
        }
        std::sort(gaps.begin(), gaps.end());
        printf("{\"mode\": \"%s\", \"median_us\": %.2f, \"p10_us\": %.2f, \"p90_us\": %.2f}\n", names[mode],
               gaps[gaps.size() / 2], gaps[gaps.size() / 10], gaps[gaps.size() * 9 / 10]);
    }
    // coherence: 64 KB read by every block of B' (all XCDs cache it), then
    // rewritten by A' on the other queue
    {
        const int n = 16384, cb = 2048;
        unsigned *data, *bad;
        CK(hipMalloc(&data, n * 4));
        CK(hipMalloc(&bad, 4));
        CK(hipMemset(data, 0, n * 4));
        CK(hipMemset(bad, 0, 4));
        unsigned total_bad = 0;
        for (int r = 1; r <= 200; ++r) {
            ++epoch;
            hipLaunchKernelGGL(kern_a2, dim3(cb), dim3(256), 0, s1, data, n, (unsigned)r, count, flag, epoch);
            CK(hipStreamWaitValue32(s2, flag, epoch, hipStreamWaitValueEq, 0xFFFFFFFFu));
            hipLaunchKernelGGL(kern_b2, dim3(cb), dim3(256), 0, s2, data, n, (unsigned)r, bad);
            CK(hipDeviceSynchronize());
        }
        CK(hipMemcpy(&total_bad, bad, 4, hipMemcpyDeviceToHost));
        printf("{\"mode\": \"coherence after a value wait\", \"stale_words\": %u, \"rounds\": 200}\n", total_bad);
    }
    // host cost of the enqueue calls themselves (the flag already set, the
    // event already fired): what a host-bound loop pays per call
    {
        const int n = 2000;
        auto host_us = [&](auto &&call) -> double {
            (void)hipDeviceSynchronize();
            const auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < n; ++i) call();
            const auto t1 = std::chrono::steady_clock::now();
            (void)hipDeviceSynchronize();
            return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
        };
        CK(hipEventRecord(ev, s1));
        const double u_launch = host_us([&] { hipLaunchKernelGGL(kern_b, dim3(1), dim3(64), 0, s2, t + 2); });
        const double u_ext = host_us([&] {
            hipExtLaunchKernelGGL(kern_b, dim3(1), dim3(64), 0, s2, nullptr, ev, 0u, t + 2);
        });
        const double u_wev = host_us([&] { (void)hipStreamWaitEvent(s2, ev, 0); });
        const double u_wval = host_us([&] { (void)hipStreamWaitValue32(s2, flag, epoch, hipStreamWaitValueEq, 0xFFFFFFFFu); });
        printf("{\"mode\": \"host us per enqueue\", \"launch\": %.2f, \"ext_launch_with_event\": %.2f, "
               "\"wait_event\": %.2f, \"wait_value32\": %.2f}\n", u_launch, u_ext, u_wev, u_wval);
    }
    return 0;
}
