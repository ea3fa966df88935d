// ubench_call_latency.hip — the floor of one synchronous object-API call on this box: what a host -> device ->
// host round trip costs with each launch / completion / output form, so that Encoder::code_with_buf and
// Recoder::recode_with_buf at the reference's 1 MB bench shapes (11-22 us on an EPYC core) can be designed
// against measured numbers.  Prints one JSON line per form (median / p10 / p90 over N calls, microseconds).
//
//   hipcc --offload-arch=gfx950 -O3 -o build/ubench_call_latency scripts/ubench_call_latency.hip
//   build/ubench_call_latency [spin]     (spin: hipSetDeviceFlags(hipDeviceScheduleSpin) first)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s: %s (%d)\n", #x, hipGetErrorString(e_), __LINE__);    \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

struct Big {
    unsigned char b[256];
};

__global__ void empty_kernel() {}

__global__ void arg_kernel(Big a, unsigned char *out) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && out) out[0] = a.b[threadIdx.x];
}

// writes n bytes (16 per lane) to dst
__global__ void write_kernel(unsigned char *dst, size_t n, unsigned v) {
    size_t i = (size_t(blockIdx.x) * blockDim.x + threadIdx.x) * 16;
    if (i + 16 <= n) *reinterpret_cast<uint4 *>(dst + i) = make_uint4(v, v, v, v);
}

// as write_kernel, then the last workgroup to finish raises *flag (system scope) -- the host spins on it
__global__ void write_flag_kernel(unsigned char *dst, size_t n, unsigned v, unsigned *count, unsigned *flag,
                                  unsigned epoch) {
    size_t i = (size_t(blockIdx.x) * blockDim.x + threadIdx.x) * 16;
    if (i + 16 <= n) *reinterpret_cast<uint4 *>(dst + i) = make_uint4(v, v, v, v);
    __syncthreads();
    if (threadIdx.x == 0) {
        __atomic_thread_fence(__ATOMIC_RELEASE);  // agent+system: the block's stores before the count
        unsigned prev = __hip_atomic_fetch_add(count, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == gridDim.x - 1) {
            *count = 0;
            __hip_atomic_store(flag, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void report(const char *name, size_t bytes, std::vector<double> &t) {
    std::sort(t.begin(), t.end());
    std::printf("{\"form\": \"%s\", \"bytes\": %zu, \"median_us\": %.2f, \"p10_us\": %.2f, \"p90_us\": %.2f}\n", name,
                bytes, t[t.size() / 2], t[t.size() / 10], t[t.size() * 9 / 10]);
    std::fflush(stdout);
}

static void run(const char *name, size_t bytes, int n, const std::function<void()> &f) {
    for (int i = 0; i < 20; ++i) f();
    std::vector<double> t;
    t.reserve(n);
    for (int i = 0; i < n; ++i) {
        double a = now_us();
        f();
        t.push_back(now_us() - a);
    }
    report(name, bytes, t);
}

int main(int argc, char **argv) {
    const bool spin = argc > 1 && std::strcmp(argv[1], "spin") == 0;
    if (spin) CK(hipSetDeviceFlags(hipDeviceScheduleSpin));
    CK(hipSetDevice(0));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    const int N = 2000;
    const size_t kMax = size_t(1) << 20;
    unsigned char *dev, *pin, *pin_c, *pin_wc;
    CK(hipMalloc(&dev, kMax));
    CK(hipHostMalloc(&pin, kMax, hipHostMallocDefault));
    CK(hipHostMalloc(&pin_c, kMax, hipHostMallocCoherent));
    CK(hipHostMalloc(&pin_wc, kMax, hipHostMallocNonCoherent));
    unsigned *cnt, *flag;
    CK(hipMalloc(&cnt, 4));
    CK(hipMemset(cnt, 0, 4));
    CK(hipHostMalloc(&flag, 64, hipHostMallocCoherent));
    *flag = 0;
    std::vector<unsigned char> page(kMax, 1), page2(kMax, 1);
    Big big{};
    std::printf("{\"mode\": \"%s\"}\n", spin ? "hipDeviceScheduleSpin" : "default");

    run("empty launch + hipStreamSynchronize", 0, N, [&] {
        hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
        CK(hipStreamSynchronize(s));
    });
    run("empty launch + event record + hipEventSynchronize", 0, N, [&] {
        hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
        CK(hipEventRecord(ev, s));
        CK(hipEventSynchronize(ev));
    });
    run("256-B kernarg launch + hipStreamSynchronize", 256, N, [&] {
        hipLaunchKernelGGL(arg_kernel, dim3(1), dim3(64), 0, s, big, (unsigned char *)nullptr);
        CK(hipStreamSynchronize(s));
    });
    run("launch only (no wait)", 0, N, [&] { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s); });
    CK(hipStreamSynchronize(s));
    run("256-B kernarg launch only (no wait)", 256, N,
        [&] { hipLaunchKernelGGL(arg_kernel, dim3(1), dim3(64), 0, s, big, (unsigned char *)nullptr); });
    CK(hipStreamSynchronize(s));
    run("pageable 32-B H2D hipMemcpyAsync + launch + sync", 32, N, [&] {
        CK(hipMemcpyAsync(dev, page.data(), 32, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
        CK(hipStreamSynchronize(s));
    });
    unsigned epoch = 0;
    for (size_t bytes : {size_t(8) << 10, size_t(64) << 10, size_t(256) << 10, size_t(1) << 20}) {
        const unsigned g = unsigned((bytes / 16 + 255) / 256);
        char nm[128];
        std::snprintf(nm, sizeof nm, "kernel -> device + pageable D2H + sync");
        run(nm, bytes, N / 4, [&] {
            hipLaunchKernelGGL(write_kernel, dim3(g), dim3(256), 0, s, dev, bytes, 7u);
            CK(hipMemcpyAsync(page.data(), dev, bytes, hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
        });
        run("kernel -> device + pinned D2H + sync + memcpy to pageable", bytes, N / 4, [&] {
            hipLaunchKernelGGL(write_kernel, dim3(g), dim3(256), 0, s, dev, bytes, 7u);
            CK(hipMemcpyAsync(pin, dev, bytes, hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
            std::memcpy(page.data(), pin, bytes);
        });
        run("kernel -> pinned(default) + sync", bytes, N / 4, [&] {
            hipLaunchKernelGGL(write_kernel, dim3(g), dim3(256), 0, s, pin, bytes, 7u);
            CK(hipStreamSynchronize(s));
        });
        run("kernel -> pinned(default) + sync + memcpy to pageable", bytes, N / 4, [&] {
            hipLaunchKernelGGL(write_kernel, dim3(g), dim3(256), 0, s, pin, bytes, 7u);
            CK(hipStreamSynchronize(s));
            std::memcpy(page.data(), pin, bytes);
        });
        run("kernel -> pinned(coherent) + sync + memcpy to pageable", bytes, N / 4, [&] {
            hipLaunchKernelGGL(write_kernel, dim3(g), dim3(256), 0, s, pin_c, bytes, 7u);
            CK(hipStreamSynchronize(s));
            std::memcpy(page.data(), pin_c, bytes);
        });
        run("kernel -> pinned(noncoherent) + sync + memcpy to pageable", bytes, N / 4, [&] {
            hipLaunchKernelGGL(write_kernel, dim3(g), dim3(256), 0, s, pin_wc, bytes, 7u);
            CK(hipStreamSynchronize(s));
            std::memcpy(page.data(), pin_wc, bytes);
        });
        run("kernel -> pinned(coherent) + flag spin + memcpy to pageable", bytes, N / 4, [&] {
            ++epoch;
            hipLaunchKernelGGL(write_flag_kernel, dim3(g), dim3(256), 0, s, pin_c, bytes, 7u, cnt, flag, epoch);
            while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != epoch) {
            }
            std::memcpy(page.data(), pin_c, bytes);
        });
        CK(hipStreamSynchronize(s));
        run("memcpy pageable -> pageable", bytes, N / 4, [&] { std::memcpy(page2.data(), page.data(), bytes); });
        run("memcpy pinned(default) -> pageable", bytes, N / 4, [&] { std::memcpy(page.data(), pin, bytes); });
    }
    CK(hipStreamSynchronize(s));
    std::printf("{\"check\": %u}\n", unsigned(page[0]) + unsigned(pin_c[0]));
    return 0;
}
