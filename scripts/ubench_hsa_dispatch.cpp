// ubench_hsa_dispatch.cpp — round trip of a small kernel launched through HIP (hipLaunchKernelGGL) against the same
// code object dispatched by writing an AQL packet into our own HSA queue (kernel arguments in pinned host memory, no
// completion signal: the host spins on the kernel's flags).  Decides whether the object API's call path should own a
// user-mode queue.
//   hipcc --offload-arch=gfx950 -O3 --genco -o build/flag_kernel.hsaco scripts/hsa/flag_kernel.hip
//   hipcc --offload-arch=gfx950 -O3 -o build/ubench_hsa_dispatch scripts/ubench_hsa_dispatch.cpp -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fcntl.h>
#include <functional>
#include <unistd.h>
#include <vector>

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::fprintf(stderr, "%s: %s (%d)\n", #x, hipGetErrorString(e_), __LINE__); \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)
#define HK(x)                                                                   \
    do {                                                                        \
        hsa_status_t s_ = (x);                                                  \
        if (s_ != HSA_STATUS_SUCCESS) {                                         \
            const char *m = nullptr;                                            \
            hsa_status_string(s_, &m);                                          \
            std::fprintf(stderr, "%s: %s (%d)\n", #x, m ? m : "?", __LINE__);  \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

struct Args {
    unsigned char *dst;
    unsigned *flag;
    unsigned n, epoch;
};

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static void run(const char *name, int n, const std::function<void()> &f) {
    for (int i = 0; i < (n < 100 ? 0 : 50); ++i) f();
    std::vector<double> t;
    for (int i = 0; i < n; ++i) {
        const double a = now_us();
        f();
        t.push_back(now_us() - a);
    }
    std::sort(t.begin(), t.end());
    std::printf("{\"form\": \"%s\", \"median_us\": %.2f, \"p10_us\": %.2f, \"p90_us\": %.2f}\n", name, t[n / 2],
                t[n / 10], t[n * 9 / 10]);
    std::fflush(stdout);
}

static hsa_status_t find_gpu(hsa_agent_t a, void *out) {
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_GPU) {
        *static_cast<hsa_agent_t *>(out) = a;
        return HSA_STATUS_INFO_BREAK;
    }
    return HSA_STATUS_SUCCESS;
}

int main(int argc, char **argv) {
    const char *co = argc > 1 ? argv[1] : "build/flag_kernel.hsaco";
    CK(hipSetDevice(0));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipModule_t mod;
    hipFunction_t fn;
    CK(hipModuleLoad(&mod, co));
    CK(hipModuleGetFunction(&fn, mod, "flag_kernel"));

    HK(hsa_init());
    hsa_agent_t gpu{};
    hsa_iterate_agents(find_gpu, &gpu);
    hsa_queue_t *q = nullptr;
    HK(hsa_queue_create(gpu, 256, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q));
    hsa_code_object_reader_t rd;
    const int fd = open(co, O_RDONLY);
    HK(hsa_code_object_reader_create_from_file(fd, &rd));
    hsa_executable_t exe;
    HK(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &exe));
    HK(hsa_executable_load_agent_code_object(exe, gpu, rd, nullptr, nullptr));
    HK(hsa_executable_freeze(exe, nullptr));
    hsa_executable_symbol_t sym;
    HK(hsa_executable_get_symbol_by_name(exe, "flag_kernel.kd", &gpu, &sym));
    uint64_t kobj = 0;
    uint32_t kas = 0, gss = 0, pss = 0;
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &kobj));
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &kas));
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &gss));
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &pss));
    std::printf("{\"kernarg_segment_size\": %u, \"group\": %u, \"private\": %u}\n", kas, gss, pss);

    unsigned char *dst;
    unsigned *flag;
    unsigned char *karg;
    CK(hipHostMalloc(&dst, 1 << 20, hipHostMallocCoherent));
    CK(hipHostMalloc(&flag, 4096, hipHostMallocCoherent));
    const int kRing = 64;
    CK(hipHostMalloc(&karg, size_t(kRing) * 512, hipHostMallocCoherent));
    std::memset(flag, 0, 4096);
    std::vector<unsigned char> page(1 << 20, 1);
    unsigned epoch = 0;
    auto spin = [&](unsigned g) {
        for (unsigned b = 0; b < g; ++b)
            while (__atomic_load_n(flag + b, __ATOMIC_ACQUIRE) != epoch) __builtin_ia32_pause();
    };
    auto hsa_launch = [&](unsigned g, unsigned n, int acq, int rel) {
        const uint64_t idx = hsa_queue_add_write_index_relaxed(q, 1);
        while (idx - hsa_queue_load_read_index_scacquire(q) >= q->size) __builtin_ia32_pause();
        Args *a = reinterpret_cast<Args *>(karg + (idx % kRing) * 512);
        a->dst = dst;
        a->flag = flag;
        a->n = n;
        a->epoch = epoch;
        auto *pk = static_cast<hsa_kernel_dispatch_packet_t *>(q->base_address) + (idx % q->size);
        pk->workgroup_size_x = 256;
        pk->workgroup_size_y = 1;
        pk->workgroup_size_z = 1;
        pk->grid_size_x = g * 256;
        pk->grid_size_y = 1;
        pk->grid_size_z = 1;
        pk->private_segment_size = pss;
        pk->group_segment_size = gss;
        pk->kernel_object = kobj;
        pk->kernarg_address = a;
        pk->completion_signal = hsa_signal_t{0};
        const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) | (1 << HSA_PACKET_HEADER_BARRIER) |
                                (acq << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                (rel << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
        const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
        __atomic_store_n(reinterpret_cast<uint32_t *>(pk), uint32_t(header) | (uint32_t(setup) << 16), __ATOMIC_RELEASE);
        hsa_signal_store_screlease(q->doorbell_signal, int64_t(idx));
    };
    for (unsigned n : {8192u, 65536u}) {
        const unsigned g = n / 16 / 256;
        char nm[160];
        std::snprintf(nm, sizeof nm, "HIP module launch + flag spin + memcpy, %u B", n);
        run(nm, 1000, [&] {
            ++epoch;
            Args a{dst, flag, n, epoch};
            void *cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, nullptr, HIP_LAUNCH_PARAM_END};
            size_t sz = sizeof a;
            cfg[3] = &sz;
            CK(hipModuleLaunchKernel(fn, g, 1, 1, 256, 1, 1, 0, s, nullptr, cfg));
            spin(g);
            std::memcpy(page.data(), dst, n);
        });
        CK(hipStreamSynchronize(s));
        for (int acq : {HSA_FENCE_SCOPE_SYSTEM, HSA_FENCE_SCOPE_AGENT})
            for (int rel : {HSA_FENCE_SCOPE_SYSTEM, HSA_FENCE_SCOPE_AGENT}) {
                std::snprintf(nm, sizeof nm, "HSA AQL dispatch (acquire %s, release %s) + flag spin + memcpy, %u B",
                              acq == HSA_FENCE_SCOPE_SYSTEM ? "system" : "agent",
                              rel == HSA_FENCE_SCOPE_SYSTEM ? "system" : "agent", n);
                run(nm, 1000, [&] {
                    ++epoch;
                    hsa_launch(g, n, acq, rel);
                    spin(g);
                    std::memcpy(page.data(), dst, n);
                });
            }
        // host cost of the dispatch alone
        std::snprintf(nm, sizeof nm, "HSA AQL dispatch host cost only, %u B", n);
        run(nm, 40, [&] {
            ++epoch;
            hsa_launch(g, n, HSA_FENCE_SCOPE_SYSTEM, HSA_FENCE_SCOPE_AGENT);
        });
        spin(g);
    }
    while (hsa_queue_load_read_index_scacquire(q) != hsa_queue_load_write_index_relaxed(q)) __builtin_ia32_pause();
    std::printf("{\"check\": %u}\n", unsigned(page[0]));
    hsa_queue_destroy(q);
    return 0;
}
