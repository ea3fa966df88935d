// ubench_doorbell.hip — can a resident "piece server" kernel answer an object-API call faster than a launch?
// A server grid of G workgroups stays resident for a bounded lease; the host posts a request by storing a sequence
// number into coherent pinned memory, the grid sees it (every workgroup polling the host word, or workgroup 0
// polling it and fanning it out through a device word), each workgroup reads a 384-byte parameter block from host
// memory, writes `bytes` of output into pinned host memory with write-through stores and counts itself; the last
// raises the host flag.  Against it: the same work as one launch per call (the round-4 form of the piece path).
// Every wait in the kernel ends at the lease's deadline (s_memrealtime, 100 MHz), so the grid drains by itself.
// Prints one JSON line per form (median / p10 / p90 over N calls, microseconds).
//
//   hipcc --offload-arch=gfx950 -O3 -o build/ubench_doorbell scripts/ubench_doorbell.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s: %s (%d)\n", #x, hipGetErrorString(e_), __LINE__);    \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

constexpr uint32_t kExit = 0xFFFFFFFFu;
constexpr int kParamWords = 96;  // 384 bytes of parameters read per request
constexpr int kWT = 17;          // sc0 | sc1: write-through to system scope

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t rt() { return __builtin_amdgcn_s_memrealtime(); }

// a load the compiler cannot hoist or merge: ld 0 plain policy (served stale from a cache: never sees a new request),
// 1 sc1, 2 nt
__device__ __forceinline__ uint32_t load_host(const uint32_t *p, int ld) {
    uint32_t v;
    if (ld == 1)
        asm volatile("global_load_dword %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    else if (ld == 2)
        asm volatile("global_load_dword %0, %1, off nt\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    else
        asm volatile("global_load_dword %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return v;
}

// mode 0: every workgroup polls the host word; mode 1: workgroup 0 polls it and stores it to dword[0] (agent scope),
// the others poll dword[0]
__global__ __launch_bounds__(256) void server_kernel(const uint32_t *mb, uint32_t *hflag, uint32_t *dword,
                                                     uint8_t *out, int bytes, uint64_t lease, int mode,
                                                     uint32_t *hbeat, int ld) {
    __shared__ uint32_t s_seq;
    __shared__ uint32_t s_par[kParamWords];
    const uint64_t t_end = rt() + lease;
    const bool skip_par = ld >= 10;  // diagnostic
    ld %= 10;
    uint32_t local = 0;
    // every branch below is wave-uniform (the wave index and the request word are readfirstlane'd): with lane-0
    // branches the compiler merged the tail of one iteration with the poll of the next across the loop's back edge
    // and left the other lanes cycling through the barriers -- the first served request hung the workgroup
    const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x) >> 6);
    for (;;) {
        if (wave == 0) {
            uint32_t s = local;
            const bool host = mode == 0 || blockIdx.x == 0;
            const uint32_t *w = host ? mb : dword;
            // followers wait a little longer than the leader, whose deadline exit reaches them as kExit
            const uint64_t end = host ? t_end : t_end + 100000;
            for (uint32_t it = 0;; ++it) {
                if ((it & 255) == 0 && hbeat && threadIdx.x == 0) {  // diagnostic heartbeat: polls, last seen, clock
                    const __amdgpu_buffer_rsrc_t hb =
                        __builtin_amdgcn_make_buffer_rsrc(hbeat + 4 * blockIdx.x, 0, 16, 0x00020000);
                    const u32x4 x = {it, s, uint32_t(rt()), uint32_t(end)};
                    __builtin_amdgcn_raw_buffer_store_b128(x, hb, 0, 0, kWT);
                }
                if (ld == 3)
                    s = local;  // diagnostic: no load, the loop ends at the deadline
                else if (ld == 4)
                    s = __hip_atomic_load(dword + 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // device word
                else
                    s = host ? load_host(w, ld) : __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                s = uint32_t(__builtin_amdgcn_readfirstlane(int(s)));
                if (s != local) break;
                if (rt() > end) {
                    s = kExit;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (mode == 1 && blockIdx.x == 0) {
                // the leader copies the parameters into device memory (sc1 stores, drained) before it releases the
                // followers, who then read them there instead of each crossing PCIe
                if (s != kExit) {
                    const int l = int(threadIdx.x);
                    const uint32_t a = skip_par ? 0u : load_host(mb + 16 + l, ld);
                    const uint32_t b = (skip_par || l >= kParamWords - 64) ? 0u : load_host(mb + 16 + 64 + l, ld);
                    __hip_atomic_store(dword + 256 + l, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (l < kParamWords - 64)
                        __hip_atomic_store(dword + 256 + 64 + l, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                if (threadIdx.x == 0) __hip_atomic_store(dword, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (threadIdx.x == 0) s_seq = s;
        }
        __syncthreads();
        const uint32_t s = uint32_t(__builtin_amdgcn_readfirstlane(int(s_seq)));
        if (s == kExit) return;
        if (threadIdx.x < kParamWords)
            s_par[threadIdx.x] = skip_par ? 0u
                                 : mode == 1 ? __hip_atomic_load(dword + 256 + threadIdx.x, __ATOMIC_RELAXED,
                                                                 __HIP_MEMORY_SCOPE_AGENT)
                                             : load_host(mb + 16 + threadIdx.x, ld);
        __syncthreads();
        const uint32_t v = s ^ s_par[threadIdx.x % kParamWords];
        if (bytes > 0) {
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc(out + size_t(blockIdx.x) * bytes, 0, 0x7FFFFFFF, 0x00020000);
            for (int o = int(threadIdx.x) * 16; o < bytes; o += int(blockDim.x) * 16) {
                const u32x4 x = {v, v, v, v};
                __builtin_amdgcn_raw_buffer_store_b128(x, rs, o, 0, kWT);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (wave == 0) {
            uint32_t prev = 0;
            if (threadIdx.x == 0) prev = __hip_atomic_fetch_add(dword + 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            prev = uint32_t(__builtin_amdgcn_readfirstlane(int(prev)));
            if (prev == gridDim.x - 1 && threadIdx.x == 0) {
                __hip_atomic_store(dword + 32, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(hflag, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        local = s;
        __syncthreads();  // the tail of this request stays ahead of the next poll for every wave
    }
}

struct Params {
    uint32_t w[kParamWords];
};

// the launch-per-call form: the parameters travel as kernel arguments
__global__ __launch_bounds__(256) void launch_kernel(Params p, uint32_t *hflag, uint32_t *dword, uint8_t *out,
                                                     int bytes, uint32_t s) {
    const uint32_t v = s ^ p.w[threadIdx.x % kParamWords];
    if (bytes > 0) {
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(out + size_t(blockIdx.x) * bytes, 0, 0x7FFFFFFF, 0x00020000);
        for (int o = int(threadIdx.x) * 16; o < bytes; o += int(blockDim.x) * 16) {
            const u32x4 x = {v, v, v, v};
            __builtin_amdgcn_raw_buffer_store_b128(x, rs, o, 0, kWT);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t prev = __hip_atomic_fetch_add(dword + 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == gridDim.x - 1) {
            __hip_atomic_store(dword + 32, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(hflag, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static bool spin(const uint32_t *f, uint32_t v) {
    const double t0 = now_us();
    while (__atomic_load_n(f, __ATOMIC_ACQUIRE) != v)
        if (now_us() - t0 > 100000.0) return false;
    return true;
}

static void report(const char *form, int G, int bytes, std::vector<double> &t) {
    std::sort(t.begin(), t.end());
    std::printf("{\"form\": \"%s\", \"workgroups\": %d, \"bytes_per_wg\": %d, \"median_us\": %.2f, \"p10_us\": %.2f, "
                "\"p90_us\": %.2f}\n",
                form, G, bytes, t[t.size() / 2], t[t.size() / 10], t[t.size() * 9 / 10]);
    std::fflush(stdout);
}

int main(int argc, char **argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 2000;
    uint32_t *mb, *hflag, *dword, *hbeat;
    uint8_t *out;
    // the mailbox: 0 coherent pinned host memory (sc1 loads of a line the CPU wrote never returned), 1 write-combined
    // host memory (the CPU's stores bypass its caches; sfence after each), 2 fine-grained device memory the CPU
    // writes across the BAR
    const int mbk = argc > 4 ? atoi(argv[4]) : 0;
    if (mbk == 1)
        CK(hipHostMalloc(&mb, 4096, hipHostMallocWriteCombined));
    else if (mbk == 2)
        CK(hipExtMallocWithFlags(reinterpret_cast<void **>(&mb), 4096, hipDeviceMallocFinegrained));
    else
        CK(hipHostMalloc(&mb, 4096, hipHostMallocCoherent));
    CK(hipHostMalloc(&hflag, 4096, hipHostMallocCoherent));
    CK(hipHostMalloc(&out, 256 * 4096, hipHostMallocCoherent));
    CK(hipMalloc(&dword, 4096));
    CK(hipHostMalloc(&hbeat, 4096, hipHostMallocCoherent));
    std::memset(hbeat, 0, 4096);
    CK(hipMemset(dword, 0, 4096));
    std::memset(mb, 0, 4096);
    std::memset(hflag, 0, 4096);
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    Params P;
    for (int i = 0; i < kParamWords; ++i) P.w[i] = 0x9E3779B9u * i;
    for (int i = 0; i < kParamWords; ++i) mb[16 + i] = P.w[i];
    __builtin_ia32_sfence();
    CK(hipDeviceSynchronize());
    const uint64_t lease = 20000000ull;  // 0.2 s at 100 MHz
    if (argc > 2 && argv[2][0] != '-') {  // diagnostic: one server of 1 workgroup with load form argv[2], no requests; report its drain
        const int ld = atoi(argv[2]);
        const int post_ms = argc > 3 ? atoi(argv[3]) : -1;
        hipLaunchKernelGGL(server_kernel, dim3(1), dim3(256), 0, s, mb, hflag, dword, out, 0, lease, 0, hbeat, ld);
        CK(hipGetLastError());
        const double q0 = now_us();
        bool answered = false;
        if (post_ms >= 0) {
            while (now_us() - q0 < post_ms * 1000.0) {
            }
            __atomic_store_n(mb, 1u, __ATOMIC_RELEASE);
            __builtin_ia32_sfence();
            answered = spin(hflag, 1u);
            std::printf("{\"diag_ld\": %d, \"mailbox\": %d, \"posted_after_ms\": %d, \"answered\": %s, \"after_us\": %.1f, "
                        "\"polls\": %u, \"seen\": %u}\n",
                        ld, mbk, post_ms, answered ? "true" : "false", now_us() - q0 - post_ms * 1000.0, hbeat[0],
                        hbeat[1]);
            std::fflush(stdout);
            __atomic_store_n(mb, kExit, __ATOMIC_RELEASE);
            __builtin_ia32_sfence();
        }
        bool drained = false;
        while (now_us() - q0 < 3e6)
            if (hipStreamQuery(s) != hipErrorNotReady) {
                drained = true;
                break;
            }
        std::printf("{\"diag_ld\": %d, \"drained\": %s, \"after_us\": %.0f, \"polls\": %u, \"seen\": %u}\n", ld,
                    drained ? "true" : "false", now_us() - q0, hbeat[0], hbeat[1]);
        std::fflush(stdout);
        return drained ? 0 : 1;
    }
    for (int bytes : {0, 1024}) {
        for (int G : {1, 64, 128}) {
            // launch per call
            {
                std::vector<double> t;
                uint32_t seq = 0;
                for (int i = 0; i < N + 50; ++i) {
                    ++seq;
                    const double a = now_us();
                    hipLaunchKernelGGL(launch_kernel, dim3(G), dim3(256), 0, s, P, hflag, dword, out, bytes, seq);
                    if (!spin(hflag, seq)) {
                        std::fprintf(stderr, "launch form: flag timeout\n");
                        return 1;
                    }
                    if (i >= 50) t.push_back(now_us() - a);
                }
                CK(hipStreamSynchronize(s));
                report("launch per call + flag spin", G, bytes, t);
            }
            for (int mm : {2, 3}) {
                const int mode = mm & 1, ld = mm >> 1;  // the host words' loads: ld 0 plain, 1 sc1, 2 nt
                __atomic_store_n(mb, 0u, __ATOMIC_RELEASE);
                __builtin_ia32_sfence();
                __atomic_store_n(hflag, 0u, __ATOMIC_RELEASE);
                CK(hipMemset(dword, 0, 4096));
                CK(hipDeviceSynchronize());
                hipLaunchKernelGGL(server_kernel, dim3(G), dim3(256), 0, s, mb, hflag, dword, out, bytes, lease, mode, hbeat,
                                   ld);
                CK(hipGetLastError());
                std::vector<double> t;
                bool ok = true;
                for (uint32_t i = 1; i <= uint32_t(N + 50); ++i) {
                    const double a = now_us();
                    __atomic_store_n(mb, i, __ATOMIC_RELEASE);
                    __builtin_ia32_sfence();
                    if (!spin(hflag, i)) {
                        std::fprintf(stderr, "server mode %d ld %d G %d: flag timeout at %u; heartbeat wg0: polls %u seen %u "
                                             "clock %u end %u; flag %u\n", mode, ld, G, i, hbeat[0], hbeat[1], hbeat[2],
                                     hbeat[3], hflag[0]);
                        ok = false;
                        break;
                    }
                    if (i > 50) t.push_back(now_us() - a);
                }
                __atomic_store_n(mb, kExit, __ATOMIC_RELEASE);
                __builtin_ia32_sfence();
                const double q0 = now_us();
                while (hipStreamQuery(s) == hipErrorNotReady) {
                    if (now_us() - q0 > 2e6) {
                        std::fprintf(stderr, "server did not drain in 2 s; heartbeat polls %u seen %u clock %u end %u\n",
                                     hbeat[0], hbeat[1], hbeat[2], hbeat[3]);
                        std::fflush(stderr);
                        break;
                    }
                }
                if (!ok) return 1;
                static const char *lds[] = {"plain", "sc1", "nt"};
                char form[128];
                static const char *mbs[] = {"coherent host", "write-combined host", "fine-grained device"};
                std::snprintf(form, sizeof form, "server, %s, %s loads of a %s mailbox",
                              mode ? "leader fan-out" : "every workgroup polls it", lds[ld], mbs[mbk]);
                report(form, G, bytes, t);
            }
        }
    }
    return 0;
}
