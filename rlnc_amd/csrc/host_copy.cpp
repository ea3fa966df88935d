// host_copy.cpp — parallel host copies (host_copy.hpp).
#include "host_copy.hpp"

#include <algorithm>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

namespace rlnc::eng {
namespace {

constexpr size_t kMinSlice = size_t(1) << 20;  // below this per thread the hand-off costs more than it saves
constexpr size_t kPage = 4096;

// one store into every 4 KiB page that dst[a, b) intersects
void touch(uint8_t *dst, size_t a, size_t b) {
    if (a >= b) return;
    volatile uint8_t *v = dst;
    v[a] = 0;
    for (size_t i = (a + kPage - reinterpret_cast<uintptr_t>(dst + a) % kPage); i < b; i += kPage) v[i] = 0;
}

// Persistent workers (created on first use, detached: they sleep on the condition variable between copies and die
// with the process).  One copy at a time; concurrent callers serialise on `call_mu` (a copy of many MiB is
// bandwidth-bound, two at once would not finish sooner).
class Pool {
   public:
    // src == nullptr: touch instead of copy (one zero byte in each 4 KiB page of each slice)
    void run(uint8_t *dst, const uint8_t *src, size_t n, int threads) {
        std::lock_guard<std::mutex> call(call_mu_);
        ensure(threads - 1);
        // slice boundaries on page boundaries of the destination ADDRESS (dst + offset), whatever dst's alignment:
        // slice 0 runs to the first page boundary past its share, every later slice starts on one, so no two threads
        // fault the same page
        const size_t per = ((n + threads - 1) / threads + kPage - 1) & ~(kPage - 1);
        const size_t lead = (kPage - reinterpret_cast<uintptr_t>(dst) % kPage) % kPage;
        {
            std::lock_guard<std::mutex> lock(mu_);
            dst_ = dst;
            src_ = src;
            n_ = n;
            per_ = per;
            lead_ = lead;
            next_ = 1;  // slice 0 is the caller's
            slices_ = n > lead + per ? (n - lead + per - 1) / per : 1;
            pending_ = slices_ - 1;
        }
        cv_.notify_all();
        copy_slice(0);
        std::unique_lock<std::mutex> lock(mu_);
        // the caller takes slices too until none is left unclaimed, then waits for the workers' last ones
        while (next_ < slices_) {
            const size_t s = next_++;
            lock.unlock();
            copy_slice(s);
            lock.lock();
            --pending_;
        }
        done_.wait(lock, [&] { return pending_ == 0; });
    }

   private:
    // slice s = [bound(s), bound(s + 1)): bound(0) = 0, bound(s) = lead + s * per (a page boundary of dst + offset)
    size_t bound(size_t s) const { return s == 0 ? 0 : std::min(n_, lead_ + s * per_); }
    void copy_slice(size_t s) {
        const size_t a = bound(s), b = s + 1 == slices_ ? n_ : bound(s + 1);
        if (src_ != nullptr) {
            std::memcpy(dst_ + a, src_ + a, b - a);
        } else {
            touch(dst_, a, b);
        }
    }
    void ensure(int workers) {
        while (int(workers_) < workers) {
            std::thread([this] { loop(); }).detach();
            ++workers_;
        }
    }
    void loop() {
        std::unique_lock<std::mutex> lock(mu_);
        for (;;) {
            cv_.wait(lock, [&] { return next_ < slices_; });
            const size_t s = next_++;
            lock.unlock();
            copy_slice(s);
            lock.lock();
            if (--pending_ == 0) done_.notify_one();
        }
    }
    std::mutex call_mu_, mu_;
    std::condition_variable cv_, done_;
    size_t workers_ = 0;
    uint8_t *dst_ = nullptr;
    const uint8_t *src_ = nullptr;
    size_t n_ = 0, per_ = 0, lead_ = 0, next_ = 0, slices_ = 0, pending_ = 0;
};

Pool &pool() {
    static Pool *p = new Pool;  // never destroyed: detached workers may still wait on it at exit
    return *p;
}

}  // namespace

void par_touch(void *dst, size_t n, int threads) {
    threads = int(std::min<size_t>(size_t(std::max(1, threads)), n / kMinSlice));
    if (threads <= 1) {
        touch(static_cast<uint8_t *>(dst), 0, n);
        return;
    }
    pool().run(static_cast<uint8_t *>(dst), nullptr, n, threads);
}

int copy_threads() {
    static const int t = [] {
        if (const char *e = std::getenv("RLNC_COPY_THREADS")) return std::max(1, std::atoi(e));
        return int(std::min<unsigned>(8, std::max<unsigned>(1, std::thread::hardware_concurrency())));
    }();
    return t;
}

void par_copy(void *dst, const void *src, size_t n, int threads) {
    threads = int(std::min<size_t>(size_t(std::max(1, threads)), n / kMinSlice));
    if (threads <= 1) {
        std::memcpy(dst, src, n);
        return;
    }
    pool().run(static_cast<uint8_t *>(dst), static_cast<const uint8_t *>(src), n, threads);
}

}  // namespace rlnc::eng
