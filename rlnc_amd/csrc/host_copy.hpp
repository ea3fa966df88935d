// host_copy.hpp — a small pool of host threads that copies large buffers in parallel (internal to librlnc_hip).
//
// Decoder::get_decoded_data hands its output to a caller buffer the caller has just allocated (the reference builds a
// fresh `vec![0u8; k·L]`, decoder.rs:141-142).  At many MiB such a buffer is a fresh mapping whose pages fault in on
// first write, and one thread copying (and faulting) 32 MiB is what bounded the copy-out (round 4: 5.8 ms of a 7 ms
// decode).  The pool splits a copy into page-aligned slices of the destination, one per thread, so the page faults
// and the bytes are spread over several cores.
#pragma once
#include <cstddef>

namespace rlnc::eng {

// dst[0, n) = src[0, n) with up to `threads` threads (the caller's included); returns when done.  Small copies stay on
// the calling thread.
void par_copy(void *dst, const void *src, size_t n, int threads);
// the pages of dst[0, n) faulted in (one zero byte written per 4 KiB) by up to `threads` threads: a caller buffer
// fresh from calloc is then warm when the device's bytes arrive (call it while the device works)
void par_touch(void *dst, size_t n, int threads);
// the thread count par_copy callers use: RLNC_COPY_THREADS (A/B knob, read once), else min(8, hardware threads)
int copy_threads();

}  // namespace rlnc::eng
