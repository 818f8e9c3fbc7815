// Process allocator settings for the scheduler's allocation pattern.
//
// A scheduler process allocates in waves: a burst of pods arrives (watch
// events, Pod objects, cycle states, binding patches), is bound, and is
// deleted. With glibc's defaults every wave's memory is handed back to the
// kernel when it is freed (heap trim, and mmap/munmap for blocks over the
// dynamic threshold) and faulted in again by the next wave, on every thread
// that touches it. The Go reference leaves this to its runtime's heap, which
// keeps freed spans; this is the glibc equivalent: keep up to 1 GiB of freed
// heap in the process, grow the heap 64 MiB at a time, and serve blocks up
// to 32 MiB (glibc's maximum) from the heap instead of fresh mappings.
#pragma once

#include <string>

namespace xsched {

// Applies the settings once per process (later calls are no-ops) unless the
// environment sets XSCHED_MALLOC_TUNE=0. Returns a one-line description of
// what is in effect, for benchmark records.
const std::string& tune_allocator();

}  // namespace xsched
