// Deferred destruction off a hot thread.
//
// The informer releases a wave's worth of deleted Pod objects at once (their
// metadata maps, container vectors, strings): tens of thousands of frees on
// the thread the scheduler's cache drain waits for. `defer` hands ownership
// to one background thread that drops it instead. The thread and its queue
// are never destroyed (a leaked singleton), so a batch still queued at
// process exit is simply not freed.
#pragma once

#include <memory>

namespace xsched {

// Takes ownership of `garbage` and destroys it on the reaper thread.
void defer_destroy(std::shared_ptr<void> garbage);

}  // namespace xsched
