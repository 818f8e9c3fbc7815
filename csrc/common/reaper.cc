#include "common/reaper.h"

#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#include "common/clock.h"

namespace xsched {
namespace {

struct Reaper {
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::shared_ptr<void>> q;

  Reaper() {
    std::thread([this] {
      name_this_thread("xs-free");
      std::unique_lock<std::mutex> lk(mu);
      for (;;) {
        cv.wait(lk, [&] { return !q.empty(); });
        std::vector<std::shared_ptr<void>> batch;
        batch.swap(q);
        lk.unlock();
        batch.clear();  // the frees
        lk.lock();
      }
    }).detach();
  }
};

Reaper& reaper() {
  static Reaper* r = new Reaper();  // never destroyed: the detached thread outlives static destruction
  return *r;
}

}  // namespace

void defer_destroy(std::shared_ptr<void> garbage) {
  if (!garbage) return;
  Reaper& r = reaper();
  {
    std::lock_guard<std::mutex> g(r.mu);
    r.q.push_back(std::move(garbage));
  }
  r.cv.notify_one();
}

}  // namespace xsched
