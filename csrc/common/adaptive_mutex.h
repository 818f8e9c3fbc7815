// A mutex that spins briefly before sleeping.
//
// std::mutex puts a contended locker to sleep on a futex at once. The
// scheduler cache's lock is taken by the scheduling thread several times per
// cycle (snapshot refresh, assume, Reserve's annotation) and by the informer
// for every confirmed binding, each time for well under a microsecond; a
// futex sleep and wake-up costs several. glibc's adaptive mutex spins (with
// backoff, bounded) on the owner before it sleeps.
#pragma once

#include <pthread.h>

namespace xsched {

class AdaptiveMutex {
 public:
  AdaptiveMutex() {
    pthread_mutexattr_t a;
    pthread_mutexattr_init(&a);
    pthread_mutexattr_settype(&a, PTHREAD_MUTEX_ADAPTIVE_NP);
    pthread_mutex_init(&m_, &a);
    pthread_mutexattr_destroy(&a);
  }
  ~AdaptiveMutex() { pthread_mutex_destroy(&m_); }
  AdaptiveMutex(const AdaptiveMutex&) = delete;
  AdaptiveMutex& operator=(const AdaptiveMutex&) = delete;
  void lock() { pthread_mutex_lock(&m_); }
  void unlock() { pthread_mutex_unlock(&m_); }
  bool try_lock() { return pthread_mutex_trylock(&m_) == 0; }

 private:
  pthread_mutex_t m_;
};

}  // namespace xsched
