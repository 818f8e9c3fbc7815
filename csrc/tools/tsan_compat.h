// Force-included into the ThreadSanitizer build only. GCC 11's libtsan does
// not intercept pthread_cond_clockwait, which libstdc++ uses for
// condition_variable::wait_for on steady_clock; TSan then loses the mutex
// re-acquisition and reports phantom races / double locks. Falling back to
// pthread_cond_timedwait (intercepted) keeps the analysis sound.
#pragma once
#include <bits/c++config.h>
#undef _GLIBCXX_USE_PTHREAD_COND_CLOCKWAIT
