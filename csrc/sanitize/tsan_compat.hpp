// Force-included into the TSan builds (bee-executor-tsan, bee-admission-test).  GCC 11's TSan
// runtime does not intercept pthread_cond_clockwait, which libstdc++ uses for
// condition_variable::wait_for on steady_clock; TSan then misses the mutex
// release inside the wait and reports a double lock plus false races on
// everything that mutex guards.  Falling back to pthread_cond_timedwait
// (intercepted) keeps the analysis exact.
#include <bits/c++config.h>
#undef _GLIBCXX_USE_PTHREAD_COND_CLOCKWAIT
