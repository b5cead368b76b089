// tsan_clockwait.cpp -- linked into the TSan harness only.  libstdc++'s
// condition_variable::wait_until on steady_clock calls pthread_cond_clockwait,
// which this toolchain's libtsan does not intercept: TSan then misses the
// unlock / relock inside the wait and reports the next lock of the mutex by
// another thread as a "double lock".  This definition (interposed by the
// executable) forwards to pthread_cond_timedwait -- intercepted -- with the
// same deadline converted to CLOCK_REALTIME.
#include <pthread.h>
#include <time.h>

extern "C" int pthread_cond_clockwait(pthread_cond_t* cond, pthread_mutex_t* mutex, clockid_t clock,
                                      const struct timespec* abstime) {
  struct timespec now_c, now_r, dl;
  clock_gettime(clock, &now_c);
  clock_gettime(CLOCK_REALTIME, &now_r);
  long long rem = (long long)(abstime->tv_sec - now_c.tv_sec) * 1000000000LL + (abstime->tv_nsec - now_c.tv_nsec);
  if (rem < 0) rem = 0;
  long long ns = (long long)now_r.tv_nsec + rem % 1000000000LL;
  dl.tv_sec = now_r.tv_sec + (time_t)(rem / 1000000000LL) + (time_t)(ns / 1000000000LL);
  dl.tv_nsec = (long)(ns % 1000000000LL);
  return pthread_cond_timedwait(cond, mutex, &dl);
}
