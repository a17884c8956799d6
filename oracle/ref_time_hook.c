/* Test infrastructure (oracle/_ref only): replaces gettimeofday() inside the reference
 * ctree build via -Wl,--wrap=gettimeofday, so that srand(tv.tv_usec) at
 * lzero/mcts/ctree/common_lib/utils.cpp:25 takes a seed chosen by the golden-vector
 * generator instead of the wall clock. Not linked into anything that ships. */
#include <sys/time.h>
static long g_usec = 0;
static long g_calls = 0;
void oracle_set_usec(long usec) { g_usec = usec; }
long oracle_get_calls(void) { return g_calls; }
int __wrap_gettimeofday(struct timeval *tv, void *tz) {
  (void)tz;
  g_calls++;
  if (tv) { tv->tv_sec = 0; tv->tv_usec = g_usec; }
  return 0;
}
