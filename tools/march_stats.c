/* march_stats.c — analysis tool (not product, not oracle): the C oracle with
 * its ORC_EVENT hook recording every photon-step's outcome, so the wave-level
 * branch statistics of the march (how often a 64-lane 8x8 tile has some lane
 * terminating / scattering / all lanes null) can be measured on the bench
 * workload. Build: gcc -O2 -shared -fPIC -ffp-contract=off tools/march_stats.c
 *   -Ioracle -o /tmp/stats/liboracle.so -lm -lpthread */
#include <stdint.h>
uint8_t* g_ev = 0;
uint32_t g_ev_R = 0, g_ev_S = 0;
#define ORC_EVENT(x, y, step, kind) \
  (g_ev ? (void)(g_ev[(((size_t)(y) * g_ev_R + (x)) * g_ev_S) + (step)] = (uint8_t)(kind)) : (void)0)
#include "../oracle/mcm_oracle.c"
void stats_set_buffer(uint8_t* ev, uint32_t R, uint32_t S) { g_ev = ev; g_ev_R = R; g_ev_S = S; }
