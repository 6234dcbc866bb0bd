// hs_oracle_flops.cpp -- TEST INFRASTRUCTURE ONLY: the oracle (hs_oracle.cpp) compiled with every
// `double` a counting cdbl (flopcount.h). Single-threaded use: hso_rollout on the calling thread,
// hso_flops_reset / hso_flops_read around it (tools/flop_count.py).
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "flopcount.h"

hso_flop_counts g_hso_flops;

#define HSO_FLOPCOUNT 1
#define double cdbl
#include "hs_oracle.cpp"
#undef double

extern "C" void hso_flops_reset(void) { g_hso_flops = hso_flop_counts{}; }
/* add, mul, div, sqrt, transcendental calls, comparisons, trivial operations */
extern "C" void hso_flops_read(uint64_t* out7) {
  const uint64_t* p = &g_hso_flops.add;
  for (int i = 0; i < 7; i++) out7[i] = p[i];
}
