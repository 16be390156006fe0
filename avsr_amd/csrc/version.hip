// Library identity and the kernel-selection options of the C-ABI (include/avsr_hip.h).
#include <atomic>

#include "common.h"

extern "C" const char* avsr_version(void) { return "avsr_hip 0.2.0 gfx950"; }

namespace {
// defaults = the production choices documented in avsr_hip.h
std::atomic<int64_t> g_opt[AVSR_OPT_COUNT] = {{0}, {1}, {0}, {1}, {1}, {1}, {1}, {1}, {1}, {1}};

bool opt_valid(int option, int64_t v) {
  switch (option) {
    case AVSR_OPT_GEMM_TILE: return v >= 0 && v <= AVSR_TILE_COUNT;
    case AVSR_OPT_ATTN_SQ_BWD: return v == 0;        // retired (round 6): accepts its default only
    case AVSR_OPT_ATTN_SQ_FWD:
    case AVSR_OPT_WGRAD_DUAL:
    case AVSR_OPT_CONV_192:
    case AVSR_OPT_CONV_S2PHASE:
    case AVSR_OPT_CONV_PATCH:
    case AVSR_OPT_CONV_WPATCH:
    case AVSR_OPT_STEM_POOL_2X2:
    case AVSR_OPT_STEM_WPATCH: return v == 0 || v == 1;
    default: return false;
  }
}
}  // namespace

int64_t avsr_opt(int option) { return g_opt[option].load(std::memory_order_relaxed); }

extern "C" int avsr_set_option(int option, int64_t value) {
  if (!opt_valid(option, value)) return AVSR_E_ARG;
  g_opt[option].store(value, std::memory_order_relaxed);
  return 0;
}

extern "C" int64_t avsr_get_option(int option) {
  if (option < 0 || option >= AVSR_OPT_COUNT) return -1;
  return avsr_opt(option);
}
