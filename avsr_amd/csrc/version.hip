// Library identity for the C-ABI (include/avsr_hip.h).
#include "common.h"
extern "C" const char* avsr_version(void) { return "avsr_hip 0.1.0 gfx950"; }
