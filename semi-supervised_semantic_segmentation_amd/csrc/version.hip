#include "common.h"

extern "C" const char* ssseg_version(void) { return "ssseg 0.1.0 gfx950"; }
