// wh_version(): library identification, tying a built binary to the sources and settings it came from.
// WH_SOURCE_SHA is the first 16 hex digits of sha256 over csrc/*.hip, *.h, *.cpp and the Makefile
// (sorted names), then include/warehouse_amd.h (the Makefile computes it; warehouse/_native.py and
// bench.py compute the same hash from the tree).  WH_VARIANT lists the build settings that did not
// come from the Makefile (e.g. EXTRA=-DWH_ABLATION), empty for the production build, so a stale or
// variant library is detected before it is trusted.
#include "warehouse_amd.h"

#ifndef WH_SOURCE_SHA
#define WH_SOURCE_SHA "unknown"
#endif
#ifndef WH_VARIANT
#define WH_VARIANT ""
#endif

#ifdef WH_CHECK
#define WH_MODE "(assert mode) "
#else
#define WH_MODE ""
#endif

// The host engine (host_engine.cpp, libwarehouse_host.so) names itself apart from the gfx950 library.
#ifdef WH_HOST_ENGINE
#define WH_LIB_NAME "warehouse_host cpu host-engine v1 "
#else
#define WH_LIB_NAME "warehouse_amd gfx950 lane-per-env v3 "
#endif

extern "C" const char* wh_version(void) {
  return sizeof(WH_VARIANT) > 1 ? WH_LIB_NAME WH_MODE "sha=" WH_SOURCE_SHA " variant=" WH_VARIANT
                                : WH_LIB_NAME WH_MODE "sha=" WH_SOURCE_SHA;
}
