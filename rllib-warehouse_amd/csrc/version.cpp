// wh_version(): library identification, tying a built binary to the kernel sources it came from.
// WH_SOURCE_SHA is the first 16 hex digits of sha256 over csrc/*.hip and csrc/*.h concatenated in
// sorted name order (the Makefile computes it; bench.py:source_sha and warehouse/_native.py compute
// the same hash from the tree), so a stale library is detected before it is trusted.
#include "warehouse_amd.h"

#ifndef WH_SOURCE_SHA
#define WH_SOURCE_SHA "unknown"
#endif

extern "C" const char* wh_version(void) {
#ifdef WH_CHECK
  return "warehouse_amd gfx950 lane-per-env v3 (assert mode) sha=" WH_SOURCE_SHA;
#else
  return "warehouse_amd gfx950 lane-per-env v3 sha=" WH_SOURCE_SHA;
#endif
}
