// Host-side helpers shared by the extern "C" entry points (error state, launch checks).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gigapath_hip.h"

void gp_set_error(const char* fmt, ...);
void gp_clear_error();

// Returns 0 after a successful launch, or the hipError_t (recording the message).
int gp_check_launch(const char* what);

#define GP_REQUIRE(cond, ...)        \
  do {                               \
    if (!(cond)) {                   \
      gp_set_error(__VA_ARGS__);     \
      return GP_EARG;                \
    }                                \
  } while (0)

inline hipStream_t gp_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
inline bool gp_aligned(const void* p, unsigned a) { return (reinterpret_cast<uintptr_t>(p) % a) == 0; }
