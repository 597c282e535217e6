// rmx_build_info.cpp — rmx_build_info() (include/rmx.h): the SHA-256 digests of the engine sources this library
// was built from and of the fast kernels' code object.  build/build_info.h is written by the Makefile from the
// RMX_HASHED files and build/rmx_fast.co, so this object is rebuilt whenever any of them changes.
#include "../../include/rmx.h"
#include "build/build_info.h"

#define RMX_STR2(x) #x
#define RMX_STR(x) RMX_STR2(x)

extern "C" const char* rmx_build_info(void) {
  return "src=" RMX_SOURCE_HASH " kern=" RMX_KERNEL_HASH " abi=" RMX_STR(RMX_ABI_VERSION) " arch=" RMX_OFFLOAD_ARCH;
}
