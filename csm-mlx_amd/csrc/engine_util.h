// Host-side error plumbing and dtype conversion shared by the CSM engine and the Mimi codec.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/csm_hip.h"

struct CsmError : std::runtime_error {
  int code;
  CsmError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

void csm_set_error(const std::string& msg);

#define HIPCHK(expr)                                                                              \
  do {                                                                                            \
    hipError_t _e = (expr);                                                                       \
    if (_e != hipSuccess)                                                                         \
      throw CsmError(CSM_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));            \
  } while (0)

#define CSM_TRY try
#define CSM_CATCH                                                   \
  catch (const CsmError& ex) {                                      \
    csm_set_error(ex.what());                                       \
    return ex.code;                                                 \
  }                                                                 \
  catch (const std::exception& ex) {                                \
    csm_set_error(ex.what());                                       \
    return CSM_ERR_HIP;                                             \
  }                                                                 \
  return CSM_OK;

// Convert n host elements of src_dtype (CSM_F32 / CSM_BF16) to the storage dtype (0 f32, 1 bf16).
std::vector<uint8_t> convert_to(const void* src, int src_dtype, size_t n, int dst_wdt);
