#include "engine_util.h"

static thread_local std::string g_last_error;

void csm_set_error(const std::string& msg) { g_last_error = msg; }

extern "C" const char* csm_last_error(void) { return g_last_error.c_str(); }

static inline uint16_t f32_to_bf16_rne(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7f800000u) == 0x7f800000u) return (uint16_t)((u >> 16) | ((u & 0xffffu) ? 0x40u : 0u));
  u = (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
  return (uint16_t)u;
}

std::vector<uint8_t> convert_to(const void* src, int src_dtype, size_t n, int dst_wdt) {
  std::vector<uint8_t> out(n * (dst_wdt == 0 ? 4 : 2));
  if (src_dtype == CSM_F32 && dst_wdt == 0) {
    std::memcpy(out.data(), src, n * 4);
  } else if (src_dtype == CSM_BF16 && dst_wdt == 1) {
    std::memcpy(out.data(), src, n * 2);
  } else if (src_dtype == CSM_F32 && dst_wdt == 1) {
    const float* s = static_cast<const float*>(src);
    uint16_t* d = reinterpret_cast<uint16_t*>(out.data());
    for (size_t i = 0; i < n; ++i) d[i] = f32_to_bf16_rne(s[i]);
  } else if (src_dtype == CSM_BF16 && dst_wdt == 0) {
    const uint16_t* s = static_cast<const uint16_t*>(src);
    float* d = reinterpret_cast<float*>(out.data());
    for (size_t i = 0; i < n; ++i) {
      uint32_t u = (uint32_t)s[i] << 16;
      std::memcpy(&d[i], &u, 4);
    }
  } else {
    throw CsmError(CSM_ERR_ARG, "unsupported source dtype");
  }
  return out;
}
