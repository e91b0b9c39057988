// Debug-only A/B overrides of measured, fixed choices, read from PLLM_AB="key=value,..." (the keys and their
// records: pretraining_llm_amd/ab.py).  Host code only.
#pragma once
#include <cstdlib>
#include <cstring>

namespace pllm {

inline int ab_int(const char* key, int dflt) {
  const char* e = std::getenv("PLLM_AB");
  if (e == nullptr) return dflt;
  const size_t kl = std::strlen(key);
  for (const char* p = e; *p != '\0';) {
    while (*p == ' ' || *p == ',') ++p;
    if (std::strncmp(p, key, kl) == 0 && p[kl] == '=') return std::atoi(p + kl + 1);
    while (*p != '\0' && *p != ',') ++p;
  }
  return dflt;
}

}  // namespace pllm
