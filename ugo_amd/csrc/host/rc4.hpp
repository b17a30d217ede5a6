// rc4.hpp -- RC4 keystream (KSA + PRGA), host side.  ugo's rc4StreamCrypto
// (ugo/crypto.go:25-39) creates a fresh crypto/rc4 cipher per packet from a
// fixed key, so every packet is XORed with the same keystream prefix; the RX
// assembly kernel takes that prefix as a device "pad".
#pragma once
#include <cstddef>
#include <cstdint>

namespace ugo {

inline void rc4_keystream(const uint8_t* key, size_t key_len, uint8_t* out, size_t n) {
  uint8_t S[256];
  for (int i = 0; i < 256; ++i) S[i] = static_cast<uint8_t>(i);
  uint8_t j = 0;
  for (int i = 0; i < 256; ++i) {
    j = static_cast<uint8_t>(j + S[i] + key[i % key_len]);
    const uint8_t t = S[i];
    S[i] = S[j];
    S[j] = t;
  }
  uint8_t i8 = 0;
  j = 0;
  for (size_t k = 0; k < n; ++k) {
    i8 = static_cast<uint8_t>(i8 + 1);
    j = static_cast<uint8_t>(j + S[i8]);
    const uint8_t t = S[i8];
    S[i8] = S[j];
    S[j] = t;
    out[k] = S[static_cast<uint8_t>(S[i8] + S[j])];
  }
}

}  // namespace ugo
