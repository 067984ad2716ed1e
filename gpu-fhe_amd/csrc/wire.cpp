// FHEC v1 wire format: host-side encoding and validation (see wire.hpp).
#include "wire.hpp"

#include <cstring>

namespace fhe {
namespace {

constexpr uint32_t kMagic = 0x43454846u;  // "FHEC"
constexpr uint16_t kVersion = 1;
constexpr size_t kHeader = 24;

uint64_t fnv1a(const unsigned char* p, size_t n) {
  uint64_t h = 0xcbf29ce484222325ull;
  for (size_t i = 0; i < n; ++i) {
    h ^= p[i];
    h *= 0x100000001b3ull;
  }
  return h;
}

template <class T>
void put(unsigned char* p, T v) {
  std::memcpy(p, &v, sizeof(T));  // the target is little-endian (x86-64 host)
}
template <class T>
T get(const unsigned char* p) {
  T v;
  std::memcpy(&v, p, sizeof(T));
  return v;
}

}  // namespace

bool wire_size(uint32_t log_n, uint64_t polys, uint64_t nlimbs, size_t* size) {
  if (log_n > 30) return false;
  unsigned __int128 words = (unsigned __int128)polys * nlimbs << log_n;
  unsigned __int128 bytes = kHeader + 8 * (unsigned __int128)nlimbs + 8 * words + 8;
  if (bytes > (unsigned __int128)SIZE_MAX) return false;
  *size = (size_t)bytes;
  return true;
}

void wire_header(unsigned char* p, uint32_t log_n, uint32_t polys, uint32_t limb0, uint32_t nlimbs,
                 int ntt_form, const uint64_t* moduli) {
  put<uint32_t>(p, kMagic);
  put<uint16_t>(p + 4, kVersion);
  put<uint16_t>(p + 6, ntt_form ? 1 : 0);
  put<uint32_t>(p + 8, log_n);
  put<uint32_t>(p + 12, polys);
  put<uint32_t>(p + 16, limb0);
  put<uint32_t>(p + 20, nlimbs);
  for (uint32_t l = 0; l < nlimbs; ++l) put<uint64_t>(p + kHeader + 8 * (size_t)l, moduli[l]);
}

void wire_seal(unsigned char* p, size_t size) { put<uint64_t>(p + size - 8, fnv1a(p, size - 8)); }

bool wire_parse(const unsigned char* p, size_t size, uint32_t log_n, const uint64_t* moduli,
                size_t M, WireInfo& info, std::string& err) {
  if (!p || size < kHeader + 8) {
    err = "fhe_deserialize: truncated blob";
    return false;
  }
  if (get<uint32_t>(p) != kMagic || get<uint16_t>(p + 4) != kVersion) {
    err = "fhe_deserialize: not an FHEC v1 blob";
    return false;
  }
  const uint16_t flags = get<uint16_t>(p + 6);
  info.log_n = get<uint32_t>(p + 8);
  info.polys = get<uint32_t>(p + 12);
  info.limb0 = get<uint32_t>(p + 16);
  info.nlimbs = get<uint32_t>(p + 20);
  info.ntt_form = flags & 1;
  if (info.log_n != log_n) {
    err = "fhe_deserialize: blob has N = 2^" + std::to_string(info.log_n) + ", context 2^" +
          std::to_string(log_n);
    return false;
  }
  if ((uint64_t)info.limb0 + info.nlimbs > M || (flags & ~1u)) {
    err = "fhe_deserialize: limb window or flags out of range for this context";
    return false;
  }
  size_t need = 0;
  if (!wire_size(log_n, info.polys, info.nlimbs, &need) || size != need) {
    err = "fhe_deserialize: size " + std::to_string(size) + " != the size implied by the header";
    return false;
  }
  if (get<uint64_t>(p + need - 8) != fnv1a(p, need - 8)) {
    err = "fhe_deserialize: checksum mismatch (corrupted blob)";
    return false;
  }
  for (uint32_t l = 0; l < info.nlimbs; ++l)
    if (get<uint64_t>(p + kHeader + 8 * (size_t)l) != moduli[info.limb0 + l]) {
      err = "fhe_deserialize: modulus of limb " + std::to_string(info.limb0 + l) +
            " differs from the context's";
      return false;
    }
  info.body = kHeader + 8 * (size_t)info.nlimbs;
  const uint64_t n = 1ull << log_n;
  info.words = (size_t)info.polys * info.nlimbs * n;
  const unsigned char* body = p + info.body;
  for (uint64_t pl = 0; pl < (uint64_t)info.polys * info.nlimbs; ++pl) {
    const uint64_t q = moduli[info.limb0 + pl % info.nlimbs];
    const unsigned char* row = body + 8 * pl * n;
    for (uint64_t i = 0; i < n; ++i)
      if (get<uint64_t>(row + 8 * i) >= q) {
        err = "fhe_deserialize: residue out of range in poly " +
              std::to_string(pl / info.nlimbs) + ", limb " +
              std::to_string(info.limb0 + pl % info.nlimbs);
        return false;
      }
  }
  return true;
}

}  // namespace fhe
