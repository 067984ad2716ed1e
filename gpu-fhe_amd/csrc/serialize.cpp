// Ciphertext / key wire format: a self-describing little-endian blob for
// any [polys][nlimbs][N] residue tensor on the device, so external callers can feed the C ABI
// from files or sockets.  Not in the reference (it has no I/O); layout:
//
//   offset  size            field
//   0       4               magic "FHEC"
//   4       2               version (1)
//   6       2               flags: bit 0 = NTT form
//   8       4               log_n
//   12      4               polys
//   16      4               limb0 (first context limb the rows use)
//   20      4               nlimbs
//   24      8 * nlimbs      the moduli of limbs limb0 .. limb0 + nlimbs - 1
//   ...     8 * P * l * N   residues, [polys][nlimbs][N], each < its limb's modulus
//   end-8   8               FNV-1a 64 of every byte before it
//
// Deserialisation checks magic, version, N, that the moduli are this context's limbs at limb0,
// the checksum and that every residue is below its modulus, before anything reaches the device.
#include <cstring>

#include "../../include/fhecore.h"
#include "internal.hpp"

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

size_t serialized_size(const fhe_ctx* c, uint32_t polys, uint32_t nlimbs) {
  return kHeader + 8 * (size_t)nlimbs + 8 * (size_t)polys * nlimbs * c->n + 8;
}

int serialize(const fhe_ctx* c, const uint64_t* dev, uint32_t polys, uint32_t limb0,
              uint32_t nlimbs, int ntt_form, void* buf, size_t size, hipStream_t s) {
  const size_t need = serialized_size(c, polys, nlimbs);
  if (!buf || size < need) {
    set_error("fhe_serialize: buffer smaller than fhe_serialized_size (" + std::to_string(need) +
              " bytes)");
    return kInvalid;
  }
  auto* p = static_cast<unsigned char*>(buf);
  put<uint32_t>(p, kMagic);
  put<uint16_t>(p + 4, kVersion);
  put<uint16_t>(p + 6, ntt_form ? 1 : 0);
  put<uint32_t>(p + 8, c->log_n);
  put<uint32_t>(p + 12, polys);
  put<uint32_t>(p + 16, limb0);
  put<uint32_t>(p + 20, nlimbs);
  for (uint32_t l = 0; l < nlimbs; ++l) put<uint64_t>(p + kHeader + 8 * l, c->moduli[limb0 + l]);
  unsigned char* body = p + kHeader + 8 * (size_t)nlimbs;
  const size_t bytes = 8 * (size_t)polys * nlimbs * c->n;
  if (bytes) {
    FHE_HIP_CHECK(hipMemcpyAsync(body, dev, bytes, hipMemcpyDeviceToHost, s));
    FHE_HIP_CHECK(hipStreamSynchronize(s));
  }
  put<uint64_t>(body + bytes, fnv1a(p, need - 8));
  return kOk;
}

int deserialize(const fhe_ctx* c, const void* buf, size_t size, uint64_t* dev, size_t dev_words,
                uint32_t* polys_out, uint32_t* limb0_out, uint32_t* nlimbs_out, int* ntt_out,
                hipStream_t s) {
  const auto* p = static_cast<const unsigned char*>(buf);
  if (!p || size < kHeader + 8) {
    set_error("fhe_deserialize: truncated blob");
    return kInvalid;
  }
  if (get<uint32_t>(p) != kMagic || get<uint16_t>(p + 4) != kVersion) {
    set_error("fhe_deserialize: not an FHEC v1 blob");
    return kInvalid;
  }
  const uint16_t flags = get<uint16_t>(p + 6);
  const uint32_t log_n = get<uint32_t>(p + 8), polys = get<uint32_t>(p + 12);
  const uint32_t limb0 = get<uint32_t>(p + 16), nlimbs = get<uint32_t>(p + 20);
  if (log_n != c->log_n) {
    set_error("fhe_deserialize: blob has N = 2^" + std::to_string(log_n) + ", context 2^" +
              std::to_string(c->log_n));
    return kInvalid;
  }
  const uint64_t M = c->moduli.size();
  if ((uint64_t)limb0 + nlimbs > M || (flags & ~1u)) {
    set_error("fhe_deserialize: limb window or flags out of range for this context");
    return kInvalid;
  }
  const size_t need = serialized_size(c, polys, nlimbs);
  if (size != need) {
    set_error("fhe_deserialize: size " + std::to_string(size) + " != " + std::to_string(need) +
              " implied by the header");
    return kInvalid;
  }
  if (get<uint64_t>(p + need - 8) != fnv1a(p, need - 8)) {
    set_error("fhe_deserialize: checksum mismatch (corrupted blob)");
    return kInvalid;
  }
  for (uint32_t l = 0; l < nlimbs; ++l)
    if (get<uint64_t>(p + kHeader + 8 * l) != c->moduli[limb0 + l]) {
      set_error("fhe_deserialize: modulus of limb " + std::to_string(limb0 + l) +
                " differs from the context's");
      return kInvalid;
    }
  const unsigned char* body = p + kHeader + 8 * (size_t)nlimbs;
  const uint64_t n = c->n;
  for (uint64_t pl = 0; pl < (uint64_t)polys * nlimbs; ++pl) {
    const uint64_t q = c->moduli[limb0 + pl % nlimbs];
    const unsigned char* row = body + 8 * pl * n;
    for (uint64_t i = 0; i < n; ++i)
      if (get<uint64_t>(row + 8 * i) >= q) {
        set_error("fhe_deserialize: residue out of range in poly " + std::to_string(pl / nlimbs) +
                  ", limb " + std::to_string(limb0 + pl % nlimbs));
        return kInvalid;
      }
  }
  const size_t words = (size_t)polys * nlimbs * n;
  if (dev && dev_words < words) {
    set_error("fhe_deserialize: device buffer holds " + std::to_string(dev_words) + " words, blob " +
              std::to_string(words));
    return kInvalid;
  }
  if (polys_out) *polys_out = polys;
  if (limb0_out) *limb0_out = limb0;
  if (nlimbs_out) *nlimbs_out = nlimbs;
  if (ntt_out) *ntt_out = flags & 1;
  if (words && dev) {
    FHE_HIP_CHECK(hipMemcpyAsync(dev, body, words * 8, hipMemcpyHostToDevice, s));
    FHE_HIP_CHECK(hipStreamSynchronize(s));
  }
  return kOk;
}

}  // namespace fhe

extern "C" {

size_t fhe_serialized_size(const fhe_ctx* c, uint32_t polys, uint32_t nlimbs) {
  return c ? fhe::serialized_size(c, polys, nlimbs) : 0;
}

int fhe_serialize(const fhe_ctx* c, const uint64_t* dev, uint32_t polys, uint32_t limb0,
                  uint32_t nlimbs, int ntt_form, void* buf, size_t size, fhe_stream_t s) {
  if (!c || (uint64_t)limb0 + nlimbs > c->moduli.size()) {
    fhe::set_error("fhe_serialize: null context or limb window out of range");
    return fhe::kInvalid;
  }
  return fhe::serialize(c, dev, polys, limb0, nlimbs, ntt_form, buf, size,
                        static_cast<hipStream_t>(s));
}

int fhe_deserialize(const fhe_ctx* c, const void* buf, size_t size, uint64_t* dev,
                    size_t dev_words, uint32_t* polys, uint32_t* limb0, uint32_t* nlimbs,
                    int* ntt_form, fhe_stream_t s) {
  if (!c) {
    fhe::set_error("fhe_deserialize: null context");
    return fhe::kInvalid;
  }
  return fhe::deserialize(c, buf, size, dev, dev_words, polys, limb0, nlimbs, ntt_form,
                          static_cast<hipStream_t>(s));
}

}  // extern "C"
