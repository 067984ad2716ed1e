// Ciphertext / key wire format: a self-describing little-endian blob for
// any [polys][nlimbs][N] residue tensor on the device, so external callers can feed the C ABI
// from files or sockets.  Not in the reference (it has no I/O).  Encoding and validation live in
// wire.cpp (host only); this file adds the device copies.  Layout:
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
#include "../../include/fhecore.h"
#include "internal.hpp"
#include "wire.hpp"

namespace fhe {

size_t serialized_size(const fhe_ctx* c, uint32_t polys, uint32_t nlimbs) {
  size_t size = 0;
  return wire_size(c->log_n, polys, nlimbs, &size) ? size : 0;
}

int serialize(const fhe_ctx* c, const uint64_t* dev, uint32_t polys, uint32_t limb0,
              uint32_t nlimbs, int ntt_form, void* buf, size_t size, hipStream_t s) {
  const size_t need = serialized_size(c, polys, nlimbs);
  if (!buf || need == 0 || size < need) {
    set_error("fhe_serialize: buffer smaller than fhe_serialized_size (" + std::to_string(need) +
              " bytes)");
    return kInvalid;
  }
  auto* p = static_cast<unsigned char*>(buf);
  wire_header(p, c->log_n, polys, limb0, nlimbs, ntt_form, c->moduli.data() + limb0);
  const size_t bytes = 8 * (size_t)polys * nlimbs * c->n;
  if (bytes) {
    FHE_HIP_CHECK(hipMemcpyAsync(p + need - 8 - bytes, dev, bytes, hipMemcpyDeviceToHost, s));
    FHE_HIP_CHECK(hipStreamSynchronize(s));
  }
  wire_seal(p, need);
  return kOk;
}

int deserialize(const fhe_ctx* c, const void* buf, size_t size, uint64_t* dev, size_t dev_words,
                uint32_t* polys_out, uint32_t* limb0_out, uint32_t* nlimbs_out, int* ntt_out,
                hipStream_t s) {
  const auto* p = static_cast<const unsigned char*>(buf);
  WireInfo info{};
  std::string err;
  if (!wire_parse(p, size, c->log_n, c->moduli.data(), c->moduli.size(), info, err)) {
    set_error(err);
    return kInvalid;
  }
  if (dev && dev_words < info.words) {
    set_error("fhe_deserialize: device buffer holds " + std::to_string(dev_words) + " words, blob " +
              std::to_string(info.words));
    return kInvalid;
  }
  if (polys_out) *polys_out = info.polys;
  if (limb0_out) *limb0_out = info.limb0;
  if (nlimbs_out) *nlimbs_out = info.nlimbs;
  if (ntt_out) *ntt_out = info.ntt_form;
  if (info.words && dev) {
    FHE_HIP_CHECK(hipMemcpyAsync(dev, p + info.body, info.words * 8, hipMemcpyHostToDevice, s));
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
