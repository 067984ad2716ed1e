// FHEC v1 wire format: encoding and validation on host buffers (plain
// C++17, no HIP).  serialize.cpp adds the device copies; tests/cpp/host_sanitize.cpp fuzzes the
// parser under ASan/UBSan.  Layout (little-endian):
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
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <string>

namespace fhe {

struct WireInfo {
  uint32_t log_n, polys, limb0, nlimbs;
  int ntt_form;
  size_t body;   // byte offset of the residues
  size_t words;  // residues in the body
};

// Bytes of a blob with these dimensions; false if the size does not fit a size_t.
bool wire_size(uint32_t log_n, uint64_t polys, uint64_t nlimbs, size_t* size);
// Header + moduli into p (>= wire_size bytes); the caller fills the body, then wire_seal.
void wire_header(unsigned char* p, uint32_t log_n, uint32_t polys, uint32_t limb0, uint32_t nlimbs,
                 int ntt_form, const uint64_t* moduli);
void wire_seal(unsigned char* p, size_t size);
// Every check short of the device copy: magic, version, flags, N, limb window against the
// context's M moduli, exact size, checksum, moduli, residue ranges.
bool wire_parse(const unsigned char* p, size_t size, uint32_t log_n, const uint64_t* moduli,
                size_t M, WireInfo& info, std::string& err);

}  // namespace fhe
