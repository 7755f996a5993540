// `.svoc` checkpoint format (see svoc_io.cpp for the byte layout).
#pragma once

#include <stdint.h>

#include <string>
#include <vector>

namespace svoc {
namespace io {

enum class DType : uint8_t { U8 = 0, I8 = 1, I32 = 2, I64 = 3, F32 = 4, BF16 = 5, I128 = 6, FELT = 7 };

struct Section {
  std::string name;
  DType dtype;
  std::vector<int64_t> shape;
  std::vector<uint8_t> bytes;
};

uint32_t crc32(const uint8_t* p, size_t n, uint32_t c = 0);
size_t elem_size(DType d);
void save(const std::string& path, const std::string& meta, const std::vector<Section>& secs);
std::string load(const std::string& path, std::vector<Section>& secs);
std::vector<uint8_t> i64_to_i128(const int64_t* v, size_t n);
void i128_to_i64(const uint8_t* p, size_t n, int64_t* out);
std::vector<uint8_t> limbs_to_felt(const int64_t* v, size_t n);
void felt_to_limbs(const uint8_t* p, size_t n, int64_t* out);

}  // namespace io
}  // namespace svoc
