// `.svoc` on-disk consensus-state format (survey §7.6): a header + named, typed, CRC-checked sections
// in the field order of the contract's Storage struct (contract/src/contract.cairo:80-102).
//
//   file    := magic "SVOC" u32 version(=1) u32 n_sections u32 meta_len, meta (UTF-8 JSON), section*
//   section := u32 name_len, name, u8 dtype, u8 ndim, u64 shape[ndim], u64 nbytes, u32 crc32, data
//   dtype   := 0 u8, 1 i8, 2 i32, 3 i64, 4 f32, 5 bf16, 6 i128 (little endian, sign-extended from
//              the engine's int64 wsad), 7 felt252 (32-byte big-endian, from 4 x int64 limbs)
// The writer streams each section with one fwrite; the reader validates magic, version, sizes and
// every CRC before handing bytes back (a torn or corrupted checkpoint fails loudly).
#include "svoc_io.hpp"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <memory>
#include <stdexcept>

namespace svoc {
namespace io {

namespace {

uint32_t crc_table[256];
bool crc_init = [] {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    crc_table[i] = c;
  }
  return true;
}();

struct File {
  FILE* f;
  explicit File(const std::string& p, const char* mode) : f(std::fopen(p.c_str(), mode)) {
    if (!f) throw std::runtime_error("svoc_io: cannot open " + p);
  }
  ~File() { if (f) std::fclose(f); }
  void w(const void* p, size_t n) {
    if (n && std::fwrite(p, 1, n, f) != n) throw std::runtime_error("svoc_io: short write");
  }
  void r(void* p, size_t n) {
    if (n && std::fread(p, 1, n, f) != n) throw std::runtime_error("svoc_io: truncated file");
  }
  uint64_t remaining() {   // bytes between the read position and the end of the file
    const long pos = std::ftell(f);
    struct stat st;
    if (pos < 0 || fstat(fileno(f), &st) != 0 || st.st_size < pos) throw std::runtime_error("svoc_io: cannot stat");
    return (uint64_t)(st.st_size - pos);
  }
};

// fsync of a path's parent directory (the rename itself must be durable too)
void sync_dir(const std::string& path) {
  const size_t k = path.find_last_of('/');
  const std::string dir = k == std::string::npos ? "." : (k == 0 ? "/" : path.substr(0, k));
  const int fd = ::open(dir.c_str(), O_RDONLY | O_DIRECTORY);
  if (fd < 0) return;   // best effort: some filesystems refuse directory handles
  ::fsync(fd);
  ::close(fd);
}

template <class T>
void wv(File& f, T v) { f.w(&v, sizeof(T)); }
template <class T>
T rv(File& f) { T v; f.r(&v, sizeof(T)); return v; }

}  // namespace

uint32_t crc32(const uint8_t* p, size_t n, uint32_t c) {
  c = ~c;
  for (size_t i = 0; i < n; ++i) c = crc_table[(c ^ p[i]) & 0xFF] ^ (c >> 8);
  return ~c;
}

size_t elem_size(DType d) {
  switch (d) {
    case DType::U8: case DType::I8: return 1;
    case DType::BF16: return 2;
    case DType::I32: case DType::F32: return 4;
    case DType::I64: return 8;
    case DType::I128: return 16;
    case DType::FELT: return 32;
  }
  return 0;
}

void save(const std::string& path, const std::string& meta, const std::vector<Section>& secs) {
  const std::string tmp = path + ".tmp";
  {
    File f(tmp, "wb");
    f.w("SVOC", 4);
    wv<uint32_t>(f, 1);
    wv<uint32_t>(f, (uint32_t)secs.size());
    wv<uint32_t>(f, (uint32_t)meta.size());
    f.w(meta.data(), meta.size());
    for (const auto& s : secs) {
      wv<uint32_t>(f, (uint32_t)s.name.size());
      f.w(s.name.data(), s.name.size());
      wv<uint8_t>(f, (uint8_t)s.dtype);
      wv<uint8_t>(f, (uint8_t)s.shape.size());
      for (auto d : s.shape) wv<uint64_t>(f, (uint64_t)d);
      wv<uint64_t>(f, (uint64_t)s.bytes.size());
      wv<uint32_t>(f, crc32(s.bytes.data(), s.bytes.size()));
      f.w(s.bytes.data(), s.bytes.size());
    }
    // crash safety: the data must be on disk before the rename publishes it, else a power loss can
    // leave the new name pointing at a truncated file in place of the previous good checkpoint
    if (std::fflush(f.f) != 0) throw std::runtime_error("svoc_io: flush failed");
    if (::fsync(fileno(f.f)) != 0) throw std::runtime_error("svoc_io: fsync failed");
  }
  if (std::rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("svoc_io: rename failed");
  sync_dir(path);
}

std::string load(const std::string& path, std::vector<Section>& secs) {
  File f(path, "rb");
  char magic[4];
  f.r(magic, 4);
  if (std::memcmp(magic, "SVOC", 4) != 0) throw std::runtime_error("svoc_io: bad magic");
  if (rv<uint32_t>(f) != 1) throw std::runtime_error("svoc_io: unsupported version");
  const uint32_t n = rv<uint32_t>(f);
  const uint32_t ml = rv<uint32_t>(f);
  if (ml > f.remaining()) throw std::runtime_error("svoc_io: corrupt metadata length");
  std::string meta(ml, '\0');
  f.r(&meta[0], ml);
  secs.clear();
  for (uint32_t i = 0; i < n; ++i) {
    Section s;
    const uint32_t nl = rv<uint32_t>(f);
    if (nl > 4096) throw std::runtime_error("svoc_io: corrupt section name");
    s.name.resize(nl);
    f.r(&s.name[0], nl);
    s.dtype = (DType)rv<uint8_t>(f);
    const uint8_t nd = rv<uint8_t>(f);
    const size_t es = elem_size(s.dtype);
    if (es == 0 || nd > 8) throw std::runtime_error("svoc_io: corrupt section header in " + s.name);
    uint64_t numel = 1;
    for (int k = 0; k < nd; ++k) {
      const uint64_t d = rv<uint64_t>(f);
      if (d > (uint64_t)INT64_MAX || __builtin_mul_overflow(numel, d, &numel))
        throw std::runtime_error("svoc_io: shape overflow in " + s.name);
      s.shape.push_back((int64_t)d);
    }
    uint64_t want;
    if (__builtin_mul_overflow(numel, (uint64_t)es, &want)) throw std::runtime_error("svoc_io: shape overflow in " + s.name);
    const uint64_t nb = rv<uint64_t>(f);
    if (nb != want) throw std::runtime_error("svoc_io: size mismatch in " + s.name);
    const uint32_t crc = rv<uint32_t>(f);
    // never allocate more than the file still holds (a corrupt header must fail, not exhaust memory)
    if (nb > f.remaining()) throw std::runtime_error("svoc_io: truncated file in " + s.name);
    s.bytes.resize(nb);
    f.r(s.bytes.data(), nb);
    if (crc32(s.bytes.data(), nb) != crc) throw std::runtime_error("svoc_io: CRC mismatch in " + s.name);
    secs.push_back(std::move(s));
  }
  return meta;
}

// int64 wsad -> i128 little endian (sign extension) and back (range-checked)
std::vector<uint8_t> i64_to_i128(const int64_t* v, size_t n) {
  std::vector<uint8_t> out(n * 16);
  for (size_t i = 0; i < n; ++i) {
    const int64_t hi = v[i] < 0 ? -1 : 0;
    std::memcpy(&out[i * 16], &v[i], 8);
    std::memcpy(&out[i * 16 + 8], &hi, 8);
  }
  return out;
}

void i128_to_i64(const uint8_t* p, size_t n, int64_t* out) {
  for (size_t i = 0; i < n; ++i) {
    int64_t lo, hi;
    std::memcpy(&lo, p + i * 16, 8);
    std::memcpy(&hi, p + i * 16 + 8, 8);
    if (hi != (lo < 0 ? -1 : 0)) throw std::runtime_error("svoc_io: i128 value outside the int64 engine range");
    out[i] = lo;
  }
}

// 4 x int64 little-endian limbs -> 32-byte big-endian felt, and back
std::vector<uint8_t> limbs_to_felt(const int64_t* v, size_t n) {
  std::vector<uint8_t> out(n * 32);
  for (size_t i = 0; i < n; ++i)
    for (int l = 0; l < 4; ++l) {
      const uint64_t x = (uint64_t)v[i * 4 + l];
      for (int byte = 0; byte < 8; ++byte) out[i * 32 + 31 - (l * 8 + byte)] = (uint8_t)(x >> (8 * byte));
    }
  return out;
}

void felt_to_limbs(const uint8_t* p, size_t n, int64_t* out) {
  for (size_t i = 0; i < n; ++i)
    for (int l = 0; l < 4; ++l) {
      uint64_t x = 0;
      for (int byte = 0; byte < 8; ++byte) x |= (uint64_t)p[i * 32 + 31 - (l * 8 + byte)] << (8 * byte);
      out[i * 4 + l] = (int64_t)x;
    }
}

}  // namespace io
}  // namespace svoc
