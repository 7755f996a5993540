// torch.ops.svoc.save_state / load_state: native .svoc checkpoint IO (csrc/engine/svoc_io.cpp).
// Tensors are copied to host; `as_types` chooses the on-disk encoding per section: "" = native,
// "i128" = int64 wsad widened to i128, "felt" = [.., 4] int64 limbs written as 32-byte felts.
#include <ATen/ATen.h>
#include <torch/library.h>

#include <cstring>

#include "../engine/svoc_io.hpp"
#include "svoc/ops.hpp"

namespace svoc {
namespace {

io::DType native_dtype(at::ScalarType t) {
  switch (t) {
    case at::kByte: return io::DType::U8;
    case at::kBool: return io::DType::U8;
    case at::kChar: return io::DType::I8;
    case at::kInt: return io::DType::I32;
    case at::kLong: return io::DType::I64;
    case at::kFloat: return io::DType::F32;
    case at::kBFloat16: return io::DType::BF16;
    default: TORCH_CHECK(false, "save_state: unsupported dtype ", t);
  }
  return io::DType::U8;
}

void save_state(const std::string& path, const std::string& meta, const std::vector<std::string>& names,
                const std::vector<at::Tensor>& tensors, const std::vector<std::string>& as_types) {
  TORCH_CHECK(names.size() == tensors.size() && as_types.size() == tensors.size(), "save_state: list sizes");
  std::vector<io::Section> secs;
  secs.reserve(tensors.size());
  for (size_t i = 0; i < tensors.size(); ++i) {
    at::Tensor t = tensors[i].detach().to(at::kCPU).contiguous();
    io::Section s;
    s.name = names[i];
    const auto& as = as_types[i];
    if (as == "i128") {
      TORCH_CHECK(t.scalar_type() == at::kLong, "i128 sections come from int64");
      s.dtype = io::DType::I128;
      s.shape = t.sizes().vec();
      s.bytes = io::i64_to_i128(t.data_ptr<int64_t>(), t.numel());
    } else if (as == "felt") {
      TORCH_CHECK(t.scalar_type() == at::kLong && t.dim() >= 1 && t.size(-1) == 4, "felt sections: [..., 4] int64");
      s.dtype = io::DType::FELT;
      s.shape = t.sizes().vec();
      s.shape.pop_back();
      s.bytes = io::limbs_to_felt(t.data_ptr<int64_t>(), t.numel() / 4);
    } else {
      if (t.scalar_type() == at::kBool) t = t.to(at::kByte);
      s.dtype = native_dtype(t.scalar_type());
      s.shape = t.sizes().vec();
      s.bytes.resize(t.numel() * t.element_size());
      std::memcpy(s.bytes.data(), t.data_ptr(), s.bytes.size());
    }
    secs.push_back(std::move(s));
  }
  io::save(path, meta, secs);
}

std::tuple<std::string, std::vector<std::string>, std::vector<at::Tensor>> load_state(const std::string& path) {
  std::vector<io::Section> secs;
  std::string meta = io::load(path, secs);
  std::vector<std::string> names;
  std::vector<at::Tensor> out;
  for (auto& s : secs) {
    names.push_back(s.name);
    if (s.dtype == io::DType::I128) {
      at::Tensor t = at::empty(s.shape, at::kLong);
      io::i128_to_i64(s.bytes.data(), t.numel(), t.data_ptr<int64_t>());
      out.push_back(t);
    } else if (s.dtype == io::DType::FELT) {
      auto shp = s.shape;
      shp.push_back(4);
      at::Tensor t = at::empty(shp, at::kLong);
      io::felt_to_limbs(s.bytes.data(), t.numel() / 4, t.data_ptr<int64_t>());
      out.push_back(t);
    } else {
      at::ScalarType st = at::kByte;
      switch (s.dtype) {
        case io::DType::U8: st = at::kByte; break;
        case io::DType::I8: st = at::kChar; break;
        case io::DType::I32: st = at::kInt; break;
        case io::DType::I64: st = at::kLong; break;
        case io::DType::F32: st = at::kFloat; break;
        case io::DType::BF16: st = at::kBFloat16; break;
        default: TORCH_CHECK(false, "load_state: bad dtype");
      }
      at::Tensor t = at::empty(s.shape, st);
      std::memcpy(t.data_ptr(), s.bytes.data(), s.bytes.size());
      out.push_back(t);
    }
  }
  return {meta, names, out};
}

}  // namespace

// device-independent (host IO): registered as catch-all kernels with the schema
void register_io_defs(torch::Library& m) {
  m.def("save_state(str path, str meta, str[] names, Tensor[] tensors, str[] as_types) -> ()", &save_state);
  m.def("load_state(str path) -> (str, str[], Tensor[])", &load_state);
}
void register_io_cpu(torch::Library&) {}

}  // namespace svoc
