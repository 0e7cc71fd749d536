// pybind11 module xotorch_support_jetson_amd._runtime: the native block manager (block_manager.h).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "block_manager.h"

namespace py = pybind11;

namespace {
void fill_batch_np(const xot_rt::BlockManager& bm, const std::vector<std::string>& rids,
                   py::array_t<int32_t, py::array::c_style> tables, py::array_t<int32_t, py::array::c_style> ctx_lens) {
  auto tb = tables.mutable_unchecked<2>();
  auto cl = ctx_lens.mutable_unchecked<1>();
  bm.fill_batch(rids, tables.mutable_data(), tb.shape(0), tb.shape(1), ctx_lens.mutable_data(), cl.shape(0));
}
}  // namespace


PYBIND11_MODULE(_runtime, m) {
  m.doc() = "xot native host runtime (paged KV block manager)";
  py::class_<xot_rt::BlockManager>(m, "BlockManager")
      .def(py::init<int64_t, int64_t>(), py::arg("num_blocks"), py::arg("block_size") = 64)
      .def_property_readonly("block_size", &xot_rt::BlockManager::block_size)
      .def_property_readonly("num_blocks", &xot_rt::BlockManager::num_blocks)
      .def_property_readonly("num_free", &xot_rt::BlockManager::num_free)
      .def_property_readonly("num_sequences", &xot_rt::BlockManager::num_sequences)
      .def("has", &xot_rt::BlockManager::has)
      .def("num_tokens", &xot_rt::BlockManager::num_tokens)
      .def("blocks_needed", &xot_rt::BlockManager::blocks_needed)
      .def("can_append", &xot_rt::BlockManager::can_append)
      .def("append", &xot_rt::BlockManager::append)
      .def("truncate", &xot_rt::BlockManager::truncate)
      .def("free", &xot_rt::BlockManager::free_seq)
      .def("fork", &xot_rt::BlockManager::fork)
      .def("block_table", &xot_rt::BlockManager::block_table)
      .def("fill_batch", &fill_batch_np)
      .def("check", &xot_rt::BlockManager::check);
}
