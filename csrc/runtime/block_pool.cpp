// Native runtime pieces of the serving stack (host side, no GPU):
//   * BlockPool    - paged-KV block allocator with ref counts, prefix-cache hash map and an LRU
//                    eviction queue of zero-ref blocks (the worker's KV block manager).
//   * block_hashes - chained 64-bit hashes of full 16-token blocks; the frontend router and the
//                    workers compute byte-identical hashes so KV events line up.
//   * KvIndexer    - router-side index block-hash -> set of workers holding it, answering
//                    "longest cached prefix per worker" for KV-aware routing.
//   * ShmRing      - /dev/shm ring that carries each step's inputs from TP rank 0 to the other
//                    ranks (shm_ring.cpp).
// Upstream Dynamo keeps these in Rust (dynamo-llm kv_router indexer) and vLLM keeps the block pool
// in Python; SURVEY.md §2.3 N05 and §7.4 item 7 size them for ~0.5 M blocks x 8 workers, which is
// why they are C++ here.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "kv_runtime.h"

namespace py = pybind11;
namespace mxs_rt {
void register_shm_ring(py::module_& m);  // shm_ring.cpp
}
using mxs_rt::BlockPool;
using mxs_rt::KvIndexer;

PYBIND11_MODULE(_rt, m) {
  m.doc() = "mxserve native host runtime: block pool, block hashing, KV indexer, shared-memory ring";
  mxs_rt::register_shm_ring(m);
  m.def("block_hashes", &mxs_rt::block_hashes, py::arg("tokens"), py::arg("block_size"), py::arg("extra") = 0,
        py::arg("parent") = 0, "Chained hashes of the full blocks of `tokens`.");
  py::class_<BlockPool>(m, "BlockPool")
      .def(py::init<int, bool>(), py::arg("num_blocks"), py::arg("prefix_caching") = true)
      .def_property_readonly("num_blocks", &BlockPool::num_blocks)
      .def("num_free", &BlockPool::num_free)
      .def("usage", &BlockPool::usage)
      .def("num_cached", &BlockPool::num_cached)
      .def("allocate", &BlockPool::allocate)
      .def("free", &BlockPool::free)
      .def("get_cached_prefix", &BlockPool::get_cached_prefix)
      .def("count_cached_prefix", &BlockPool::count_cached_prefix)
      .def("cache_blocks", &BlockPool::cache_blocks)
      .def("reset_prefix_cache", &BlockPool::reset_prefix_cache)
      .def("take_events", [](BlockPool& p) { auto e = p.take_events(); return py::make_tuple(e.first, e.second); })
      .def("hit_rate", &BlockPool::hit_rate)
      .def("ref_count", &BlockPool::ref_count)
      .def("check_invariants", &BlockPool::check_invariants);
  py::class_<KvIndexer>(m, "KvIndexer")
      .def(py::init<>())
      .def("apply_stored", &KvIndexer::apply_stored)
      .def("apply_removed", &KvIndexer::apply_removed)
      .def("remove_worker", &KvIndexer::remove_worker)
      .def("find_matches", &KvIndexer::find_matches)
      .def("num_blocks", &KvIndexer::num_blocks)
      .def("size", &KvIndexer::size);
}
