// dalle_amd._tokenizer -- pybind11 surface of the native unigram caption tokenizer (unigram_core.h).
// The Python side (dalle_amd/data/tokenizer.py) reads a tokenizer.json and configures a Pipeline;
// encode_batch tokenizes a whole caption batch on a few host threads with the GIL released, so the
// data-loader's preprocessing (reference data.py:24, batched tokenizer call) never serialises on Python.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <exception>
#include <thread>

#include "unigram_core.h"

namespace py = pybind11;
using dalle_tok::Pipeline;

namespace {

std::vector<std::vector<int>> encode_batch(const Pipeline& p, const std::vector<std::string>& texts, bool add_special,
                                           long max_length, bool truncation, int threads) {
  std::vector<std::vector<int>> out(texts.size());
  py::gil_scoped_release nogil;
  const int nt = std::max(1, std::min<int>(threads, int(texts.size() / 16) + 1));
  if (nt == 1) {
    for (size_t i = 0; i < texts.size(); ++i) out[i] = p.encode(texts[i], add_special, max_length, truncation);
    return out;
  }
  // an exception inside a worker (bad_alloc, a malformed model) must not std::terminate the data-loader:
  // each worker parks it, the first one is rethrown on the calling thread after the join (pybind11 then
  // raises it as a Python exception)
  std::vector<std::exception_ptr> errs(nt);
  std::vector<std::thread> pool;
  for (int t = 0; t < nt; ++t)
    pool.emplace_back([&, t] {
      try {
        for (size_t i = t; i < texts.size(); i += nt) out[i] = p.encode(texts[i], add_special, max_length, truncation);
      } catch (...) {
        errs[t] = std::current_exception();
      }
    });
  for (auto& th : pool) th.join();
  for (auto& e : errs)
    if (e) std::rethrow_exception(e);
  return out;
}

}  // namespace

PYBIND11_MODULE(_tokenizer, m) {
  m.doc() = "native SentencePiece-unigram caption tokenizer (T5TokenizerFast-compatible pipeline)";
  py::class_<Pipeline>(m, "Pipeline")
      .def(py::init<>())
      .def("add_charsmap", [](Pipeline& p, py::bytes blob) { p.add_charsmap(std::string(blob)); })
      .def("add_strip", &Pipeline::add_strip)
      .def("add_lower_ascii", &Pipeline::add_lower_ascii)
      .def("add_replace", &Pipeline::add_replace)
      .def("set_pretokenizer",
           [](Pipeline& p, bool ws, bool meta, const std::string& rep, int prepend, bool split) {
             p.pre.whitespace_split = ws;
             p.pre.metaspace = meta;
             p.pre.replacement = rep;
             p.pre.prepend = prepend;
             p.pre.split = split;
           })
      .def("set_model",
           [](Pipeline& p, const std::vector<std::pair<std::string, double>>& vocab, int unk_id, bool fuse_unk) {
             p.model = dalle_tok::Unigram(vocab, unk_id, fuse_unk);
           })
      .def("set_added", &Pipeline::set_added)
      .def("set_suffix", [](Pipeline& p, std::vector<int> ids) { p.suffix = std::move(ids); })
      .def("normalize", &Pipeline::normalize)
      .def("pretokenize",
           [](const Pipeline& p, const std::string& s) {
             std::vector<std::string> v;
             p.pretokenize(s, true, &v);
             return v;
           })
      .def("encode", &Pipeline::encode, py::arg("text"), py::arg("add_special") = false, py::arg("max_length") = -1,
           py::arg("truncation") = false, py::call_guard<py::gil_scoped_release>())
      .def("encode_batch", &encode_batch, py::arg("texts"), py::arg("add_special") = false, py::arg("max_length") = -1,
           py::arg("truncation") = false, py::arg("threads") = 4);
}
