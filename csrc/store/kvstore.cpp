// dalle_amd._kvstore -- a small native TCP key/value store that replaces the hivemind DHT + libp2p
// daemon for one node. The store, protocol, server and client live in
// kvstore_core.h (no Python dependency, sanitizer-tested); this file is the pybind11 surface. Every
// network call releases the GIL, so a WAIT parked on the server does not stall other Python threads.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "kvstore_core.h"

namespace py = pybind11;

namespace {

using dalle_kv::ClientCore;
using dalle_kv::KVServer;

class KVClient {
 public:
  KVClient(const std::string& host, int port, double connect_timeout) : c_(host, port, connect_timeout) {}
  bool store(const std::string& key, const std::string& sub, const py::bytes& val, double exp, const std::string& owner) {
    std::string v(val);
    py::gil_scoped_release nogil;
    return c_.store(key, sub, v, exp, owner);
  }
  py::list get(const std::string& key) {
    std::vector<dalle_kv::Entry> v;
    {
      py::gil_scoped_release nogil;
      v = c_.get(key);
    }
    py::list out;
    for (auto& t : v) out.append(py::make_tuple(py::bytes(std::get<0>(t)), py::bytes(std::get<1>(t)), std::get<2>(t)));
    return out;
  }
  void del(const std::string& key) {
    py::gil_scoped_release nogil;
    c_.del(key);
  }
  std::vector<std::string> keys(const std::string& prefix) {
    py::gil_scoped_release nogil;
    return c_.keys(prefix);
  }
  bool ping() {
    py::gil_scoped_release nogil;
    return c_.ping();
  }
  uint32_t wait(const std::string& key, uint32_t count, double timeout) {
    py::gil_scoped_release nogil;
    return c_.wait(key, count, timeout);
  }

 private:
  ClientCore c_;
};

}  // namespace

PYBIND11_MODULE(_kvstore, m) {
  m.doc() = "native TCP key/value store with subkeys, expiration and owner tags (DHT replacement)";
  py::class_<KVServer>(m, "KVServer")
      .def(py::init<const std::string&, int>(), py::arg("host") = "127.0.0.1", py::arg("port") = 0)
      .def_property_readonly("port", &KVServer::port)
      .def("stop", &KVServer::stop, py::call_guard<py::gil_scoped_release>());
  py::class_<KVClient>(m, "KVClient")
      .def(py::init<const std::string&, int, double>(), py::arg("host"), py::arg("port"), py::arg("connect_timeout") = 10.0)
      .def("store", &KVClient::store, py::arg("key"), py::arg("subkey"), py::arg("value"), py::arg("expiration_time"),
           py::arg("owner") = "")
      .def("get", &KVClient::get)
      .def("delete", &KVClient::del)
      .def("keys", &KVClient::keys, py::arg("prefix") = "")
      .def("ping", &KVClient::ping)
      .def("wait", &KVClient::wait, py::arg("key"), py::arg("count"), py::arg("timeout"));
  m.def("get_time", &dalle_kv::now_s);
}
