// pybind11 layer over the host runtime core (csrc/runtime_core.h): BatchDispenser (the
// DistributedDataset FCFS queue, /root/reference/src/server/dataset.ts:21-67) and StalenessGate
// (bounded-staleness bookkeeping of the async parameter server).  All logic and locking lives in
// the header so that the sanitizer stress test exercises exactly the shipped code.
#include "native_runtime.h"

#include <pybind11/stl.h>

#include "runtime_core.h"

namespace py = pybind11;

namespace dfa {

static py::dict state_to_dict(const BatchDispenser& d) {
  const DispenserState s = d.state();
  py::dict out;
  out["epoch"] = s.epoch;
  out["cursor"] = s.cursor;
  out["incomplete"] = s.incomplete;
  out["perm"] = s.perm;
  out["dispatched"] = s.dispatched;
  return out;
}

static void state_from_dict(BatchDispenser& d, const py::dict& in) {
  DispenserState s;
  s.epoch = in["epoch"].cast<int>();
  s.cursor = in["cursor"].cast<int64_t>();
  s.perm = in["perm"].cast<std::vector<int64_t>>();
  s.dispatched = in["dispatched"].cast<int64_t>();
  s.incomplete = in["incomplete"].cast<std::vector<int64_t>>();
  d.load_state(s);
}

void register_runtime(py::module_& m) {
  py::class_<BatchDispenser>(m, "BatchDispenser")
      .def(py::init<int64_t, int64_t, int, bool, bool, uint64_t>(), py::arg("num_examples"), py::arg("batch_size"),
           py::arg("epochs"), py::arg("small_last_batch") = false, py::arg("shuffle") = false, py::arg("seed") = 0)
      .def("next", &BatchDispenser::next)
      .def("complete", &BatchDispenser::complete)
      .def("example_indices", &BatchDispenser::example_indices)
      .def("state", &state_to_dict)
      .def("load_state", &state_from_dict)
      .def_property_readonly("num_batches", &BatchDispenser::num_batches)
      .def_property_readonly("epoch", &BatchDispenser::epoch)
      .def_property_readonly("remaining", &BatchDispenser::remaining)
      .def_property_readonly("dispatched", &BatchDispenser::dispatched)
      .def_property_readonly("redispatch_rounds", &BatchDispenser::redispatch_rounds)
      .def_property_readonly("done", &BatchDispenser::done);
  py::class_<StalenessGate>(m, "StalenessGate")
      .def(py::init<int64_t>(), py::arg("max_staleness"))
      .def("admit", &StalenessGate::admit)
      .def("histogram", &StalenessGate::histogram)
      .def_property_readonly("accepted", &StalenessGate::accepted)
      .def_property_readonly("rejected", &StalenessGate::rejected)
      .def_property_readonly("max_staleness", &StalenessGate::max_staleness);
}

}  // namespace dfa
