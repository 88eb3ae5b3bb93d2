// Native (host C++) runtime pieces of distriflow_amd, exposed through the same _C module.
#pragma once
#include <pybind11/pybind11.h>

namespace dfa {
void register_runtime(pybind11::module_& m);
}  // namespace dfa
