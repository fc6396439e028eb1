// Extension module entry: `distributed_pytorch_example_amd._C`.
#include <torch/extension.h>

#include "../comm/comm.h"

void register_ops(pybind11::module& m);
namespace dpe_gemm {
void register_gemm(pybind11::module& m);
}

PYBIND11_MODULE(_C, m) {
  m.doc() = "MI355X (gfx950) kernels, RCCL communicator and DDP reducer";
  m.attr("ARCH") = "gfx950";
  register_ops(m);
  dpe_gemm::register_gemm(m);
  dpe::register_comm(m);
}
