// main_gpu.cc — `wtfgpu`: the batched wtf node on one MI355X.
//   wtfgpu run  --name tlv_server --target targets/tlv --lanes 4096 [--input dir] [--full-coverage]
//   wtfgpu fuzz --name tlv_server --target targets/tlv --lanes 65536 --runs N --seed 1337
// The same runner drives the oracle twin (oracle/twin_main.cc) for parity.
#include <cstdio>

#include "gpu_backend.h"
#include "runner.h"

int main(int argc, char **argv) {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  wtfgpu_host::RunnerOptions O;
  if (!wtfgpu_host::ParseRunnerArgs(argc, argv, O)) return 2;
  Options_t Opts;
  CpuState_t State;
  if (!wtfgpu_host::LoadTarget(O, Opts, State)) return 1;
  auto *B = new wtfgpu_host::GpuBackend_t();  // like g_Backend: lives for the process
  g_Backend = B;
  if (!B->Initialize(Opts, State)) {
    printf("Failed to initialize the gpu backend\n");
    return 1;
  }
  return wtfgpu_host::RunnerMain(O, *B, Opts, State);
}
