// main_gpu.cc — `wtfgpu`: the batched wtf node on one MI355X.
//   wtfgpu run  --name tlv_server --target targets/tlv --lanes 4096 [--input dir] [--full-coverage]
//   wtfgpu fuzz --name tlv_server --target targets/tlv --lanes 65536 --runs N --seed 1337
//   wtfgpu fuzz ... --device r --rank r --world n --nccl-id-file /tmp/id   (one process per GPU:
//       shard r mutates with seed + r; coverage maps merged with RCCL MAX after every batch)
//   wtfgpu fuzz ... --rccl-force   (world 1 through the same RCCL merge: a one-rank communicator)
//   wtfgpu master --name tlv_server --target targets/tlv --address tcp://127.0.0.1:31337 --nodes 8 --batched
//   wtfgpu fuzz --name tlv_server --target targets/tlv --lanes 65536 --address tcp://127.0.0.1:31337 --batched
//       (a master process and one node per GPU over the wire protocol, remote.h / wire.h)
// The same runner drives the oracle twin (oracle/twin_backend.cc) for parity.
#include <cstdio>
#include <memory>

#include "gpu_backend.h"
#include "rccl_exchange.h"
#include "remote.h"
#include "runner.h"

int main(int argc, char **argv) {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  wtfgpu_host::RunnerOptions O;
  if (!wtfgpu_host::ParseRunnerArgs(argc, argv, O)) return 2;
  if (O.mode == "master") return wtfgpu_host::MasterMain(O);  // no GPU: corpus + mutator + nodes
  Options_t Opts;
  CpuState_t State;
  if (!wtfgpu_host::LoadTarget(O, Opts, State)) return 1;
  auto *B = new wtfgpu_host::GpuBackend_t();  // like g_Backend: lives for the process
  g_Backend = B;
  if (!B->Initialize(Opts, State)) {
    printf("Failed to initialize the gpu backend\n");
    return 1;
  }
  if (O.regroup != ~0ull) wtfgpu_set_regroup(B->Engine(), O.regroup);
  std::unique_ptr<wtfgpu_host::RcclExchange_t> X;
  if (O.world > 1 || O.rccl_force) {
    uint8_t Id[wtfgpu_host::kRcclIdBytes];
    const bool got = O.world == 1 && O.nccl_id_file.empty()
                         ? wtfgpu_host::RcclUniqueId(Id)  // forced at world 1: this process is the only rank
                         : !O.nccl_id_file.empty() && wtfgpu_host::RcclIdViaFile(O.nccl_id_file, O.rank, Id);
    if (!got) {
      printf("--world > 1 needs --nccl-id-file (rank 0 writes the RCCL id there)\n");
      return 1;
    }
    X = std::make_unique<wtfgpu_host::RcclExchange_t>(O.rank, O.world, O.rccl_force);
    if (!X->Init(Id, wtfgpu_stream(B->Engine()))) return 1;
  }
  return wtfgpu_host::RunnerMain(O, *B, Opts, State, X.get());
}
