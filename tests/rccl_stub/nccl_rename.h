// TEST-ONLY: the RCCL entry points libghs_mst.so calls, renamed for the rccl-stub test build
// (tests/rccl_stub/libghs_mst_rcclstub.so: csrc/multi.hip compiled with -include of this header
// and linked against libnccl_stub.so), so that no process-wide librccl (torch loads one) can
// interpose the real RCCL in place of the stub.
#pragma once
#define ncclGetUniqueId stub_ncclGetUniqueId
#define ncclCommInitRank stub_ncclCommInitRank
#define ncclCommInitAll stub_ncclCommInitAll
#define ncclCommDestroy stub_ncclCommDestroy
#define ncclCommAbort stub_ncclCommAbort
#define ncclGetErrorString stub_ncclGetErrorString
#define ncclAllReduce stub_ncclAllReduce
#define ncclReduceScatter stub_ncclReduceScatter
#define ncclAllGather stub_ncclAllGather
