// vm_internal.hpp -- the compiled program and the stack pass shared by the host trace generator (vm.cpp) and the
// device trace generator (vm_gpu.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "f128.hpp"

namespace zk {
namespace vm {

enum : uint8_t { NOOP = 0x00, PUSH = 0x10, READ = 0x11, READ2 = 0x12, ADD = 0x08, MUL = 0x09, SADD = 0x0a,
                 SMUL = 0x0c, ADD2 = 0x0b };
constexpr int CYCLE = 16, NUM_ROUNDS = 14, MAX_STACK = 16, MIN_TRACE = 16;

// the message of the last VM error on this thread (zk_vm_last_error)
extern thread_local std::string vm_err;

struct Op {
    uint8_t code, value;
};

// Program::compile (vm/src/program/mod.rs:37-131) plus the chiplet's per-step sponge states: the sponge (columns
// 7-10) absorbs (op code, op value) of every step and nothing else, so it is a function of the code alone.
struct CompiledProgram {
    std::vector<Op> code;
    std::vector<fe> sponge[4];  // state after step k (k = 0..len; k = 0 is the zero state), per lane
    fe hash[2];
    size_t chiplet_err = 0;     // 1-based step of a non-noop op on a non-round step (0: none)
    size_t trace_len = 0;       // Processor::trace length (power of two)
};

// The inputs of one run (ProgramInputs: public u8 values, secret ciphertexts of L elements) and the ServerKey scalar
struct Inputs {
    const uint8_t *pub;
    size_t npub;
    const uint8_t *sec;  // nsec * L elements, 16 B little-endian each
    size_t nsec;
    uint32_t L, delta;
};

// The stack machine's state shown at one trace row: registers top first (zero beyond depth), depth, and the read
// positions of the public and secret input tapes.  272 bytes, the layout the device generator uploads.
struct VmState {
    fe reg[MAX_STACK];
    uint32_t depth, ta, tb, pad;
};

// Processor::run's stack pass (vm/src/processor/stack.rs) without writing rows: returns ZK_OK and fills
// states[c] = the state shown at row c * stride - 1 (c = 0: the zero state; rows past the program show the final
// state) for c < nstates, and the 16 outputs -- or, on any error, the reference's status and message (vm_err), as
// zk_program_trace reports them.  The stack lives bottom first in a 16-slot array, so an op touches only the slots
// it reads or writes (PUSH one store, SMUL L multiplies) instead of shifting all sixteen.  max_depth (optional): the
// largest stack depth of the run -- a function of the code and L alone, like the whole depth column.
int stack_pass(const CompiledProgram &P, const Inputs &in, size_t stride, size_t nstates, VmState *states,
               fe *outputs, uint32_t *max_depth = nullptr);

}  // namespace vm
}  // namespace zk

// A compiled program (zk_program_compile), and its copies on the devices that generated traces from it
// (vm_gpu.hip: the code and the sponge columns, uploaded once per device and kept until zk_program_free).
struct zk_program {
    zk::vm::CompiledProgram P;
    // zk_vm_prove's preprocessed columns of this program for one (lwe_size, blowup) on one device (prover.hip
    // FixedCols): the program-only columns' coefficients and LDE, and the last row's Lagrange polynomial
    struct Fixed {
        uint32_t L, B;
        int md;  // maximum stack depth
        fe *fpolys, *flde, *lagr, *lagr_lde;
        // the LDE cosets held: r0 + j, j < ncos (a sharded rank's own block of B / G cosets; 0, B: all of them)
        int r0 = 0, ncos = 0;
    };
    struct Device {
        int device;
        zk::vm::Op *code;  // len ops
        fe *sponge;        // 4 lanes x (len + 1)
        std::vector<Fixed> fixed;
    };
    std::mutex mu;
    std::vector<std::unique_ptr<Device>> dev;  // stable addresses: a Device is used without the lock held
    ~zk_program();
};
