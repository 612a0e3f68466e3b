// Host side of the batched STARK verifier: AIR descriptor parsing/levelization, BFieldCodec
// proof-stream decoding into ProofDesc offsets, the per-proof Fiat-Shamir program, device
// staging, and the C ABI (include/neptune_hip.h: nhip_air_*, nhip_batch_*, nhip_verify_batch).
//
// Decoding restates triton-vm 1.0's `ProofStream::try_from(&Proof)` + the dequeue order of
// `Stark::verify` (parity unpinned beyond the Claim layout, which is pinned by
// neptune-core/src/protocol/consensus/transaction/validity/tasm/claims/new_claim.rs:38-100).
// Any structural error gives verdict 0 (triton_vm::verify returns false on every Err), never an
// infrastructure error: the reference's reject tests (verifier.rs:95-118 bogus proof,
// neptune_proof.rs:118-133 empty / all-zero proofs) must come out as `false`.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <system_error>
#include <thread>
#include <vector>

#include "../../include/neptune_hip.h"
#include "device_scope.hpp"
#include "host_copy.hpp"
#include "host_numa.hpp"
#include "../../include/nhip_challenge_id.h"
#include "goldilocks.hpp"
#include "kernels.hpp"
#include "stark.hpp"

using namespace nhip;

namespace {

constexpr size_t OUT_HDR = CNT_N * 8;  // pinned readback: [device counters | plan counters | verdicts]
// hash levels launched before the OOD / FRI / DEEP chain is released (NHIP_AUX_AFTER_LEVEL
// overrides); tuned on MI355X
constexpr uint32_t AUX_AFTER_LEVEL_DEFAULT = 0;

// What the host knows of a batch: its layout in the device word buffer and the scratch sizes,
// from the proof lengths and the padded height each proof header declares.  Everything else (the
// proof-stream walk, descriptors, Fiat-Shamir programs, decode failures) is k_decode's, every run.
struct HostBatch {
    Dims D{};
    uint32_t n = 0;
    uint64_t proof_words = 0;   // proof region [0, proof_words) of the word buffer
    uint64_t words_total = 0;   // + the staged claim encodings
    uint32_t max_R = 0, max_last_cw = 1, levels = 0;
    uint32_t fs_stride = 0, xs_stride = 0;
    uint64_t perms_static = 0, perms_lcw = 0;  // device-counted, per run
};

uint64_t claim_words(const nhip_claim& c) { return (uint64_t)c.output_len + c.input_len + 10; }

// The claim's BFieldCodec encoding (pinned layout, new_claim.rs:38-100):
// [out_n + 1, out_n, out.., in_n + 1, in_n, in.., version, digest(5)], staged in the batch's input
// form (the kernels read the claim and the proof words alike): the caller's field elements reduced
// mod p in their own form, the lengths and the version (plain integers) converted into it.
void encode_claim(const nhip_claim& claim, bool mont, uint64_t* c) {
    auto len = [&](uint64_t v) { return mont ? to_mont(v) : v; };
    *c++ = len(claim.output_len + 1);
    *c++ = len(claim.output_len);
    for (size_t i = 0; i < claim.output_len; ++i) *c++ = canon(claim.output[i]);
    *c++ = len(claim.input_len + 1);
    *c++ = len(claim.input_len);
    for (size_t i = 0; i < claim.input_len; ++i) *c++ = canon(claim.input[i]);
    *c++ = len(claim.version);
    for (int i = 0; i < 5; ++i) *c++ = canon(claim.program_digest[i]);
}

// The staging copy of a proof (pageable caller memory -> pinned staging) with non-temporal
// stores: the staging is written once and read only by the DMA engine, so ordinary stores would
// first read every destination line into the cache (a read-for-ownership) and then evict it: one
// more host-DRAM pass per proof byte.  The feed path's host bandwidth is what an 8-GPU node runs
// out of first, so the copy streams: 8-byte head to 16-byte alignment, 64-byte
// blocks of four 16-byte streaming stores, then the tail.  The caller fences (_mm_sfence) before
// the DMA of the chunk is issued.  NHIP_STAGE_NT=0: plain memcpy (A/B).
static bool stage_nt() {
    static const bool on = [] {
        const char* v = nhip::ab_env("NHIP_STAGE_NT");
        return !v || std::strtol(v, nullptr, 10) != 0;
    }();
    return on;
}
// Host threads for staging copies (at most 16, the GPU box's CPU share).
unsigned host_threads(uint64_t bytes) {
    unsigned t = nhip::host_threads_env() ? nhip::host_threads_env() : std::thread::hardware_concurrency();
    t = std::max(1u, std::min(t, 16u));
    return bytes < (8ull << 20) ? 1u : t;
}

// Pinned host ranges handed out by nhip_host_alloc / registered by nhip_host_register: proofs that
// live in one are DMA'd to the device straight from the caller's memory (no staging copy).
struct PinnedRanges {
    std::mutex mu;
    std::vector<std::pair<uintptr_t, size_t>> r;  // (start, bytes)
    bool contains(const void* p, size_t bytes) {
        const uintptr_t a = (uintptr_t)p;
        std::lock_guard<std::mutex> g(mu);
        for (const auto& x : r)
            if (a >= x.first && a + bytes <= x.first + x.second && a + bytes >= a) return true;
        return false;
    }
};
PinnedRanges& pinned() {
    static PinnedRanges p;
    return p;
}

}  // namespace

// ====================================================================== AIR object
// One compiled OOD program (air_compile): instructions, step offsets, constant table, slot count.
struct OodProgram {
    std::vector<OodIns> prog;
    std::vector<uint32_t> prog_off;
    std::vector<Xfe> consts;
    uint32_t slots = 0;
    uint32_t width = 0;
};

struct nhip_air {
    StarkDims dims_air{};  // num_main, num_aux, num_sampled, num_constraints filled
    std::vector<AirNode> nodes;
    std::vector<uint32_t> level_off;  // node-level histogram (nhip_air_info)
    uint4 cons_off{};
    // compiled programs (see OodIns in stark.hpp, air_compile): [0] narrow steps (fewer live values:
    // more proofs per CU, for batches that fill the GPU), [1] wide steps (fewer barriers: lower
    // latency per proof, for smaller batches); a batch takes one by its size (ood_program_for)
    OodProgram progs[2];
    // slots held in LDS (the rest in the per-proof global area): AIR_LDS_SLOTS_MAX, or less when
    // nhip_air_options.lds_slots asks for it at creation (tests of the global-slot path)
    uint32_t lds_cap = AIR_LDS_SLOTS_MAX;
    // device copies, one per GPU that has used this AIR (read-only, so every context on that GPU
    // shares it; a group drives several contexts from one process, possibly concurrently);
    // created on first use, freed with the AIR
    struct Dev {
        int device;
        OodIns* d_prog[2];
        uint32_t* d_prog_off[2];
        Xfe* d_consts[2];
    };
    std::mutex mu;
    std::vector<Dev> devs;
};

// Device memory, streams, events and pinned readback of nhip_verify_batch, kept in the context
// and reused call after call: a one-proof call is otherwise dominated by hipMalloc / stream /
// event / pinned-buffer setup and teardown (~10 ms against ~2 ms of device work).  `mu` holds
// the scratch for a whole call, so concurrent callers are serialized.
struct VerifyScratch {
    std::mutex mu;
    void* dmem = nullptr;
    size_t dmem_bytes = 0;
    void* dwords = nullptr;  // proof words (uploaded while they are decoded)
    size_t dwords_bytes = 0;
    hipStream_t main = nullptr, aux = nullptr;
    hipEvent_t ev[STARK_EVENTS] = {};
    bool streams = false;
    uint8_t* h_out = nullptr;
    size_t h_out_bytes = 0;
};

static void free_verify_scratch(void* p) {
    auto* sc = (VerifyScratch*)p;
    if (sc->streams) {
        (void)hipStreamSynchronize(sc->main);
        (void)hipStreamSynchronize(sc->aux);
        for (int i = 0; i < STARK_EVENTS; ++i) (void)hipEventDestroy(sc->ev[i]);
        (void)hipStreamDestroy(sc->main);
        (void)hipStreamDestroy(sc->aux);
    }
    if (sc->h_out) (void)hipHostFree(sc->h_out);
    if (sc->dmem) (void)hipFree(sc->dmem);
    if (sc->dwords) (void)hipFree(sc->dwords);
    delete sc;
}

struct nhip_batch {
    HostBatch H;
    VerifyScratch* scratch = nullptr;  // borrowed resources (nhip_verify_batch), not owned
    const nhip_air* air = nullptr;
    int device = 0;
    // device buffers
    void* dmem = nullptr;
    StarkBatchDev dev{};
    StarkPhaseTimer tm{};
    hipStream_t main = nullptr;  // hashing chain (rows -> Merkle levels -> roots -> verdicts)
    hipStream_t aux = nullptr;   // latency-bound chain (Fiat-Shamir -> plan -> OOD -> FRI -> DEEP)
    uint8_t* h_out = nullptr;    // pinned: [device counters | plan counters | verdicts (n B)]
    size_t dmem_bytes = 0, h_out_bytes = 0;  // owned allocations (refill reuses them when they fit)
    void* dwords = nullptr;                  // proof words (owned unless borrowed from the scratch)
    size_t dwords_bytes = 0;
    bool timed = false, in_flight = false;
    struct {
        double decode, fs, rows, plan, hash, roots, ood, fri, deep, total;
    } ph{};
    double stage_ms = 0, upload_ms = 0;
    // The batch's launch sequence captured into a HIP graph (nhip_batch_set_graph): replayed by every
    // untimed launch while the contents and streams are unchanged, captured again at the next launch
    // after a refill or a stream change.  The capture records its own fork / join events (gev): an
    // event once captured into a graph cannot be recorded on a stream again.
    hipGraphExec_t gexec = nullptr;
    bool graph_on = false;
    bool last_graph = false;  // the last launch replayed the graph (no phase timestamps)
    hipEvent_t gev[STARK_EVENTS] = {};
    double mp_hash_exec_ms = 0;  // summed dispatch durations of the hash launches
    double row_hash_exec_ms = 0;  // the row-hashing launch's dispatch duration
    uint64_t merkle_perms = 0;
    std::vector<uint64_t> mp_cap;  // multiproof op capacity per level
};

// ctx internals live in capi.hip; access the stream / device via these helpers
extern "C" hipStream_t nhip_internal_stream(nhip_ctx* c);
extern "C" int nhip_internal_device(nhip_ctx* c);
extern "C" std::mutex* nhip_internal_mutex(nhip_ctx* c);
extern "C" void* nhip_internal_staging(nhip_ctx* c, size_t bytes);
extern "C" void* nhip_internal_verify_scratch(nhip_ctx* c, void* (*make)(), void (*freefn)(void*));
extern "C" const void* nhip_internal_topo(nhip_ctx* c);
extern "C" unsigned nhip_internal_host_threads(nhip_ctx* c);
static const nhip::HostTopo& ctx_topo(nhip_ctx* c) { return *(const nhip::HostTopo*)nhip_internal_topo(c); }

namespace {

int hipfail(hipError_t e) { return e == hipSuccess ? NHIP_OK : (e == hipErrorOutOfMemory ? NHIP_ERR_OOM : NHIP_ERR_HIP); }

bool dims_from(const nhip_stark_params* sp, const nhip_air* air, Dims& D) {
    if (!sp || !air) return false;
    if (sp->num_collinearity_checks < 1 || sp->num_collinearity_checks > (uint32_t)MAX_CHECKS) return false;
    if (sp->log2_fri_expansion < 1 || sp->log2_fri_expansion > 8) return false;
    if (sp->num_main != air->dims_air.num_main || sp->num_aux != air->dims_air.num_aux) return false;
    if (sp->num_quotient_segments < 1 || sp->num_quotient_segments > 64) return false;
    if (sp->input_form != NHIP_INPUT_CANONICAL && sp->input_form != NHIP_INPUT_MONTGOMERY) return false;
    // DEEP kernel: carry-free accumulators (M + 3A row words, DEEP_ROW_WORDS_MAX), weights in LDS
    if (sp->num_main + 3ull * sp->num_aux >= DEEP_ROW_WORDS_MAX) return false;
    StarkDims& d = D.d;
    d.num_main = sp->num_main;
    d.num_aux = sp->num_aux;
    d.num_quot_seg = sp->num_quotient_segments;
    d.num_checks = sp->num_collinearity_checks;
    d.num_deep = 3;
    d.log2_expansion = sp->log2_fri_expansion;
    d.num_trace_randomizers = sp->num_collinearity_checks + 2 * 3;
    d.num_sampled = air->dims_air.num_sampled;
    d.num_constraints = air->dims_air.num_constraints;
    D.expansion = 1u << sp->log2_fri_expansion;
    D.mont_words = sp->input_form == NHIP_INPUT_MONTGOMERY ? 1u : 0u;
    if (deep_rows8_lds_bytes(d) > 160 * 1024 - 8192) return false;
    // the last FRI codeword has at most 2^(floor(log2 k) + 1 + log2 expansion) XFEs; bound its
    // Merkle-tree scratch (n x max_len digests)
    if ((1ull << (log2_u64(d.num_checks) + 1 + d.log2_expansion)) > 4096) return false;
    return true;
}

// The device copy of the compiled AIR on this context's GPU (uploaded on first use).
int air_upload(nhip_ctx* ctx, nhip_air* a, nhip_air::Dev* out) {
    std::lock_guard<std::mutex> g(a->mu);
    const int device = nhip_internal_device(ctx);
    for (const auto& d : a->devs)
        if (d.device == device) {
            *out = d;
            return NHIP_OK;
        }
    nhip_air::Dev d{device, {nullptr, nullptr}, {nullptr, nullptr}, {nullptr, nullptr}};
    auto free_dev = [&]() {
        for (int k = 0; k < 2; ++k) {
            if (d.d_prog[k]) (void)hipFree(d.d_prog[k]);
            if (d.d_prog_off[k]) (void)hipFree(d.d_prog_off[k]);
            if (d.d_consts[k]) (void)hipFree(d.d_consts[k]);
        }
    };
    hipError_t e = hipSuccess;
    for (int k = 0; k < 2 && e == hipSuccess; ++k) {
        const OodProgram& pg = a->progs[k];
        e = hipMalloc(&d.d_prog[k], pg.prog.size() * sizeof(OodIns) + 16);
        if (e == hipSuccess) e = hipMalloc(&d.d_prog_off[k], pg.prog_off.size() * 4 + 4);
        if (e == hipSuccess) e = hipMalloc(&d.d_consts[k], pg.consts.size() * sizeof(Xfe) + 24);
        if (e == hipSuccess && !pg.prog.empty())
            e = hipMemcpy(d.d_prog[k], pg.prog.data(), pg.prog.size() * sizeof(OodIns), hipMemcpyHostToDevice);
        if (e == hipSuccess)
            e = hipMemcpy(d.d_prog_off[k], pg.prog_off.data(), pg.prog_off.size() * 4, hipMemcpyHostToDevice);
        if (e == hipSuccess && !pg.consts.empty())
            e = hipMemcpy(d.d_consts[k], pg.consts.data(), pg.consts.size() * sizeof(Xfe), hipMemcpyHostToDevice);
    }
    if (e != hipSuccess) {
        free_dev();
        return hipfail(e);
    }
    try {
        a->devs.reserve(a->devs.size() + 1);
    } catch (const std::bad_alloc&) {
        free_dev();
        return NHIP_ERR_OOM;
    }
    a->devs.push_back(d);
    *out = d;
    return NHIP_OK;
}

// Instructions per step of the compiled AIR program: two per thread of k_ood_air's 256-thread
// workgroups (nhip_air_options.step_width sets another, tests of the compiler).
static constexpr uint32_t OOD_STEP_WIDTH = 512;

// The program a batch of n proofs runs: the wide-step one up to NHIP_OOD_WIDE_PROG_MAX proofs (default
// 1,024), where one proof's evaluation latency matters more than proofs per CU.  Config 4 per-GPU
// shares (profiles/r04f): 512 proofs 416-419k proofs/s wide vs 398k narrow, 1,024: 427-430k vs 420k,
// 2,048: 368-374k vs 440k (8 steps in flight: the wide program's one workgroup per CU is the
// bottleneck there), 4,096: 425k vs 436-437k.
int ood_program_for(uint32_t n) {
    static const uint32_t lim = [] {
        const char* e = nhip::ab_env("NHIP_OOD_WIDE_PROG_MAX");
        return e ? (uint32_t)std::strtoul(e, nullptr, 10) : 1024u;
    }();
    return n <= lim ? 1 : 0;
}

// Compile the circuit into the slot program of k_ood_air (OodIns, stark.hpp): a sequence of
// steps, each a set of independent instructions the workgroup runs between two barriers, every
// value in a slot from the step that computes it to the step of its last use (a slot is reused
// from the step after).  The steps come from list scheduling with a liveness priority instead of
// the circuit's levels: a level-by-level program keeps every value of a wide level live at once
// (triton-air-sized circuits: ~13k slots, half of them past the LDS budget in global memory), while
// here each step takes up to `width` ready nodes, those that retire an operand (its last use) first,
// then in the order of the first constraint that needs them, so constraints are finished one after
// another and their values released (the same circuit: ~2.3k slots, all in LDS, 3x the steps).
// A step never takes a node past the LDS slot budget unless it retires a value or the step would be
// empty.  A constraint's value is copied (OOD_ACC) in the step after it is computed into its own slot
// of the top C slots (slots - C + c), and the kernel weighs all C of them in full waves after the last
// step: folded into the steps, each step paid one mostly idle wave of two XFE products per lane for
// its handful of constraints.  Within a step the instructions are grouped by kind (copies, products,
// sums, differences): a wave then runs one kind of XFE operation instead of the divergent union of
// several.
void air_compile(const nhip_air* a, const std::vector<uint32_t>& cons, uint32_t width, uint32_t slot_budget,
                 OodProgram& pg) {
    pg = OodProgram{};
    pg.width = width;
    const size_t NN = a->nodes.size();
    const auto is_op = [&](size_t i) {
        const uint32_t op = a->nodes[i].op;
        return op == AIR_ADD || op == AIR_SUB || op == AIR_MUL;
    };
    // nodes the constraints reach, each with the first constraint (descriptor order) that needs it
    std::vector<uint32_t> corder(NN, UINT32_MAX);
    {
        std::vector<uint32_t> st;
        for (size_t c = 0; c < cons.size(); ++c) {
            st.push_back(cons[c]);
            while (!st.empty()) {
                const uint32_t i = st.back();
                st.pop_back();
                if (corder[i] != UINT32_MAX) continue;
                corder[i] = (uint32_t)c;
                if (is_op(i)) {
                    st.push_back(a->nodes[i].a);
                    st.push_back(a->nodes[i].b);
                }
            }
        }
    }
    // every live value in a slot: inputs and constants are copied in (LOAD from the inputs or the
    // constant table), so the operands of ADD / SUB / MUL are slots only and the kernel reads them
    // from LDS without telling slots from constants (each constant is used about once)
    std::vector<uint32_t> ref(NN, 0), cidx(NN, 0);
    std::vector<uint8_t> slotted(NN, 0);  // live nodes (every one takes a slot)
    for (size_t i = 0; i < NN; ++i) {
        if (corder[i] == UINT32_MAX) continue;  // dead node
        if (a->nodes[i].op == AIR_CONST) {
            cidx[i] = (uint32_t)pg.consts.size();
            pg.consts.push_back(Xfe{a->nodes[i].k0, a->nodes[i].k1, a->nodes[i].k2});
        }
        slotted[i] = 1;
    }
    // remaining uses of each slotted value (operand occurrences + accumulations), pending operands of
    // each node, and the users of each value (CSR)
    std::vector<uint32_t> remaining(NN, 0), deps(NN, 0), uoff(NN + 1, 0);
    for (size_t i = 0; i < NN; ++i)
        if (slotted[i] && is_op(i))
            for (uint32_t o : {a->nodes[i].a, a->nodes[i].b})
                if (slotted[o]) ++remaining[o], ++deps[i], ++uoff[o + 1];
    for (uint32_t c : cons)
        if (slotted[c]) ++remaining[c];
    for (size_t i = 0; i < NN; ++i) uoff[i + 1] += uoff[i];
    std::vector<uint32_t> users(uoff[NN]);
    {
        std::vector<uint32_t> fill(uoff.begin(), uoff.end() - 1);
        for (size_t i = 0; i < NN; ++i)
            if (slotted[i] && is_op(i))
                for (uint32_t o : {a->nodes[i].a, a->nodes[i].b})
                    if (slotted[o]) users[fill[o]++] = (uint32_t)i;
    }
    std::vector<std::vector<uint32_t>> acc_of(NN);  // per node: the constraints whose value it is
    for (size_t c = 0; c < cons.size(); ++c) acc_of[cons[c]].push_back((uint32_t)c);
    std::vector<uint32_t> ready;
    for (size_t i = 0; i < NN; ++i)
        if (slotted[i] && deps[i] == 0) ready.push_back((uint32_t)i);
    // working slots; the C constraint slots above them take their share of the LDS first
    // (nhip_air_options.slot_budget lowers it: tests of the compiler)
    uint32_t budget = AIR_LDS_SLOTS_MAX > cons.size() + 256 ? AIR_LDS_SLOTS_MAX - (uint32_t)cons.size() : 256u;
    if (slot_budget) budget = std::min<uint32_t>(budget, std::max<uint32_t>(64u, slot_budget));
    std::vector<uint32_t> free_slots, to_free;
    uint32_t next_slot = 0, live = 0;
    std::vector<OodIns> cur, acc_next;
    std::vector<std::pair<int32_t, uint64_t>> key(NN);
    auto retires = [&](uint32_t i) {  // operands whose last use this node is
        if (!is_op(i)) return 0;
        const uint32_t x = a->nodes[i].a, y = a->nodes[i].b;
        int r = 0;
        if (slotted[x] && remaining[x] == (x == y ? 2u : 1u)) ++r;
        if (slotted[y] && y != x && remaining[y] == 1u) ++r;
        return r;
    };
    auto use = [&](uint32_t o) {  // a read of o in this step (its slot index is ref[o])
        if (slotted[o] && --remaining[o] == 0) to_free.push_back(ref[o]);
    };
    pg.prog_off.assign(1, 0);
    while (!ready.empty() || !acc_next.empty()) {
        cur.swap(acc_next);  // the accumulations of the values of the step before
        acc_next.clear();
        for (const OodIns& ins : cur)
            if (slotted[cons[ins.b]]) use(cons[ins.b]);
        for (uint32_t i : ready) key[i] = {-retires(i), ((uint64_t)corder[i] << 32) | i};
        std::sort(ready.begin(), ready.end(), [&](uint32_t x, uint32_t y) { return key[x] < key[y]; });
        // the step's constraint copies count against its width (width + a few would be one more,
        // nearly empty pass of the workgroup)
        const size_t room = width > cur.size() ? width - cur.size() : 1;
        std::vector<uint32_t> chosen, rest;
        for (uint32_t i : ready) {
            if (chosen.size() < room && (live < budget || key[i].first < 0 || chosen.empty())) {
                chosen.push_back(i);
                ++live;
            } else {
                rest.push_back(i);
            }
        }
        ready.swap(rest);
        for (uint32_t i : chosen) {
            uint32_t sl;
            if (!free_slots.empty()) {
                sl = free_slots.back();
                free_slots.pop_back();
            } else {
                sl = next_slot++;
            }
            const AirNode& nd = a->nodes[i];
            if (nd.op == AIR_INPUT) {
                cur.push_back(OodIns{OOD_LOAD, OOD_REF_INPUT | (nd.a << 27) | nd.b, 0, sl});
            } else if (nd.op == AIR_CONST) {
                cur.push_back(OodIns{OOD_LOAD, OOD_REF_CONST | cidx[i], 0, sl});
            } else {
                cur.push_back(OodIns{nd.op, ref[nd.a], ref[nd.b], sl});
                use(nd.a);
                use(nd.b);
            }
            ref[i] = OOD_REF_SLOT | sl;
            for (uint32_t c : acc_of[i]) acc_next.push_back(OodIns{OOD_ACC, ref[i], c, 0});
        }
        for (uint32_t i : chosen)
            for (uint32_t k = uoff[i]; k < uoff[i + 1]; ++k)
                if (--deps[users[k]] == 0) ready.push_back(users[k]);
        // values whose last use was in this step: their slots take new values from the next step on
        live -= (uint32_t)to_free.size();
        free_slots.insert(free_slots.end(), to_free.begin(), to_free.end());
        to_free.clear();
        auto kind_rank = [](uint32_t op) {
            return op == OOD_LOAD || op == OOD_ACC ? 0 : (op == AIR_MUL ? 1 : (op == AIR_ADD ? 2 : 3));
        };
        std::stable_sort(cur.begin(), cur.end(),
                         [&](const OodIns& x, const OodIns& y) { return kind_rank(x.op) < kind_rank(y.op); });
        pg.prog.insert(pg.prog.end(), cur.begin(), cur.end());
        pg.prog_off.push_back((uint32_t)pg.prog.size());
        cur.clear();
    }
    for (OodIns& ins : pg.prog)
        if (ins.op == OOD_ACC) ins.dst = next_slot + ins.b;
    pg.slots = next_slot + (uint32_t)cons.size();
}

inline size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

// Size of a buffer that must grow from `have` to hold `need`: exact for a one-shot batch; for
// buffers refilled again and again (streams, the queue's slots, the verify scratch) with headroom
// and at least doubling, so that batches of varying size stop reallocating after a few calls (a
// hipFree / hipHostFree waits for the device, which stalls the other batches in flight).
inline size_t grown(size_t need, size_t have, bool refilled) {
    if (!refilled) return need;
    return std::max(need + need / 4, have ? 2 * have : 0);
}

}  // namespace

extern "C" {

void nhip_stark_params_default(nhip_stark_params* out) {
    if (!out) return;
    out->security_level = 160;
    out->log2_fri_expansion = 2;
    out->num_collinearity_checks = 80;  // security_level / log2_fri_expansion
    out->num_main = 379;
    out->num_aux = 88;
    out->num_quotient_segments = 4;
    out->input_form = NHIP_INPUT_CANONICAL;
}

int nhip_air_create(const uint64_t* w, size_t n, nhip_air** out) { return nhip_air_create_ex(w, n, nullptr, out); }

int nhip_air_create_ex(const uint64_t* w, size_t n, const nhip_air_options* opt, nhip_air** out) {
    if (!w || !out || n < 9) return NHIP_ERR_ARG;
    *out = nullptr;
    const nhip_air_options o = opt ? *opt : nhip_air_options{0, 0, 0};
    const uint32_t width = o.step_width ? o.step_width : OOD_STEP_WIDTH;
    if (width < 16 || width > (1u << 16)) return NHIP_ERR_ARG;
    if (w[0] != 0x41495231ull) return NHIP_ERR_ARG;
    const uint64_t M = w[1], A = w[2], K = w[3], NN = w[4];
    const uint64_t nc[4] = {w[5], w[6], w[7], w[8]};
    const uint64_t C = nc[0] + nc[1] + nc[2] + nc[3];
    // K: the sampled challenges, triton-air's Challenges::SAMPLE_COUNT (include/nhip_challenge_id.h);
    // the derived ones (K .. K + 3) read sampled ChallengeIds up to LookupTablePublicIndeterminate
    if (M > (1u << 20) || A > (1u << 20) || K != NHIP_CHALLENGE_SAMPLE_COUNT || NN > (1u << 24) || C > (1u << 24))
        return NHIP_ERR_ARG;
    if (n != 9 + 4 * NN + C) return NHIP_ERR_ARG;
    nhip_air* a = new (std::nothrow) nhip_air();
    if (!a) return NHIP_ERR_OOM;
    a->dims_air.num_main = (uint32_t)M;
    a->dims_air.num_aux = (uint32_t)A;
    a->dims_air.num_sampled = (uint32_t)K;
    a->dims_air.num_constraints = (uint32_t)C;
    a->nodes.resize(NN);
    std::vector<uint32_t> level(NN, 0);
    uint32_t max_level = 0;
    const uint64_t* nw = w + 9;
    for (uint64_t i = 0; i < NN; ++i) {
        const uint64_t op = nw[4 * i], x = nw[4 * i + 1], y = nw[4 * i + 2], z = nw[4 * i + 3];
        AirNode nd{};
        nd.op = (uint32_t)op;
        bool ok = true;
        if (op == AIR_INPUT) {
            const uint64_t lim = x == IN_MAIN_CURR || x == IN_MAIN_NEXT ? M
                                 : (x == IN_AUX_CURR || x == IN_AUX_NEXT ? A : (x == IN_CHALLENGE ? K + NHIP_NUM_DERIVED_CHALLENGES : 0));
            ok = x <= IN_CHALLENGE && y < lim;
            nd.a = (uint32_t)x;
            nd.b = (uint32_t)y;
        } else if (op == AIR_CONST) {
            nd.k0 = to_mont(x);
            nd.k1 = to_mont(y);
            nd.k2 = to_mont(z);
        } else if (op == AIR_ADD || op == AIR_SUB || op == AIR_MUL) {
            ok = x < i && y < i;
            nd.a = (uint32_t)x;
            nd.b = (uint32_t)y;
            if (ok) level[i] = 1 + std::max(level[x], level[y]);
        } else {
            ok = false;
        }
        if (!ok) {
            delete a;
            return NHIP_ERR_ARG;
        }
        a->nodes[i] = nd;
        max_level = std::max(max_level, level[i]);
    }
    a->level_off.assign(max_level + 2, 0);
    for (uint64_t i = 0; i < NN; ++i) a->level_off[level[i] + 1]++;
    for (uint32_t l = 0; l <= max_level; ++l) a->level_off[l + 1] += a->level_off[l];
    const uint64_t* cw = nw + 4 * NN;
    std::vector<uint32_t> cons(C);
    for (uint64_t i = 0; i < C; ++i) {
        if (cw[i] >= NN) {
            delete a;
            return NHIP_ERR_ARG;
        }
        cons[i] = (uint32_t)cw[i];
    }
    a->cons_off = make_uint4((uint32_t)nc[0], (uint32_t)(nc[0] + nc[1]), (uint32_t)(nc[0] + nc[1] + nc[2]), (uint32_t)C);
    air_compile(a, cons, width, o.slot_budget, a->progs[0]);
    air_compile(a, cons, 2 * width, o.slot_budget, a->progs[1]);
    if (o.lds_slots) a->lds_cap = std::min<uint32_t>(AIR_LDS_SLOTS_MAX, o.lds_slots);
    *out = a;
    return NHIP_OK;
}

void nhip_air_destroy(nhip_air* a) {
    if (!a) return;
    for (const auto& d : a->devs) {
        const DeviceScope device_scope(d.device);
        for (int k = 0; k < 2; ++k) {
            (void)hipFree(d.d_prog[k]);
            (void)hipFree(d.d_prog_off[k]);
            (void)hipFree(d.d_consts[k]);
        }
    }
    delete a;
}

int nhip_air_info(const nhip_air* a, uint32_t* num_nodes, uint32_t* num_levels, uint32_t* num_constraints) {
    if (!a) return NHIP_ERR_ARG;
    if (num_nodes) *num_nodes = (uint32_t)a->nodes.size();
    if (num_levels) *num_levels = (uint32_t)a->level_off.size() - 1;
    if (num_constraints) *num_constraints = a->dims_air.num_constraints;
    return NHIP_OK;
}

// Slots of the compiled AIR program: held in LDS, and past the LDS budget (global memory).
int nhip_air_slots(const nhip_air* a, uint32_t* lds_slots, uint32_t* global_slots) {
    if (!a) return NHIP_ERR_ARG;
    const uint32_t l = std::min<uint32_t>(a->progs[0].slots, a->lds_cap);
    if (lds_slots) *lds_slots = l;
    if (global_slots) *global_slots = a->progs[0].slots - l;
    return NHIP_OK;
}

int nhip_air_program(const nhip_air* a, uint32_t* step_off, size_t step_cap, uint32_t* ins, size_t ins_cap,
                     size_t* n_steps, size_t* n_ins) {
    if (!a) return NHIP_ERR_ARG;
    const OodProgram& pg = a->progs[0];
    const size_t ns = pg.prog_off.size() - 1, ni = pg.prog.size();
    if (n_steps) *n_steps = ns;
    if (n_ins) *n_ins = ni;
    if (step_off) {
        if (step_cap < ns + 1) return NHIP_ERR_ARG;
        std::memcpy(step_off, pg.prog_off.data(), (ns + 1) * 4);
    }
    if (ins) {
        if (ins_cap < 4 * ni) return NHIP_ERR_ARG;
        for (size_t i = 0; i < ni; ++i) {
            ins[4 * i] = pg.prog[i].op;
            ins[4 * i + 1] = pg.prog[i].a;
            ins[4 * i + 2] = pg.prog[i].b;
            ins[4 * i + 3] = pg.prog[i].dst;
        }
    }
    return NHIP_OK;
}

// Host-only structural check (no GPU): 1 if the proof stream decodes with the expected item
// sequence and counts, else 0.  Used by CPU tests of the decoder and by callers that want to
// reject garbage before touching a device.
int nhip_proof_decodes(const nhip_air* air, const nhip_stark_params* sp, const nhip_claim* claim,
                       const nhip_proof* proof) {
    Dims D{};
    if (!claim || !proof || (proof->len && !proof->words) || !dims_from(sp, air, D)) return -NHIP_ERR_ARG;
    // the same walk k_decode runs, straight on the caller's words (proof_codec.hpp)
    ProofDesc pd;
    FsOp ops[fs_ops_for(MAX_FRI_ROUNDS)];
    uint64_t perms, perms_lcw;
    const ClaimLoc cl{0, (uint32_t)claim->input_len, (uint32_t)claim->output_len};
    const uint32_t f = D.mont_words ? decode_stream<true>(proof->words, 0, proof->len, cl, D, pd, ops, perms, perms_lcw)
                                    : decode_stream<false>(proof->words, 0, proof->len, cl, D, pd, ops, perms, perms_lcw);
    return f ? 0 : 1;
}

namespace {
// Stage + upload a batch: proof words (raw; k_decode walks them on the device every run) and
// the staged claim encodings into the batch word buffer, the per-proof ProofIn records, and the
// scratch sized from the padded height each proof header declares.  reuse == nullptr: a new batch
// (*out); otherwise `reuse` is refilled in place (same streams and events; its device memory reused
// when large enough).
int batch_prepare(nhip_ctx* ctx, nhip_air* air, const nhip_stark_params* sp, const nhip_claim* claims,
                  const nhip_proof* proofs, size_t n, nhip_batch** out, VerifyScratch* scr,
                  nhip_batch* reuse = nullptr) {
    if (!ctx || !out || (n && (!claims || !proofs))) return NHIP_ERR_ARG;
    if (reuse && (reuse->in_flight || reuse->scratch)) return NHIP_ERR_ARG;
    if (!reuse) *out = nullptr;
    Dims D{};
    if (!dims_from(sp, air, D)) return NHIP_ERR_ARG;
    if (n > 0xFFFFFFFFull) return NHIP_ERR_ARG;
    for (size_t i = 0; i < n; ++i)
        if ((proofs[i].len && !proofs[i].words) || (claims[i].input_len && !claims[i].input) ||
            (claims[i].output_len && !claims[i].output) || claims[i].input_len > 0xFFFFFFFFull ||
            claims[i].output_len > 0xFFFFFFFFull)
            return NHIP_ERR_ARG;
    std::lock_guard<std::mutex> g(*nhip_internal_mutex(ctx));
    const DeviceScope device_scope(nhip_internal_device(ctx));
    nhip_batch* b = reuse ? reuse : new (std::nothrow) nhip_batch();
    if (!b) return NHIP_ERR_OOM;
    // on failure: a new batch is deleted; a refilled one is left empty (n = 0) but usable
    auto fail_out = [&](int rc) {
        if (!reuse) {
            if (!scr && b->dmem) (void)hipFree(b->dmem);
            if (!scr && b->dwords) (void)hipFree(b->dwords);
            delete b;
        } else {
            b->H = HostBatch{};
            b->dev.n_proofs = 0;
        }
        return rc;
    };
    // a host allocation failing below leaves no half-built batch behind (the upload threads are
    // joined before anything after their start can throw)
    try {
        b->air = air;
        b->device = nhip_internal_device(ctx);
        b->scratch = scr;
        b->H = HostBatch{};
        HostBatch& H = b->H;
        H.D = D;
        H.n = (uint32_t)n;
        const auto t0 = std::chrono::steady_clock::now();
        // ---- layout and scratch sizes: proof words back to back, then the claim encodings; the
        // padded height each proof declares (its first item, 5 header words) sizes the multiproof plan,
        // the sample areas and the Fiat-Shamir program slots.  k_decode re-reads it and rejects a proof
        // whose walk disagrees (never happens for one buffer; guards the scratch bounds).
        std::vector<ProofIn> pin(n);
        std::vector<ProofShape> shp(n);
        uint64_t cur = 0;
        for (size_t i = 0; i < n; ++i) {
            pin[i].off = cur;
            pin[i].len = proofs[i].len;
            cur += proofs[i].len;
        }
        H.proof_words = cur;
        for (size_t i = 0; i < n; ++i) {
            pin[i].claim_off = cur;
            pin[i].claim_in_n = (uint32_t)claims[i].input_len;
            pin[i].claim_out_n = (uint32_t)claims[i].output_len;
            cur += claim_words(claims[i]);
        }
        H.words_total = cur;
        for (size_t i = 0; i < n; ++i) {
            uint64_t lph = 0;
            ProofShape s{};
            const bool hdr = D.mont_words ? header_log2_ph<true>(proofs[i].words, proofs[i].len, lph)
                                          : header_log2_ph<false>(proofs[i].words, proofs[i].len, lph);
            if (hdr && shape_of(D, lph, s)) {
                pin[i].sized_log2_ph = s.log2_ph;
                shp[i] = s;
                H.max_R = std::max(H.max_R, s.R);
                H.levels = std::max(H.levels, s.log2_N);
                H.max_last_cw = std::max(H.max_last_cw, 1u << (s.log2_N - s.R));
            } else {
                pin[i].sized_log2_ph = SHAPE_NONE;
            }
        }
        H.fs_stride = fs_ops_for(H.max_R);
        H.xs_stride = SampleLayout::of(D.d, H.max_R).total;
        // ---- device word buffer (grow-only; its own allocation)
        const size_t wbytes = H.words_total * 8 + 8;
        {
            void** dw = scr ? &scr->dwords : &b->dwords;
            size_t* dwb = scr ? &scr->dwords_bytes : &b->dwords_bytes;
            if (*dwb < wbytes) {
                const size_t have = *dwb;  // read before the free: the growth rule doubles from it
                if (*dw) (void)hipFree(*dw);
                *dw = nullptr;
                *dwb = 0;
                const size_t want = grown(wbytes, have, reuse || scr);
                const hipError_t ea = hipMalloc(dw, want);
                if (ea != hipSuccess) {
                    if (scr) b->dwords = nullptr;
                    return fail_out(hipfail(ea));
                }
                *dwb = want;
            }
            b->dwords = *dw;
        }
        hipStream_t st = nhip_internal_stream(ctx);
        uint64_t* d_words = (uint64_t*)b->dwords;
        hipError_t e = hipSuccess;
        auto dma = [&](uint64_t dst_word, const uint64_t* src, uint64_t nw) {
            if (e == hipSuccess && nw) e = hipMemcpyAsync(d_words + dst_word, src, nw * 8, hipMemcpyHostToDevice, st);
        };
        // ---- upload.  Proofs in pinned caller memory (nhip_host_alloc / nhip_host_register) are
        // DMA'd as they lie, adjacent ones as one copy; the others are copied into the context's
        // pinned staging (same layout as the device buffer) by host threads, ~64 MB chunks in proof
        // order, each chunk's DMA issued as soon as its copies are done.  The claim encodings go
        // through the staging too.
        {
            std::vector<uint8_t> direct(n, 0);
            for (size_t i = 0; i < n; ++i)
                direct[i] = proofs[i].len && pinned().contains(proofs[i].words, proofs[i].len * 8) ? 1 : 0;
            for (size_t i = 0; i < n;) {  // direct segments first: the DMA engine starts right away
                if (!direct[i]) {
                    ++i;
                    continue;
                }
                size_t j = i + 1;
                while (j < n && direct[j] && proofs[j].words == proofs[j - 1].words + proofs[j - 1].len) ++j;
                dma(pin[i].off, proofs[i].words, pin[j - 1].off + pin[j - 1].len - pin[i].off);
                i = j;
            }
            std::vector<uint64_t> pageable;
            uint64_t* stage = (uint64_t*)nhip_internal_staging(ctx, wbytes);
            if (!stage) {
                pageable.resize(H.words_total + 1);
                stage = pageable.data();
            }
            for (size_t i = 0; i < n; ++i) encode_claim(claims[i], D.mont_words != 0, stage + pin[i].claim_off);
            std::vector<size_t> todo;  // staged proofs, in order
            uint64_t staged_bytes = 0;
            for (size_t i = 0; i < n; ++i)
                if (!direct[i] && proofs[i].len) todo.push_back(i), staged_bytes += proofs[i].len * 8;
            constexpr uint64_t CHUNK_WORDS = 8ull << 20;  // 64 MB
            std::vector<size_t> cut{0};                   // chunk c = todo[cut[c] .. cut[c + 1])
            for (size_t q = 1; q < todo.size(); ++q)
                if (pin[todo[q]].off - pin[todo[cut.back()]].off >= CHUNK_WORDS) cut.push_back(q);
            cut.push_back(todo.size());
            const size_t nc = todo.empty() ? 0 : cut.size() - 1;
            std::unique_ptr<std::atomic<size_t>[]> left(new std::atomic<size_t>[nc + 1]);
            std::vector<size_t> chunk_of(todo.size());
            for (size_t c = 0; c < nc; ++c) {
                left[c].store(cut[c + 1] - cut[c]);
                for (size_t q = cut[c]; q < cut[c + 1]; ++q) chunk_of[q] = c;
            }
            std::atomic<size_t> next{0};
            const bool nt = stage_nt() && stage != pageable.data();
            auto work = [&]() {
                for (size_t q; (q = next.fetch_add(1)) < todo.size();) {
                    const size_t i = todo[q];
                    if (nt) {
                        copy_words_nt(stage + pin[i].off, proofs[i].words, proofs[i].len);
                        _mm_sfence();  // the streaming stores are globally visible before the chunk is released
                    } else {
                        std::memcpy(stage + pin[i].off, proofs[i].words, proofs[i].len * 8);
                    }
                    left[chunk_of[q]].fetch_sub(1, std::memory_order_release);
                }
            };
            std::vector<std::thread> pool;
            // copy threads on the CPUs of the GPU's NUMA node, where the staging lives (host_numa.cpp):
            // at most that node's CPUs, or the count set by nhip_set_host_threads (a group divides a
            // node's CPUs among the members on it)
            const nhip::HostTopo& topo = ctx_topo(ctx);
            unsigned threads = host_threads(staged_bytes);
            if (const unsigned set = nhip_internal_host_threads(ctx); set && threads > 1 && !nhip::host_threads_env())
                threads = set;
            if (!topo.cpus.empty() && nhip::numa_enabled()) threads = std::min<unsigned>(threads, (unsigned)topo.cpus.size());
            if (threads > 1 && stage != pageable.data()) {
                pool.reserve(threads);
                for (unsigned t = 0; t < threads; ++t) {
                    try {
                        pool.emplace_back([&]() {
                            (void)nhip::bind_thread(topo.cpus);
                            work();
                        });
                    } catch (const std::system_error&) {
                        break;  // fewer threads: the running ones (and this one, below) take the rest
                    }
                }
            }
            if (pool.empty()) work();
            // DMA each chunk once copied: its staged proofs, adjacent ones as one copy
            for (size_t c = 0; c < nc; ++c) {
                while (left[c].load(std::memory_order_acquire) != 0) {
                    if (pool.empty()) break;
                    std::this_thread::sleep_for(std::chrono::microseconds(20));
                }
                for (size_t q = cut[c]; q < cut[c + 1];) {
                    size_t r = q + 1;
                    while (r < cut[c + 1] && todo[r] == todo[r - 1] + 1) ++r;
                    const size_t i0 = todo[q], i1 = todo[r - 1];
                    dma(pin[i0].off, stage + pin[i0].off, pin[i1].off + pin[i1].len - pin[i0].off);
                    q = r;
                }
            }
            for (auto& th : pool) th.join();
            dma(H.proof_words, stage + H.proof_words, H.words_total - H.proof_words);
            if (stage == pageable.data() && e == hipSuccess) e = hipStreamSynchronize(st);  // pageable source
        }
        const auto t1 = std::chrono::steady_clock::now();
        b->stage_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
        if (e != hipSuccess) {
            (void)hipStreamSynchronize(st);
            if (scr) b->dwords = nullptr;
            return fail_out(hipfail(e));
        }
        nhip_air::Dev adev{};
        int rc = air_upload(ctx, air, &adev);
        if (rc) {
            (void)hipStreamSynchronize(st);
            return fail_out(rc);
        }
        {
            static std::mutex attrs_mu;
            static uint64_t attrs_set = 0;  // devices whose kernel attributes are set
            std::lock_guard<std::mutex> attrs_lock(attrs_mu);
            const int adevice = nhip_internal_device(ctx);
            if (adevice >= 64 || !((attrs_set >> adevice) & 1u)) {
                if (stark_set_kernel_attributes() != hipSuccess) {
                    (void)hipStreamSynchronize(st);
                    return fail_out(NHIP_ERR_HIP);
                }
                if (adevice < 64) attrs_set |= 1ull << adevice;
            }
        }
        const uint32_t k = D.d.num_checks;
        const int pk = ood_program_for((uint32_t)n);
        const OodProgram& pg = air->progs[pk];
        // multiproof op capacity per (level, shard): a tree of height h has at most min(k, 2^(h-1-l))
        // parents at level l; shard = proof index % MP_SHARDS
        const uint32_t tpp = 4 + H.max_R;
        const uint32_t levels = H.levels;
        std::vector<uint64_t> mp_scap((size_t)levels * MP_SHARDS, 0), mp_sbase((size_t)levels * MP_SHARDS, 0);
        b->mp_cap.assign(levels, 0);
        for (size_t i = 0; i < n; ++i) {
            if (pin[i].sized_log2_ph == SHAPE_NONE) continue;
            const ProofShape& s = shp[i];
            const uint32_t sh = (uint32_t)(i % MP_SHARDS);
            for (uint32_t t = 0; t < 4 + s.R; ++t) {
                const uint32_t h = t < 4 ? s.log2_N : s.log2_N - (t - 4);
                for (uint32_t l = 0; l < h; ++l)
                    mp_scap[(size_t)l * MP_SHARDS + sh] += std::min<uint64_t>(k, 1ull << std::min(h - 1 - l, 40u));
            }
        }
        uint64_t mp_total = 0;
        for (uint32_t l = 0; l < levels; ++l)
            for (uint32_t q = 0; q < MP_SHARDS; ++q) {
                mp_sbase[(size_t)l * MP_SHARDS + q] = mp_total;
                mp_total += mp_scap[(size_t)l * MP_SHARDS + q];
                b->mp_cap[l] += mp_scap[(size_t)l * MP_SHARDS + q];
            }
        const size_t N1 = std::max<size_t>(1, n);
        const size_t sz[] = {8,  // (slot 0 unused: the words have their own allocation)
                             N1 * sizeof(ProofDesc),
                             N1 * H.fs_stride * sizeof(FsOp),
                             N1 * H.xs_stride * 24,
                             N1 * k * 4,
                             N1 * 3 * k * 40,
                             N1 * 9 * 8,
                             N1 * 4,
                             N1 * sizeof(ProofIn),
                             // the readback region, laid out as the pinned h_out: [device counters |
                             // plan counters | verdicts], so one memset clears the counters and one
                             // copy brings everything back (three fewer dependent packets per batch)
                             OUT_HDR + (size_t)levels * MP_SHARDS * 4 + N1 + 8,
                             0,
                             mp_total * 16 + 16,
                             mp_total * 40 + 40,
                             (size_t)levels * MP_SHARDS * 8 + 8,
                             (size_t)levels * MP_SHARDS * 8 + 8,
                             0,
                             N1 * tpp * sizeof(MpRoot),
                             N1 * (1 + H.max_R) * k * 8,
                             N1 * (1 + H.max_R) * 4,
                             N1 * k * 8,
                             N1 * H.max_last_cw * 40,
                             // OOD slots past the LDS budget (an AIR larger than ~6K live XFEs)
                             N1 * (size_t)(pg.slots - std::min<uint32_t>(pg.slots, air->lds_cap)) * 24 + 24,
                             // per (proof, tree group, level) op ranges of the plan (k_mp_climb)
                             N1 * (1 + H.max_R) * (size_t)(levels + 1) * 8,
                             N1 * (1 + H.max_R) * (size_t)(levels + 1) * 4,
                             N1 * (1 + H.max_R) * 4};
        constexpr int NBUF = sizeof(sz) / sizeof(sz[0]);
        size_t total = 0;
        for (size_t x : sz) total += al(x);
        if (scr) {  // grow-only device scratch of the context
            if (scr->dmem_bytes < total) {
                (void)hipStreamSynchronize(st);
                const size_t want = grown(total, scr->dmem_bytes, true);
                if (scr->dmem) (void)hipFree(scr->dmem);
                scr->dmem = nullptr;
                scr->dmem_bytes = 0;
                e = hipMalloc(&scr->dmem, want);
                if (e == hipSuccess) scr->dmem_bytes = want;
            }
            b->dmem = scr->dmem;
        } else if (b->dmem_bytes < total) {  // new batch, or a refill that no longer fits
            (void)hipStreamSynchronize(st);
            const size_t want = grown(total, b->dmem_bytes, reuse != nullptr);
            if (b->dmem) (void)hipFree(b->dmem);
            b->dmem = nullptr;
            b->dmem_bytes = 0;
            e = hipMalloc(&b->dmem, want);
            if (e == hipSuccess) b->dmem_bytes = want;
        }
        if (e != hipSuccess) {
            (void)hipStreamSynchronize(st);
            if (scr) b->dmem = nullptr;
            return fail_out(hipfail(e));
        }
        char* p = (char*)b->dmem;
        void* ptr[NBUF];
        for (int i = 0; i < NBUF; ++i) {
            ptr[i] = p;
            p += al(sz[i]);
        }
        if (n) e = hipMemcpyAsync(ptr[8], pin.data(), n * sizeof(ProofIn), hipMemcpyHostToDevice, st);
        if (e == hipSuccess && levels)
            e = hipMemcpyAsync(ptr[13], mp_sbase.data(), mp_sbase.size() * 8, hipMemcpyHostToDevice, st);
        if (e == hipSuccess && levels)
            e = hipMemcpyAsync(ptr[14], mp_scap.data(), mp_scap.size() * 8, hipMemcpyHostToDevice, st);
        {
            const hipError_t es = hipStreamSynchronize(st);  // the sources are host vectors / the staging
            if (e == hipSuccess) e = es;
        }
        const auto t2 = std::chrono::steady_clock::now();
        b->upload_ms = std::chrono::duration<double, std::milli>(t2 - t1).count();
        if (e != hipSuccess) return fail_out(hipfail(e));
        StarkBatchDev& dv = b->dev;
        dv.n_proofs = (uint32_t)n;
        dv.max_R = H.max_R;
        dv.dims = D.d;
        dv.D = D;
        dv.fs_stride = H.fs_stride;
        dv.xs_stride = H.xs_stride;
        dv.words = d_words;
        dv.desc = (ProofDesc*)ptr[1];
        dv.ops = (FsOp*)ptr[2];
        dv.xs = (uint64_t*)ptr[3];
        dv.idx = (uint32_t*)ptr[4];
        dv.dig = (uint64_t*)ptr[5];
        dv.ood = (uint64_t*)ptr[6];
        dv.fail = (uint32_t*)ptr[7];
        dv.in = (const ProofIn*)ptr[8];
        dv.counters = (unsigned long long*)ptr[9];
        dv.verdicts = (uint8_t*)ptr[9] + OUT_HDR + (size_t)levels * MP_SHARDS * 4;
        dv.mp.ops = (uint64_t*)ptr[11];
        dv.mp.arena = (uint64_t*)ptr[12];
        dv.mp.shard_base = (const uint64_t*)ptr[13];
        dv.mp.shard_cap = (const uint64_t*)ptr[14];
        dv.mp.counter = (uint32_t*)((char*)ptr[9] + OUT_HDR);
        dv.mp.roots = (MpRoot*)ptr[16];
        dv.mp.dups = (uint32_t*)ptr[17];
        dv.mp.ndup = (uint32_t*)ptr[18];
        dv.mp.levels = levels;
        dv.xdom = (uint64_t*)ptr[19];
        dv.lcw = (uint64_t*)ptr[20];
        dv.max_lcw = H.max_last_cw;
        dv.mp_cap_host = b->mp_cap.data();
        dv.air_prog = adev.d_prog[pk];
        dv.air_prog_off = adev.d_prog_off[pk];
        dv.air_n_levels = (uint32_t)pg.prog_off.size() - 1;
        dv.air_consts = adev.d_consts[pk];
        dv.air_cons_off = air->cons_off;
        dv.air_lds_slots = std::min<uint32_t>(pg.slots, air->lds_cap);
        dv.air_gslot_n = pg.slots - dv.air_lds_slots;
        dv.air_gslots = (Xfe*)ptr[21];
        dv.mp.lvl_g0 = (uint64_t*)ptr[22];
        dv.mp.lvl_cnt = (uint32_t*)ptr[23];
        dv.mp.lvl_n = (uint32_t*)ptr[24];
        dv.air_lds_bytes = AIR_LDS_HEADER + (size_t)dv.air_lds_slots * 24;
        // 256 threads per proof: 1,024-thread workgroups for a triton-air-sized circuit (one workgroup
        // per CU either way, the slot area fills its LDS) ran the 256-proof evaluation 0.248 -> 0.213 ms
        // alone but took the wave slots the concurrent hashing needs (config 4: 354k -> 305k proofs/s)
        dv.air_block = 256u;
        *out = b;
        return NHIP_OK;
    } catch (const std::bad_alloc&) {
        (void)hipStreamSynchronize(nhip_internal_stream(ctx));
        if (scr) {
            b->dwords = nullptr;
            b->dmem = nullptr;
        }
        return fail_out(NHIP_ERR_OOM);
    }
}
}  // namespace

// host allocations failing inside an entry point become an error code, never an exception
// crossing the C ABI
#define NHIP_GUARD(expr)                                    \
    try {                                                   \
        return (expr);                                      \
    } catch (const std::bad_alloc&) {                       \
        return NHIP_ERR_OOM;                                \
    } catch (...) {                                         \
        return NHIP_ERR_HIP;                                \
    }

static int launch_resources(nhip_batch* b);
// A resident batch: prepared, and its launch resources made now rather than at its first launch (a
// failure there is left to the launch to report)
static void drop_graph(nhip_batch* b);

static int prepare_resident(nhip_ctx* ctx, nhip_air* air, const nhip_stark_params* sp, const nhip_claim* claims,
                            const nhip_proof* proofs, size_t n, nhip_batch** out, nhip_batch* reuse) {
    if (reuse && !reuse->in_flight) {  // new contents: the captured launch sequence is stale
        const DeviceScope device_scope(reuse->device);
        drop_graph(reuse);
    }
    const int rc = batch_prepare(ctx, air, sp, claims, proofs, n, out, nullptr, reuse);
    if (rc != NHIP_OK || !*out) return rc;
    std::lock_guard<std::mutex> g(*nhip_internal_mutex(ctx));
    const DeviceScope device_scope((*out)->device);
    (void)launch_resources(*out);
    return NHIP_OK;
}

int nhip_batch_prepare(nhip_ctx* ctx, nhip_air* air, const nhip_stark_params* sp, const nhip_claim* claims,
                       const nhip_proof* proofs, size_t n, nhip_batch** out) {
    NHIP_GUARD(prepare_resident(ctx, air, sp, claims, proofs, n, out, nullptr))
}

int nhip_batch_refill(nhip_ctx* ctx, nhip_batch* b, nhip_air* air, const nhip_stark_params* sp,
                      const nhip_claim* claims, const nhip_proof* proofs, size_t n) {
    if (!b) return NHIP_ERR_ARG;
    nhip_batch* out = b;
    NHIP_GUARD(prepare_resident(ctx, air, sp, claims, proofs, n, &out, b))
}

// The batch's launch resources: its two streams and timing events (or a verify scratch's) and the
// pinned readback.  Made when the batch is prepared (and on the first launch of one prepared
// before): creating streams, events and pinned memory waits on the device, so doing it at a
// batch's first launch stalled the other batches in flight (a run whose resident batches first
// launch inside a timed region: config 4 at 512 proofs and 10 in flight, 5 warm-up steps, ran at a
// quarter of its rate).
static int launch_resources(nhip_batch* b) {
    if (!b->timed) {
        const char* pm = nhip::ab_env("NHIP_PHASE_MARKS");  // A/B: 0 = the phase events off
        b->tm.phase_marks = !(pm && pm[0] == '0');
        const char* al = nhip::ab_env("NHIP_AUX_AFTER_LEVEL");
        b->tm.aux_after_level = al ? (uint32_t)std::strtoul(al, nullptr, 10) : AUX_AFTER_LEVEL_DEFAULT;
        const size_t out_bytes = OUT_HDR + (size_t)b->dev.mp.levels * MP_SHARDS * 4 + b->dev.n_proofs + 16;
        if (VerifyScratch* sc = b->scratch) {
            if (!sc->streams) {
                for (int i = 0; i < STARK_EVENTS; ++i)
                    if (hipEventCreate(&sc->ev[i]) != hipSuccess) return NHIP_ERR_HIP;
                if (hipStreamCreateWithFlags(&sc->main, hipStreamNonBlocking) != hipSuccess) return NHIP_ERR_HIP;
                if (hipStreamCreateWithFlags(&sc->aux, hipStreamNonBlocking) != hipSuccess) return NHIP_ERR_HIP;
                sc->streams = true;
            }
            if (sc->h_out_bytes < out_bytes) {
                if (sc->h_out) (void)hipHostFree(sc->h_out);
                sc->h_out = nullptr;
                sc->h_out_bytes = 0;
                if (hipHostMalloc((void**)&sc->h_out, out_bytes * 2, hipHostMallocDefault) != hipSuccess)
                    return NHIP_ERR_OOM;
                sc->h_out_bytes = out_bytes * 2;
            }
            for (int i = 0; i < STARK_EVENTS; ++i) b->tm.ev[i] = sc->ev[i];
            b->main = sc->main;
            b->aux = sc->aux;
            b->h_out = sc->h_out;
        } else {
            for (int i = 0; i < STARK_EVENTS; ++i)
                if (hipEventCreate(&b->tm.ev[i]) != hipSuccess) return NHIP_ERR_HIP;
            for (uint32_t i = 0; i < 2 * MAX_HASH_LAUNCHES; ++i)  // per hash launch
                if (hipEventCreate(&b->tm.lev[i]) != hipSuccess) {
                    for (uint32_t j = 0; j < i; ++j) (void)hipEventDestroy(b->tm.lev[j]);
                    for (uint32_t j = 0; j < 2 * MAX_HASH_LAUNCHES; ++j) b->tm.lev[j] = nullptr;
                    break;  // untimed hash launches: a fault of the timing only
                }
            {
                hipEvent_t r0 = nullptr, r1 = nullptr;
                if (hipEventCreate(&r0) == hipSuccess && hipEventCreate(&r1) == hipSuccess) {
                    b->tm.rev[0] = r0;
                    b->tm.rev[1] = r1;
                } else if (r0) {
                    (void)hipEventDestroy(r0);  // an untimed row launch: a fault of the timing only
                }
            }
            if (hipStreamCreateWithFlags(&b->main, hipStreamNonBlocking) != hipSuccess) return NHIP_ERR_HIP;
            if (hipStreamCreateWithFlags(&b->aux, hipStreamNonBlocking) != hipSuccess) return NHIP_ERR_HIP;
        }
        b->timed = true;
    }
    if (!b->scratch) {  // pinned readback, grown when a refill needs more
        const size_t out_bytes = OUT_HDR + (size_t)b->dev.mp.levels * MP_SHARDS * 4 + b->dev.n_proofs + 16;
        if (b->h_out_bytes < out_bytes) {
            const size_t want = std::max<size_t>(grown(out_bytes, b->h_out_bytes, true), 64u << 10);
            if (b->h_out) (void)hipHostFree(b->h_out);
            b->h_out = nullptr;
            b->h_out_bytes = 0;
            if (hipHostMalloc((void**)&b->h_out, want, hipHostMallocDefault) != hipSuccess) return NHIP_ERR_OOM;
            b->h_out_bytes = want;
        }
    }
    return NHIP_OK;
}

// Every device phase of the batch, its counter resets and its readback, on the batch's streams.
static hipError_t enqueue_batch(nhip_batch* b) {
    hipStream_t st = b->main;
    const uint32_t n = b->dev.n_proofs;
    const size_t cnt_bytes = (size_t)b->dev.mp.levels * MP_SHARDS * 4;
    // [device counters | plan counters | verdicts] are one device region in h_out's layout
    hipError_t e = hipMemsetAsync(b->dev.counters, 0, OUT_HDR + cnt_bytes, st);
    if (e == hipSuccess) e = launch_stark_phases(b->dev, st, b->aux, &b->tm);
    if (e == hipSuccess) e = hipMemcpyAsync(b->h_out, b->dev.counters, OUT_HDR + cnt_bytes + n, hipMemcpyDeviceToHost, st);
    return e;
}

static void drop_graph(nhip_batch* b) {
    if (b->gexec) (void)hipGraphExecDestroy(b->gexec);
    b->gexec = nullptr;
}

// The graph bakes in the launch-order wave priority, which applies from 2,048 proofs on: larger
// batches always launch directly.
static constexpr uint32_t GRAPH_MAX_PROOFS = 1024;
static bool graphs_enabled() {  // NHIP_GRAPHS=0 (A/B builds only): every launch direct
    static const bool on = [] {
        const char* e = nhip::ab_env("NHIP_GRAPHS");
        return !e || e[0] != '0';
    }();
    return on;
}

// Capture the batch's launch sequence (its two streams joined, as enqueue_batch leaves them) into an
// executable graph, with the capture's own events; false (and no graph) if the runtime cannot
// capture it: the direct launch is used then.
static bool capture_graph(nhip_batch* b) {
    if (!b->gev[0])
        for (int i = 0; i < STARK_EVENTS; ++i)
            if (hipEventCreateWithFlags(&b->gev[i], hipEventDisableTiming) != hipSuccess) return false;
    hipGraph_t graph = nullptr;
    if (hipStreamBeginCapture(b->main, hipStreamCaptureModeThreadLocal) != hipSuccess) return false;
    StarkPhaseTimer saved = b->tm;
    for (int i = 0; i < STARK_EVENTS; ++i) b->tm.ev[i] = b->gev[i];
    b->tm.phase_marks = false;
    const hipError_t e = enqueue_batch(b);
    const uint32_t launches = b->tm.mp_hash_launches;  // the captured sequence's hash launches
    b->tm = saved;
    b->tm.mp_hash_launches = launches;
    const hipError_t ee = hipStreamEndCapture(b->main, &graph);
    if (e != hipSuccess || ee != hipSuccess || !graph) {
        if (graph) (void)hipGraphDestroy(graph);
        (void)hipGetLastError();
        return false;
    }
    hipGraphExec_t exec = nullptr;
    const hipError_t ei = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    if (ei != hipSuccess || !exec) {
        (void)hipGetLastError();
        return false;
    }
    b->gexec = exec;
    return true;
}

// Enqueue every device phase of the batch on the batch's own two streams (no host wait).  Batches
// launched back to back run concurrently on the device.
int nhip_batch_launch(nhip_ctx* ctx, nhip_batch* b) {
    if (!ctx || !b) return NHIP_ERR_ARG;
    std::lock_guard<std::mutex> g(*nhip_internal_mutex(ctx));
    const DeviceScope device_scope(b->device);
    if (b->in_flight) return NHIP_ERR_ARG;
    if (int rc = launch_resources(b)) return rc;
    hipError_t e = hipSuccess;
    const bool graphable = b->graph_on && !b->tm.launch_events && b->dev.n_proofs <= GRAPH_MAX_PROOFS;
    if (graphable && !b->gexec) (void)capture_graph(b);  // after a refill or a stream change
    b->last_graph = graphable && b->gexec;
    if (b->last_graph) e = hipGraphLaunch(b->gexec, b->main);
    else e = enqueue_batch(b);
    if (e != hipSuccess) return hipfail(e);
    b->in_flight = true;
    return NHIP_OK;
}

// Replay the batch's launch sequence from a captured HIP graph (on != 0): one submission per launch
// instead of ~25 runtime calls, for resident batches of at most 1,024 proofs relaunched many times
// (a pipeline enqueueing R batches back to back delays the device's start of the last one by R host
// enqueues, ~0.2 ms each at 512 proofs).  A launch with launch timing on is always direct; a replayed
// launch reports no phase split (nhip_stats phase fields 0).  NHIP_ERR_ARG while in flight or for a
// batch past 1,024 proofs; a runtime that cannot capture leaves the direct launch (NHIP_OK).
int nhip_batch_set_graph(nhip_batch* b, int on) {
    if (!b || b->in_flight || b->scratch) return NHIP_ERR_ARG;
    if (on && b->dev.n_proofs > GRAPH_MAX_PROOFS) return NHIP_ERR_ARG;
    if (on && !graphs_enabled()) return NHIP_OK;  // an A/B build with graphs off: direct launches
    const DeviceScope device_scope(b->device);
    b->graph_on = on != 0;
    if (!b->graph_on) {
        drop_graph(b);
        return NHIP_OK;
    }
    if (int rc = launch_resources(b)) return rc;
    if (!b->gexec) (void)capture_graph(b);  // now, before the batch's first replay
    return NHIP_OK;
}

// Dispatch begin / end timestamps on the batch's Merkle hash launches and its row launch (the
// bench's kernel timing: nhip_stats.ms_mp_hash_exec / ms_row_hash_exec); off by default, since
// they cost a small batch ~2% of its rate and the product paths do not read them.
int nhip_batch_set_launch_timing(nhip_batch* b, int on) {
    if (!b || b->in_flight) return NHIP_ERR_ARG;
    b->tm.launch_events = on != 0;  // a timed launch is never the graph (its events are per launch)
    return NHIP_OK;
}

// One stream or two for a resident batch.  Two (the default): the latency-bound chain (decode,
// Fiat-Shamir replay, plan, OOD / FRI / DEEP) and the VALU-bound hashing overlap within the batch.
// One: every phase in order on the main stream, one hardware queue per batch, so a caller can keep
// twice as many batches in flight — the better trade for tiny batches run many at a time
// (BASELINE config 5's 8-64 proofs per GPU: +12-18% at twice the depth), the worse one from a few
// hundred proofs on (config 4 at 512-4,096 proofs: -10 to -23%).
int nhip_batch_set_streams(nhip_batch* b, int streams) {
    if (!b || b->in_flight || b->scratch || (streams != 1 && streams != 2)) return NHIP_ERR_ARG;
    const DeviceScope device_scope(b->device);
    if (int rc = launch_resources(b)) return rc;
    const bool had_graph = b->gexec != nullptr;
    if (streams == 1 && b->aux != b->main) {
        drop_graph(b);
        (void)hipStreamSynchronize(b->aux);
        (void)hipStreamDestroy(b->aux);
        b->aux = b->main;
    } else if (streams == 2 && b->aux == b->main) {
        drop_graph(b);
        hipStream_t s2 = nullptr;
        if (hipStreamCreateWithFlags(&s2, hipStreamNonBlocking) != hipSuccess) return NHIP_ERR_HIP;
        b->aux = s2;
    }
    if (had_graph && b->graph_on && !b->gexec) (void)capture_graph(b);  // the new stream layout, now
    return NHIP_OK;
}

// Internal (queue.cpp): has every phase of a launched batch completed?  Its last packets (the verdict
// copy) are on the main stream, which joins the aux chain before them.
bool nhip_internal_batch_done(nhip_batch* b) {
    if (!b || !b->in_flight) return true;
    const DeviceScope device_scope(b->device);
    return hipStreamQuery(b->main) != hipErrorNotReady;
}

// Wait for a launched batch; verdicts (n bytes, nullable) and the batch AND (nullable).
int nhip_batch_wait(nhip_ctx* ctx, nhip_batch* b, uint8_t* verdicts, uint8_t* all_ok) {
    if (!ctx || !b) return NHIP_ERR_ARG;
    if (!b->in_flight) return NHIP_ERR_ARG;
    const DeviceScope device_scope(b->device);
    hipError_t e = hipStreamSynchronize(b->main);
    b->in_flight = false;
    if (e != hipSuccess) return hipfail(e);
    const uint32_t n = b->dev.n_proofs;
    // Merkle permutations: multiproof ops reserved by the plan (per level and shard) minus the ops of
    // trees whose authentication structure failed, plus the last-codeword trees; the sponge + row
    // permutations of the proofs k_decode accepted
    const size_t cnt_n = (size_t)b->dev.mp.levels * MP_SHARDS;
    uint64_t cnt[CNT_N], reserved = 0;
    std::memcpy(cnt, b->h_out, sizeof(cnt));
    for (size_t i = 0; i < cnt_n; ++i) {
        uint32_t c;
        std::memcpy(&c, b->h_out + OUT_HDR + 4 * i, 4);
        reserved += c;
    }
    {  // the hash launches' own durations (dispatch begin / end timestamps; launch timing on)
        double exec = 0;
        const bool ev = b->tm.launch_events;
        const uint32_t nl = ev ? std::min<uint32_t>(b->tm.mp_hash_launches, MAX_HASH_LAUNCHES) : 0u;
        for (uint32_t i = 0; i < nl && b->tm.lev[0]; ++i) {
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, b->tm.lev[2 * i], b->tm.lev[2 * i + 1]) == hipSuccess) exec += ms;
        }
        b->mp_hash_exec_ms = exec;
        float rms = 0.f;
        b->row_hash_exec_ms =
            ev && b->tm.rev[0] && hipEventElapsedTime(&rms, b->tm.rev[0], b->tm.rev[1]) == hipSuccess ? rms : 0.0;
    }
    b->H.perms_static = cnt[CNT_PERMS_STATIC];
    b->H.perms_lcw = cnt[CNT_PERMS_LCW];
    b->merkle_perms = reserved - cnt[CNT_MP_SKIPPED] + b->H.perms_lcw;
    // phases overlap (two streams): each is timed from the event its inputs wait on
    auto el = [&](int a, int c) {
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, b->tm.ev[a], b->tm.ev[c]);
        return (double)ms;
    };
    if (b->last_graph || !b->tm.phase_marks) {
        b->ph = {};  // a replayed launch (its events are the graph's own, untimed) or one without marks
    } else if (n) {
        b->ph.decode = el(12, 0);
        b->ph.fs = el(0, 1);
        b->ph.rows = el(0, 2);
        b->ph.plan = el(1, 3);
        b->ph.hash = std::min(el(2, 4), el(3, 4));
        b->ph.roots = el(4, 5);
        b->ph.ood = el(11, 6);
        const bool small = n <= climb_max_proofs();  // FRI on the main stream (launch_stark_phases)
        b->ph.fri = small ? el(13, 7) : el(6, 7);
        b->ph.deep = small ? el(6, 8) : el(7, 8);
        b->ph.total = el(12, 9);
    }
    const uint8_t* v = b->h_out + OUT_HDR + cnt_n * 4;
    if (verdicts && n) std::memcpy(verdicts, v, n);
    if (all_ok) {
        uint8_t a = 1;
        for (uint32_t i = 0; i < n; ++i) a &= v[i];
        *all_ok = a;
    }
    return NHIP_OK;
}

int nhip_batch_run(nhip_ctx* ctx, nhip_batch* b, uint8_t* verdicts, uint8_t* all_ok) {
    const int rc = nhip_batch_launch(ctx, b);
    if (rc) return rc;
    return nhip_batch_wait(ctx, b, verdicts, all_ok);
}

int nhip_batch_stats(const nhip_batch* b, nhip_stats* s) {
    if (!b || !s) return NHIP_ERR_ARG;
    std::memset(s, 0, sizeof(*s));
    s->num_proofs = b->dev.n_proofs;
    s->proof_words = b->H.proof_words;
    s->ms_decode = b->stage_ms;
    s->ms_upload = b->upload_ms;
    s->ms_fiat_shamir = b->ph.fs;
    s->ms_row_hash = b->ph.rows;
    s->ms_merkle = b->ph.plan + b->ph.hash + b->ph.roots;
    s->ms_merkle_hash = b->ph.hash;
    s->merkle_hash_launches = b->tm.mp_hash_launches;
    s->ms_ood_air = b->ph.ood;
    s->ms_fri = b->ph.fri;
    s->ms_deep = b->ph.deep;
    s->ms_device_total = b->ph.total;
    s->ms_device_decode = b->ph.decode;
    s->ms_mp_hash_exec = b->mp_hash_exec_ms;
    s->ms_row_hash_exec = b->row_hash_exec_ms;
    s->tip5_perms_static = b->H.perms_static;
    s->tip5_perms_merkle = b->merkle_perms;
    // every Merkle hash launch (k_mp_hash + the 16-lane-row k_mp_hash_wide): back to back on the
    // batch's main stream, so the phase span is their summed duration
    s->ms_mp_hash_kernel = b->ph.hash;
    s->mp_hash_kernel_launches = b->tm.mp_hash_launches;
    s->mp_hash_kernel_perms = b->merkle_perms;
    return NHIP_OK;
}

int nhip_batch_transcript(nhip_ctx* ctx, const nhip_batch* b, size_t proof, uint64_t* xfe_out, size_t xfe_cap,
                          uint32_t* idx_out, size_t idx_cap, uint32_t* fail_out, size_t* n_xfe) {
    if (!ctx || !b || proof >= b->dev.n_proofs || b->in_flight) return NHIP_ERR_ARG;
    std::lock_guard<std::mutex> g(*nhip_internal_mutex(ctx));
    const DeviceScope device_scope(b->device);
    hipStream_t st = nhip_internal_stream(ctx);
    ProofDesc pd{};
    hipError_t e = hipMemcpyAsync(&pd, b->dev.desc + proof, sizeof(pd), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return hipfail(e);
    const size_t nx = pd.n_xs;
    if (n_xfe) *n_xfe = nx;
    std::vector<uint64_t> raw(nx * 3);
    if (nx) e = hipMemcpyAsync(raw.data(), b->dev.xs + pd.xs_off * 3, nx * 24, hipMemcpyDeviceToHost, st);
    std::vector<uint32_t> ix(b->dev.dims.num_checks);
    if (e == hipSuccess)
        e = hipMemcpyAsync(ix.data(), b->dev.idx + pd.idx_off, ix.size() * 4, hipMemcpyDeviceToHost, st);
    uint32_t f = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&f, b->dev.fail + proof, 4, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return hipfail(e);
    if (xfe_out)
        for (size_t i = 0; i < std::min(nx * 3, xfe_cap * 3); ++i) xfe_out[i] = from_mont(raw[i]);
    if (idx_out) std::memcpy(idx_out, ix.data(), std::min(ix.size(), idx_cap) * 4);
    if (fail_out) *fail_out = f;
    return NHIP_OK;
}

void nhip_batch_destroy(nhip_batch* b) {
    if (!b) return;
    const DeviceScope device_scope(b->device);
    if (b->in_flight && b->main) (void)hipStreamSynchronize(b->main);
    drop_graph(b);
    for (hipEvent_t e : b->gev)
        if (e) (void)hipEventDestroy(e);
    if (b->scratch) {  // resources belong to the context's verify scratch
        delete b;
        return;
    }
    if (b->timed) {
        for (int i = 0; i < STARK_EVENTS; ++i) (void)hipEventDestroy(b->tm.ev[i]);
        for (uint32_t i = 0; i < 2 * MAX_HASH_LAUNCHES; ++i)
            if (b->tm.lev[i]) (void)hipEventDestroy(b->tm.lev[i]);
        for (hipEvent_t e : b->tm.rev)
            if (e) (void)hipEventDestroy(e);
    }
    if (b->aux && b->aux != b->main) (void)hipStreamDestroy(b->aux);
    if (b->main) (void)hipStreamDestroy(b->main);
    if (b->h_out) (void)hipHostFree(b->h_out);
    if (b->dmem) (void)hipFree(b->dmem);
    if (b->dwords) (void)hipFree(b->dwords);
    delete b;
}

int nhip_host_alloc(size_t bytes, void** out) {
    if (!out) return NHIP_ERR_ARG;
    *out = nullptr;
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocPortable) != hipSuccess) return NHIP_ERR_OOM;
    try {
        std::lock_guard<std::mutex> g(pinned().mu);
        pinned().r.emplace_back((uintptr_t)p, bytes);
    } catch (const std::bad_alloc&) {
        (void)hipHostFree(p);
        return NHIP_ERR_OOM;
    }
    *out = p;
    return NHIP_OK;
}

int nhip_host_alloc_near(nhip_ctx* ctx, size_t bytes, void** out) {
    if (!ctx || !out) return NHIP_ERR_ARG;
    *out = nullptr;
    void* p = nullptr;
    if (nhip::host_malloc_on(&p, bytes ? bytes : 1, ctx_topo(ctx).numa_node, hipHostMallocPortable) != hipSuccess)
        return NHIP_ERR_OOM;
    try {
        std::lock_guard<std::mutex> g(pinned().mu);
        pinned().r.emplace_back((uintptr_t)p, bytes);
    } catch (const std::bad_alloc&) {
        (void)hipHostFree(p);
        return NHIP_ERR_OOM;
    }
    *out = p;
    return NHIP_OK;
}

static bool pinned_forget(void* p) {
    std::lock_guard<std::mutex> g(pinned().mu);
    auto& r = pinned().r;
    for (size_t i = 0; i < r.size(); ++i)
        if (r[i].first == (uintptr_t)p) {
            r.erase(r.begin() + (ptrdiff_t)i);
            return true;
        }
    return false;
}

int nhip_host_free(void* p) {
    if (!p) return NHIP_OK;
    if (!pinned_forget(p)) return NHIP_ERR_ARG;
    return hipfail(hipHostFree(p));
}

int nhip_host_register(void* p, size_t bytes) {
    if (!p || !bytes) return NHIP_ERR_ARG;
    const hipError_t e = hipHostRegister(p, bytes, hipHostRegisterPortable);
    if (e != hipSuccess) return hipfail(e);
    try {
        std::lock_guard<std::mutex> g(pinned().mu);
        pinned().r.emplace_back((uintptr_t)p, bytes);
    } catch (const std::bad_alloc&) {
        (void)hipHostUnregister(p);
        return NHIP_ERR_OOM;
    }
    return NHIP_OK;
}

int nhip_host_unregister(void* p) {
    if (!p || !pinned_forget(p)) return NHIP_ERR_ARG;
    return hipfail(hipHostUnregister(p));
}

int nhip_verify_batch(nhip_ctx* ctx, nhip_air* air, const nhip_stark_params* sp, const nhip_claim* claims,
                      const nhip_proof* proofs, size_t n, uint8_t* verdicts, nhip_stats* stats) {
    if (!verdicts && n) return NHIP_ERR_ARG;
    if (!ctx) return NHIP_ERR_ARG;
    auto* scr = (VerifyScratch*)nhip_internal_verify_scratch(
        ctx, []() -> void* { return new (std::nothrow) VerifyScratch(); }, &free_verify_scratch);
    if (!scr) return NHIP_ERR_OOM;
    std::lock_guard<std::mutex> g(scr->mu);
    nhip_batch* b = nullptr;
    int rc;
    try {
        rc = batch_prepare(ctx, air, sp, claims, proofs, n, &b, scr);
    } catch (const std::bad_alloc&) {
        return NHIP_ERR_OOM;
    }
    if (rc) return rc;
    rc = nhip_batch_run(ctx, b, verdicts, nullptr);
    if (!rc && stats) nhip_batch_stats(b, stats);
    nhip_batch_destroy(b);
    return rc;
}

}  // extern "C"
