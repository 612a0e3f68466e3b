/*
 * nhip_challenge_id.h — the challenge layout of an AIR descriptor (nhip_air_create).
 *
 * A descriptor's INPUT nodes of kind 4 (challenge) index the verifier's challenge vector, which is
 * triton-air 1.0.0's `ChallengeId` (Cargo.lock:4194; the enum in triton-air's challenge_id.rs,
 * crates.io source, not vendored under /root/reference): the 59 challenges Stark::verify squeezes
 * (`proof_stream.sample_scalars(Challenges::SAMPLE_COUNT)`), in declaration order, followed by the 4
 * that `Challenges::new(sampled, claim)` derives and appends, also in declaration order.  The
 * exporter (neptune-core_amd/rust/neptune-hip/src/air_export.rs) writes `ChallengeId::index()`
 * unchanged, so this table must equal the crate's enum.  PARITY UNPINNED: no vector under
 * /root/reference fixes these indices; the order below is the public triton-air 1.0 enum.
 *
 * One list, used by the kernels (stark_kernels.hip), the host (stark_host.cpp: descriptor check)
 * and the C oracle (oracle/stark_oracle.c); the Python oracle (oracle/stark_ref.py CHALLENGE_IDS)
 * keeps an independent copy that tests/test_challenge_ids.py compares with this file.
 *
 * Plain C (C99 / C++ / HIP).
 */
#ifndef NHIP_CHALLENGE_ID_H
#define NHIP_CHALLENGE_ID_H

/* X(name): triton-air ChallengeId variants in declaration order (index = position). */
#define NHIP_CHALLENGE_IDS(X)                                                                        \
    /* 0-12: evaluation / lookup / permutation argument indeterminates */                            \
    X(CompressProgramDigestIndeterminate)                                                            \
    X(StandardInputIndeterminate)                                                                    \
    X(StandardOutputIndeterminate)                                                                   \
    X(InstructionLookupIndeterminate)                                                                \
    X(HashInputIndeterminate)                                                                        \
    X(HashDigestIndeterminate)                                                                       \
    X(SpongeIndeterminate)                                                                           \
    X(OpStackIndeterminate)                                                                          \
    X(RamIndeterminate)                                                                              \
    X(JumpStackIndeterminate)                                                                        \
    X(U32Indeterminate)                                                                              \
    X(ClockJumpDifferenceLookupIndeterminate)                                                        \
    X(RamTableBezoutRelationIndeterminate)                                                           \
    /* 13-15: program table */                                                                       \
    X(ProgramAddressWeight)                                                                          \
    X(ProgramInstructionWeight)                                                                      \
    X(ProgramNextInstructionWeight)                                                                  \
    /* 16-19: op stack */                                                                            \
    X(OpStackClkWeight)                                                                              \
    X(OpStackIb1Weight)                                                                              \
    X(OpStackPointerWeight)                                                                          \
    X(OpStackFirstUnderflowElementWeight)                                                            \
    /* 20-23: RAM */                                                                                 \
    X(RamClkWeight)                                                                                  \
    X(RamPointerWeight)                                                                              \
    X(RamValueWeight)                                                                                \
    X(RamInstructionTypeWeight)                                                                      \
    /* 24-28: jump stack */                                                                          \
    X(JumpStackClkWeight)                                                                            \
    X(JumpStackCiWeight)                                                                             \
    X(JumpStackJspWeight)                                                                            \
    X(JumpStackJsoWeight)                                                                            \
    X(JumpStackJsdWeight)                                                                            \
    /* 29-31: program attestation, hash table */                                                     \
    X(ProgramAttestationPrepareChunkIndeterminate)                                                   \
    X(ProgramAttestationSendChunkIndeterminate)                                                      \
    X(HashCIWeight)                                                                                  \
    /* 32-47: stack weights */                                                                       \
    X(StackWeight0) X(StackWeight1) X(StackWeight2) X(StackWeight3)                                  \
    X(StackWeight4) X(StackWeight5) X(StackWeight6) X(StackWeight7)                                  \
    X(StackWeight8) X(StackWeight9) X(StackWeight10) X(StackWeight11)                                \
    X(StackWeight12) X(StackWeight13) X(StackWeight14) X(StackWeight15)                              \
    /* 48-50: hash <-> cascade lookup */                                                             \
    X(HashCascadeLookupIndeterminate)                                                                \
    X(HashCascadeLookInWeight)                                                                       \
    X(HashCascadeLookOutWeight)                                                                      \
    /* 51: cascade <-> lookup */                                                                     \
    X(CascadeLookupIndeterminate)                                                                    \
    /* 52-54: lookup table */                                                                        \
    X(LookupTableInputWeight)                                                                        \
    X(LookupTableOutputWeight)                                                                       \
    X(LookupTablePublicIndeterminate)                                                                \
    /* 55-58: U32 table */                                                                           \
    X(U32LhsWeight)                                                                                  \
    X(U32RhsWeight)                                                                                  \
    X(U32CiWeight)                                                                                   \
    X(U32ResultWeight)                                                                               \
    /* 59-62: derived by Challenges::new (not sampled) */                                            \
    X(StandardInputTerminal)                                                                         \
    X(StandardOutputTerminal)                                                                        \
    X(LookupTablePublicTerminal)                                                                     \
    X(CompressedProgramDigest)

#define NHIP_CHALLENGE_ENUM_ENTRY(name) NHIP_CH_##name,
enum nhip_challenge_id { NHIP_CHALLENGE_IDS(NHIP_CHALLENGE_ENUM_ENTRY) NHIP_CHALLENGE_COUNT };
#undef NHIP_CHALLENGE_ENUM_ENTRY

/* ChallengeId::NUM_DERIVED_CHALLENGES and Challenges::SAMPLE_COUNT */
#define NHIP_NUM_DERIVED_CHALLENGES 4
#define NHIP_CHALLENGE_SAMPLE_COUNT (NHIP_CHALLENGE_COUNT - NHIP_NUM_DERIVED_CHALLENGES)

#endif /* NHIP_CHALLENGE_ID_H */
