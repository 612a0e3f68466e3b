"""The ChallengeId table (triton-air 1.0 `ChallengeId`, PARITY UNPINNED: public design, no vector
under /root/reference) exists twice: include/nhip_challenge_id.h (kernels, host descriptor check, C
oracle) and oracle/stark_ref.CHALLENGE_IDS (Python oracle, synthetic provers).  They were written
out independently; this test holds them equal, and pins the indices Challenges::new reads."""
import os
import re

import stark_ref as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_ids():
    text = open(os.path.join(ROOT, "include", "nhip_challenge_id.h")).read()
    body = text[text.index("#define NHIP_CHALLENGE_IDS(X)"):text.index("#define NHIP_CHALLENGE_ENUM_ENTRY")]
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    return re.findall(r"\bX\((\w+)\)", body)


def test_header_equals_python_table():
    assert header_ids() == list(S.CHALLENGE_IDS)


def test_layout():
    ids = S.CHALLENGE_IDS
    assert len(ids) == 63 and len(set(ids)) == 63
    assert S.CHALLENGE_SAMPLE_COUNT == 59 and S.NUM_DERIVED_CHALLENGES == 4
    # the sampled indeterminates Challenges::new folds the derived challenges with
    assert S.CH_COMPRESS_PROGRAM_DIGEST_INDETERMINATE == 0
    assert S.CH_STANDARD_INPUT_INDETERMINATE == 1
    assert S.CH_STANDARD_OUTPUT_INDETERMINATE == 2
    assert S.CH_LOOKUP_TABLE_PUBLIC_INDETERMINATE == 54
    assert ids[15] == "ProgramNextInstructionWeight"  # round 2 read the lookup indeterminate here
    # derived challenges follow the sampled ones, in declaration order
    assert ids[59:] == ("StandardInputTerminal", "StandardOutputTerminal", "LookupTablePublicTerminal",
                        "CompressedProgramDigest")
    # group sizes of the enum: 13 indeterminates, 3 program, 4 op stack, 4 RAM, 5 jump stack,
    # 3 attestation / hash, 16 stack, 3 hash-cascade, 1 cascade, 3 lookup, 4 U32
    assert ids.index("ProgramAddressWeight") == 13
    assert ids.index("OpStackClkWeight") == 16
    assert ids.index("RamClkWeight") == 20
    assert ids.index("JumpStackClkWeight") == 24
    assert ids.index("ProgramAttestationPrepareChunkIndeterminate") == 29
    assert ids.index("StackWeight0") == 32 and ids.index("StackWeight15") == 47
    assert ids.index("HashCascadeLookupIndeterminate") == 48
    assert ids.index("CascadeLookupIndeterminate") == 51
    assert ids.index("U32LhsWeight") == 55


def test_derive_challenges_reads_the_named_indeterminates():
    """Challenges::new: each derived challenge is an EvalArg terminal over its own indeterminate, so
    perturbing exactly that sampled challenge changes exactly that derived one."""
    from field_ref import xadd
    sampled = [((7 * i + 1) % S.P, i, 3) for i in range(S.CHALLENGE_SAMPLE_COUNT)]
    claim = ([1, 2, 3, 4, 5], 0, [6, 7], [8])
    base = S.derive_challenges(sampled, claim)
    assert base[:59] == sampled
    for ind, derived in ((1, 59), (2, 60), (54, 61), (0, 62)):
        s2 = list(sampled)
        s2[ind] = xadd(s2[ind], (1, 0, 0))
        d2 = S.derive_challenges(s2, claim)
        assert [j for j in range(59, 63) if d2[j] != base[j]] == [derived], ind
    # an unrelated sampled challenge (the old, wrong index 15) changes nothing derived
    s2 = list(sampled)
    s2[15] = xadd(s2[15], (1, 0, 0))
    assert S.derive_challenges(s2, claim)[59:] == base[59:]
    # the lookup terminal folds tip5::LOOKUP_TABLE from 1
    import tip5_ref as T
    assert base[61] == S.eval_arg_terminal(T.LOOKUP_TABLE, sampled[54])
