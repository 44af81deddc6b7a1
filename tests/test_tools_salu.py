"""tools/salu_lines.py's pieces that need no compiler: the instruction classes
(what SQ_INSTS_SALU counts and what it does not), the source-function map
(top-level functions and the Engine's indented methods) and the per-line tally
of a disassembly with line records."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import salu_lines as S  # noqa: E402


def test_instruction_classes():
    assert S.klass("s_add_u32") == "salu"
    assert S.klass("s_cselect_b64") == "salu"
    assert S.klass("s_waitcnt") == "other_s"
    assert S.klass("s_nop") == "other_s"
    assert S.klass("s_cbranch_scc1") == "branch"
    assert S.klass("s_branch") == "branch"
    assert S.klass("s_load_dwordx2") == "smem"
    assert S.klass("v_readlane_b32") == "valu"
    assert S.klass("ds_read_b128") == "lds"
    assert S.klass("global_load_lds_dwordx4") == "vmem"


def test_function_map(tmp_path):
    src = tmp_path / "k.hip"
    src.write_text("\n".join([
        "__device__ __forceinline__ int helper(int x) {",     # 1
        "    return x;",
        "}",
        "template <int NL, bool LH = false>",
        "struct Engine {",                                     # 5
        "    __device__ __forceinline__ int access(int core) {",
        "        return core;",
        "    }",
        "};",
        "__global__ void kern(int* p) {",                      # 10
        "    p[0] = 1;",
        "}",
    ]) + "\n")
    fns = S.functions(str(src))
    assert (1, "helper") in fns
    assert (6, "Engine::access") in fns
    assert (10, "kern") in fns


def test_tally_charges_instructions_to_lines():
    dis = "\n".join([
        "0000000000001000 <other>:",
        "; /x/engine.hip:5",
        "\ts_add_u32 s0, s1, s2",
        "0000000000002000 <pu_jit_uncore_s1_h0>:",
        "; /x/engine.hip:10",
        "\ts_add_u32 s0, s1, s2",
        "\tv_add_u32_e32 v0, v1, v2",
        "; /x/engine.hip:11",
        "\ts_waitcnt vmcnt(0)",
        "\ts_cbranch_scc1 3",
    ])
    per = S.tally(dis, "pu_jit_uncore_s1_h0")
    assert per[("engine.hip", 10)]["salu"] == 1
    assert per[("engine.hip", 10)]["valu"] == 1
    assert per[("engine.hip", 11)]["other_s"] == 1
    assert per[("engine.hip", 11)]["branch"] == 1
    assert ("engine.hip", 5) not in per     # another kernel's code
