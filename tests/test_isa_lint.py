"""scripts/isa_reload_lint.py, the static check for the round-6 miscompile (a 12-byte folded
reload whose fourth dword is then read without being restored), on ISA excerpts
of the D 64 one-lane kD kernel that hit it: the compiler's own reload-reuse pattern passes, the
miscompiled final-state reload is flagged."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import isa_reload_lint as L  # noqa: E402

GOOD = """_kernel:
	v_accvgpr_read_b32 v9, a205             ;  Reload Reuse
	scratch_load_dwordx3 v[6:8], off, off offset:2144 ; 12-byte Folded Reload
	s_waitcnt vmcnt(0)
	v_add_f64 v[20:21], v[8:9], -v[18:19]
	s_endpgm
"""
BAD = """_kernel:
	global_load_dwordx4 a[136:139], v[64:65], off offset:64
	v_mov_b32_e32 v4, 0x198
	s_nop 0
	v_mov_b32_e32 v5, 0x198
	s_nop 0
	scratch_load_dwordx3 a[136:138], off, off offset:2144 ; 12-byte Folded Reload
	scratch_load_dwordx4 a[132:135], off, off offset:2160 ; 16-byte Folded Reload
	s_waitcnt vmcnt(0)
	global_store_dwordx2 v[2:3], a[136:137], off
	global_store_dwordx2 v[2:3], a[138:139], off
	s_endpgm
"""
REWRITTEN = BAD.replace("\tglobal_store_dwordx2 v[2:3], a[136:137], off\n",
                        "\tv_accvgpr_mov_b32 a139, a205\n\tglobal_store_dwordx2 v[2:3], a[136:137], off\n")


def _scan(tmp_path, text):
    f = tmp_path / "k.s"
    f.write_text(text)
    return L.scan(str(f))


def test_reload_reuse_pattern_passes(tmp_path):
    assert _scan(tmp_path, GOOD) == []


def test_stale_fourth_dword_is_flagged(tmp_path):
    hits = _scan(tmp_path, BAD)
    assert len(hits) == 1 and "a[138:139]" in hits[0][3]


def test_fourth_dword_written_after_the_reload_passes(tmp_path):
    assert _scan(tmp_path, REWRITTEN) == []


def test_register_parser():
    assert L.regs("a[136:139]") == {("a", 136), ("a", 137), ("a", 138), ("a", 139)}
    assert L.regs("v9") == {("v", 9)} and L.regs("s[0:1]") == set()
