"""ISA check of librod.so's gfx950 code objects: no VGPR that a buffer store reads (its data or
its address) is written within 5 wait states after the store, in ANY kernel.

Why: the compiler inserts the VALU-write-after-store wait state for a
>8-byte MUBUF store only when the store's SGPR offset is the constant 0.  librod's streaming
kernels carry the row in an SGPR offset (rod_common.h `buf_st`), and on the MI355X a VALU write
of the data registers right after such a store corrupted stored elements run to run.  `buf_st`
fences every store with `s_nop 4` between scheduling barriers; this test proves the fence (or
enough independent instructions) is there after every buffer store the compiler emitted —
including the non-zero-soffset stores of pwbwd.hip and any store a future kernel adds.

CPU only: the code objects are unbundled from the built library with llvm-objdump --offloading
(in a temporary directory) and disassembled; no kernel runs."""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

from rod import _abi

LLVM = '/opt/rocm/llvm/bin'
WINDOW = 5   # wait states after the store in which its VGPRs must not be written

_VREG = re.compile(r'^([va])(\d+)$')
_VRANGE = re.compile(r'^([va])\[(\d+):(\d+)\]$')


def _regs(tok):
    tok = tok.strip()
    m = _VRANGE.match(tok)
    if m:
        return {(m.group(1), i) for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = _VREG.match(tok)
    if m:
        return {(m.group(1), int(m.group(2)))}
    return set()


def _written(mnem, ops):
    """VGPRs / AGPRs an instruction writes: the first operand of a VALU op or of anything that
    returns data into vector registers (loads, LDS reads, permutes); stores write none."""
    if not ops or mnem.startswith('s_'):
        return set()
    if 'store' in mnem or mnem.startswith('ds_write') or mnem.startswith('exp'):
        return set()
    if mnem.startswith('v_cmp') or mnem.startswith('v_readlane') or mnem.startswith('v_readfirstlane'):
        return set()    # SGPR / VCC destinations
    return _regs(ops[0])


def _code_objects(tmp):
    so = os.path.join(tmp, 'librod.so')
    shutil.copy(_abi.LIB_PATH, so)
    subprocess.run([os.path.join(LLVM, 'llvm-objdump'), '--offloading', so], cwd=tmp, check=True,
                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    return sorted(os.path.join(tmp, f) for f in os.listdir(tmp) if f.endswith('gfx950'))


def _instructions(path):
    out = subprocess.run([os.path.join(LLVM, 'llvm-objdump'), '-d', '--mcpu=gfx950', '--no-show-raw-insn', path],
                         check=True, capture_output=True, text=True).stdout
    fn, body = None, []
    for line in out.splitlines():
        m = re.match(r'^[0-9a-f]+ <(.+)>:$', line)
        if m:
            if fn is not None:
                yield fn, body
            fn, body = m.group(1), []
            continue
        t = line.split('//')[0].strip()
        if fn is None or not t or t.endswith(':') or t.startswith('.'):
            continue
        body.append(t)
    if fn is not None:
        yield fn, body


def scan(instrs, window=WINDOW):
    """[(store, offending instruction, wait states before it)] for one function's instructions.
    The window follows the fall-through path; a branch or s_endpgm inside it ends the scan
    conservatively as a finding unless the window was already covered."""
    bad = []
    for i, ins in enumerate(instrs):
        mnem, _, rest = ins.partition(' ')
        if not mnem.startswith('buffer_store'):
            continue
        ops = [o.strip() for o in rest.split(',')]
        regs = _regs(ops[0]) | (_regs(ops[1]) if len(ops) > 1 else set())
        ws = 0
        for nxt in instrs[i + 1:]:
            if ws >= window:
                break
            m2, _, r2 = nxt.partition(' ')
            m = re.match(r's_nop\s+(0x[0-9a-f]+|\d+)', nxt)
            if m:
                ws += int(m.group(1), 0) + 1
                continue
            if m2.startswith('s_branch') or m2.startswith('s_cbranch') or m2 in ('s_endpgm', 's_setpc_b64'):
                bad.append((ins, nxt, ws))
                break
            if _written(m2, [o.strip() for o in r2.split(',')]) & regs:
                bad.append((ins, nxt, ws))
                break
            ws += 1
    return bad


def test_scan_flags_a_hazard_and_passes_a_fence():
    """The scanner itself: a VALU write of the data registers in the next instruction is found;
    the same write behind s_nop 4 is not; an address-register write is found too."""
    hot = ['buffer_store_dwordx4 v[4:7], v1, s[8:11], s2 offen', 'v_mov_b32_e32 v5, 0']
    assert len(scan(hot)) == 1
    fenced = ['buffer_store_dwordx4 v[4:7], v1, s[8:11], s2 offen', 's_nop 4', 'v_mov_b32_e32 v5, 0']
    assert scan(fenced) == []
    addr = ['buffer_store_dword v4, v1, s[8:11], 0 offen', 'v_add_u32_e32 v2, 4, v2', 'v_add_u32_e32 v1, 4, v1']
    assert len(scan(addr)) == 1
    far = ['buffer_store_dwordx2 v[4:5], v1, s[8:11], s2 offen'] + ['v_add_u32_e32 v9, 1, v9'] * 5 + \
          ['v_mov_b32_e32 v4, 0']
    assert scan(far) == []


@pytest.mark.skipif(not os.path.exists(os.path.join(LLVM, 'llvm-objdump')), reason='no llvm-objdump in this image')
def test_no_vgpr_write_within_window_of_any_buffer_store():
    if not os.path.exists(_abi.LIB_PATH):
        pytest.skip('librod.so not built')
    with tempfile.TemporaryDirectory() as tmp:
        cos = _code_objects(tmp)
        assert cos, 'no gfx950 code object in librod.so'
        stores, wide, findings, kernels = 0, 0, [], set()
        for co in cos:
            for fn, body in _instructions(co):
                n = sum(1 for t in body if t.startswith('buffer_store'))
                if not n:
                    continue
                kernels.add(fn)
                stores += n
                wide += sum(1 for t in body if re.match(r'buffer_store_dwordx[34]\b', t))
                findings += [(fn, s, o, w) for s, o, w in scan(body)]
    # the streaming kernels (depthwise, pw backward, GEMM epilogues) use buffer stores: the scan
    # must actually have seen them, including the >8-byte form the hazard is about
    assert stores >= 500 and wide >= 100, (stores, wide)
    assert any('pw_bwd' in k for k in kernels) and any('dw3x3' in k for k in kernels)
    assert not findings, '\n'.join(f'{fn[:80]}: {s} -> {o} after {w} wait states' for fn, s, o, w in findings[:20])
