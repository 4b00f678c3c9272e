#!/usr/bin/env python3
"""Build oracle/_ref/libref_tristan.so: the reference's own TRISTAN decode,
compiled verbatim (TEST INFRASTRUCTURE ONLY -- the checker, never shipped).

src/tristan.c cannot be compiled whole here: it includes src/dqdk.h, which
needs libbpf/libxdp headers this image lacks.  The decode
path itself needs none of that, so this recipe extracts, at build time and
by name pattern (not line numbers), the exact text of:

  src/tristan.h                 struct energy_evt + tristan_energy_evt_t
                                (:13-27), the histogram geometry macros
                                (:53-60, :95), tristan_mode_t (:62-67),
                                chnl_t / tristan_histo_t (:71-77), tristan_t
                                (:79-93)
  src/dqdk-async-processor.h    the opaque `typedef struct dqdk_async_processor
                                dqdk_async_processor_t;` tristan_t points to (:10)
  src/tristan.c                 is_store_histo (:65-70),
                                get_energy_events_count (:72-85),
                                histogram_event (:233-245),
                                process_events_unrolled16 (:247-304),
                                SWEETSPOT_BATCHSZ (:306), tristan_process (:308-330)

into a translation unit under /tmp that includes the reference's own
src/ctypes.h and src/dlog.h (-I<ref>/src) and libc headers -- no stand-in
headers or types -- plus a thin `rt_*` C wrapper layer (below) so ctypes can
call the static functions.  The extracted text never enters the repository:
only this recipe does; the .so goes to oracle/_ref/ (git-ignored).

get_udp_payload / process_frame / fetch_xsk (src/dqdk.c) are NOT built:
their only type, dqdk_worker_t (src/dqdk.h:87-105), embeds libxdp ring
structs, so they would need stand-ins (their composition
stays a restatement, with every verdict-deciding call pinned).
"""
from __future__ import annotations

import argparse
import os
import re
import subprocess
import sys
import tempfile
from pathlib import Path

HERE = Path(__file__).resolve().parent


def _block_ending(text: str, end_name: str) -> str:
    """`typedef struct|enum { ... } <end_name>;` -- the block whose closing
    line names end_name, from the nearest preceding `typedef ... {`."""
    m = re.search(r"^\}\s*" + re.escape(end_name) + r"\s*;[^\n]*$", text, re.M)
    if not m:
        raise SystemExit(f"extract: no block ending in {end_name}")
    start = text.rfind("typedef", 0, m.start())
    if start < 0:
        raise SystemExit(f"extract: no typedef before {end_name}")
    return text[start:m.end()]


def _struct(text: str, tag: str) -> str:
    """`struct <tag> { ... } <attrs>;`"""
    m = re.search(r"^struct\s+" + re.escape(tag) + r"\s*\{", text, re.M)
    if not m:
        raise SystemExit(f"extract: no struct {tag}")
    end = re.compile(r"^\}[^\n]*;[^\n]*$", re.M).search(text, m.end())
    return text[m.start():end.end()]


def _line(text: str, pattern: str) -> str:
    m = re.search(pattern, text, re.M)
    if not m:
        raise SystemExit(f"extract: no line matching {pattern!r}")
    return m.group(0)


def _function(text: str, name: str) -> str:
    """A top-level function definition `static ... name(...) { ... }`."""
    m = re.search(r"^static\b[^\n;]*\b" + re.escape(name) + r"\s*\([^;{]*\)\s*\{", text, re.M)
    if not m:
        raise SystemExit(f"extract: no function {name}")
    depth, i = 0, text.index("{", m.start())
    while True:
        c = text[i]
        if c == "{":
            depth += 1
        elif c == "}":
            depth -= 1
            if depth == 0:
                return text[m.start():i + 1]
        i += 1


MACROS = ("TRISTAN_HISTO_EVT_SZ", "HISTO_BINS", "CHANNELHISTO_COUNT", "TILECHNLS_COUNT", "TILES_COUNT",
          "CHNLS_COUNT", "HISTO_MAXVAL", "TRISTAN_HISTO_SZ")
FUNCTIONS = ("is_store_histo", "get_energy_events_count", "histogram_event", "process_events_unrolled16",
             "tristan_process")

# Thin wrappers: give the static reference functions external names and hand
# tristan_process a tristan_t set up the way tristan_init leaves it for the
# fields the sync path reads (mode, payloadsz, histo, histo_fd, rawdata_fd,
# the two atomics).  No reference logic lives here.
WRAPPERS = r"""
#include <stddef.h>
size_t rt_sizeof_energy_evt(void) { return sizeof(tristan_energy_evt_t); }
unsigned long long rt_histo_sz(void) { return (unsigned long long)TRISTAN_HISTO_SZ; }
int rt_chnls_count(void) { return CHNLS_COUNT; }
int rt_is_store_histo(int mode) { return is_store_histo((tristan_mode_t)mode); }
u32 rt_get_energy_events_count(int mode, u32 payloadsz) { return get_energy_events_count((tristan_mode_t)mode, payloadsz); }
int rt_histogram_event(tristan_histo_t* histo, u8* evt) { return histogram_event(histo, (tristan_energy_evt_t*)evt); }
int rt_tristan_process(int mode, u32 payloadsz, tristan_histo_t* histo, int histo_fd, int rawdata_fd,
                       u8* buffer, u32 len, u32 burst, u64* total_events, u64* total_bytes)
{
    static tristan_t t;
    memset(&t, 0, sizeof(t));
    t.mode = (tristan_mode_t)mode;
    t.payloadsz = payloadsz;
    t.histo = histo;
    t.histo_fd = histo_fd;
    t.rawdata_fd = rawdata_fd;
    atomic_init(&t.total_events, *total_events);
    atomic_init(&t.total_bytes, *total_bytes);
    int ret = tristan_process(&t, buffer, len, burst);
    *total_events = atomic_load(&t.total_events);
    *total_bytes = atomic_load(&t.total_bytes);
    return ret;
}
void rt_flush_stdout(void) { fflush(stdout); }
"""


def harness_source(ref: Path) -> str:
    src = ref / "src"
    th = (src / "tristan.h").read_text()
    tc = (src / "tristan.c").read_text()
    ah = (src / "dqdk-async-processor.h").read_text()
    parts = [
        "/* generated by oracle/ref_tristan.py from " + str(src) + " -- extracted verbatim, see the recipe */",
        "#define _GNU_SOURCE",
        "#include <stdatomic.h>",
        "#include <stdio.h>",
        "#include <string.h>",
        "#include <unistd.h>",
        "#include <time.h>",
        "#include <linux/limits.h>",
        '#include "ctypes.h"',
        '#include "dlog.h"',
        _line(ah, r"^typedef\s+struct\s+dqdk_async_processor\s+dqdk_async_processor_t\s*;.*$"),
        _struct(th, "energy_evt"),
        _line(th, r"^typedef\s+struct\s+energy_evt\s+tristan_energy_evt_t\s*;.*$"),
    ]
    for mname in MACROS:
        parts.append(_line(th, r"^#define\s+" + mname + r"\b.*$"))
    parts += [_block_ending(th, "tristan_mode_t"), _block_ending(th, "chnl_t"),
              _block_ending(th, "tristan_histo_t"), _block_ending(th, "tristan_t")]
    parts.append(_line(tc, r"^#define\s+SWEETSPOT_BATCHSZ\b.*$"))
    for f in FUNCTIONS:
        parts.append(_function(tc, f))
    parts.append(WRAPPERS)
    return "\n\n".join(parts) + "\n"


def build(ref: Path, out: Path, cc: str = "gcc") -> Path:
    out.parent.mkdir(parents=True, exist_ok=True)
    with tempfile.TemporaryDirectory(prefix="dqdk_ref_tristan_") as tmp:
        c = Path(tmp) / "ref_tristan.c"
        c.write_text(harness_source(ref))
        # src/Makefile:13 flags minus -march=native (the .so must load on any x86-64 host)
        cmd = [cc, "-O3", "-g", "-std=gnu11", "-fPIC", "-shared", "-I", str(ref / "src"), "-o", str(out), str(c)]
        print("+", " ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default=os.environ.get("DQDK_REFERENCE", "/root/reference"))
    ap.add_argument("--out", default=str(HERE / "_ref" / "libref_tristan.so"))
    ap.add_argument("--print", action="store_true", help="print the generated TU instead of building")
    a = ap.parse_args()
    ref = Path(a.ref)
    if not (ref / "src" / "tristan.c").exists():
        print(f"{ref}/src/tristan.c not found: reference absent, nothing built", file=sys.stderr)
        return 1
    if a.print:
        sys.stdout.write(harness_source(ref))
        return 0
    build(ref, Path(a.out))
    return 0


if __name__ == "__main__":
    sys.exit(main())
