"""A small emulation of MATLAB ``textscan`` on a file identifier, enough to
run the reference's run.log readers unchanged (test infrastructure).

Semantics emulated (MATLAB documentation of ``textscan``):
* the file position persists between calls on the same fid;
* ``'HeaderLines', H`` skips the REMAINDER OF THE CURRENT LINE as the first
  header line, then H - 1 further lines;
* the format is applied ``N`` times (all repetitions that match when N is
  omitted); before each literal word and each numeric conversion,
  whitespace and end-of-line characters are skipped (the delimiter '\\n' of
  the readers is whitespace-like here);
* ``%d`` reads an integer, ``%f`` a floating-point number; a literal word
  must match exactly; a repetition that fails to match stops the scan with
  the position restored to where that repetition started.
"""
from __future__ import annotations

import re

_NUM = {"d": re.compile(r"[-+]?\d+"), "f": re.compile(r"[-+]?(\d+\.?\d*([eE][-+]?\d+)?|\.\d+([eE][-+]?\d+)?|Inf|NaN)")}


def _tokens(fmt):
    out = []
    for part in re.split(r"(%[df])", fmt):
        if part in ("%d", "%f"):
            out.append(("conv", part[1]))
        else:
            out.extend(("lit", w) for w in part.split())
    return out


class Fid:
    def __init__(self, text):
        self.text = text
        self.pos = 0

    def _skip_ws(self):
        while self.pos < len(self.text) and self.text[self.pos] in " \t\r\n\b":
            self.pos += 1

    def _skip_line(self):
        i = self.text.find("\n", self.pos)
        self.pos = len(self.text) if i < 0 else i + 1

    def textscan(self, fmt, N=None, headerlines=0):
        """Returns one list per conversion in ``fmt`` (MATLAB's cell array)."""
        if headerlines > 0:
            for _ in range(headerlines):
                self._skip_line()
        toks = _tokens(fmt)
        nconv = sum(1 for t in toks if t[0] == "conv")
        cols = [[] for _ in range(nconv)]
        rep = 0
        while N is None or rep < N:
            start = self.pos
            vals = []
            ok = True
            for kind, v in toks:
                self._skip_ws()
                if kind == "lit":
                    if self.text.startswith(v, self.pos):
                        self.pos += len(v)
                    else:
                        ok = False
                        break
                else:
                    m = _NUM[v].match(self.text, self.pos)
                    if not m:
                        ok = False
                        break
                    vals.append(int(m.group(0)) if v == "d" else float(m.group(0)))
                    self.pos = m.end()
            if not ok:
                self.pos = start
                break
            for c, x in zip(cols, vals):
                c.append(x)
            rep += 1
        return cols


def load_data_header(path):
    """analysis/load_data.m:14-27 (and symplectic_full_fourier.m:66-82's
    parse_data, the same five scans): Resolution, Npackets, f, Cg, Ug."""
    fid = Fid(open(path).read())
    resolution = fid.textscan("Resolution: %dx%d", 1, headerlines=10)
    npackets = fid.textscan("Number of packets: %d", 1)
    f = fid.textscan("Coriolis parameter: %f", headerlines=7)
    cg = fid.textscan("Group velocity: %f", 1)
    ug = fid.textscan("Background velocity (parameter,computed): (%f,%f)", 1)
    first = lambda c: c[0] if c else None  # noqa: E731  (MATLAB: an empty cell on a failed scan)
    return dict(resolution=(first(resolution[0]), first(resolution[1])), Npackets=first(npackets[0]),
                f=first(f[0]), Cg=first(cg[0]), Ug=(first(ug[0]), first(ug[1])))
