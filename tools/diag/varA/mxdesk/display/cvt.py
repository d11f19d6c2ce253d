"""VESA CVT modeline generator.

The reference builds a reduced-blanking modeline with ``cvt -r W H R`` for a monitor-less
GPU (entrypoint.sh:100) and injects it into xorg.conf (entrypoint.sh:106).  ``cvt``/``xcvt``
are not in this image, so this is an independent implementation of the VESA Coordinated
Video Timings v1.1 formulas (normal and reduced blanking), matching ``cvt`` output, e.g.
``cvt -r 1920 1080 60`` -> ``Modeline "1920x1080R"  138.50  1920 1968 2000 2080  1080 1083
1088 1111 +hsync -vsync``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

CELL_GRAN = 8
MIN_V_PORCH = 3  # lines
MIN_V_BPORCH = 6  # lines (reduced blanking)
# normal blanking
MIN_VSYNC_BP = 550.0  # us
H_SYNC_PER = 0.08
C_PRIME = 30.0  # (C - J) * K / 256 + J with C=40, J=20, K=128
M_PRIME = 300.0  # K / 256 * M with M=600, K=128
# reduced blanking
RB_MIN_V_BLANK = 460.0  # us
RB_H_BLANK = 160
RB_H_SYNC = 32
RB_V_FPORCH = 3
CLOCK_STEP = 0.25  # MHz


def _vsync_for_aspect(w: int, h: int) -> int:
    if h * 4 // 3 == w and w % 4 == 0 or w * 3 == h * 4:
        return 4
    if w * 9 == h * 16:
        return 5
    if w * 10 == h * 16:
        return 6
    if w * 4 == h * 5:
        return 7
    if w * 9 == h * 15:
        return 7
    return 10


@dataclass
class Modeline:
    name: str
    clock_mhz: float
    hdisplay: int
    hsync_start: int
    hsync_end: int
    htotal: int
    vdisplay: int
    vsync_start: int
    vsync_end: int
    vtotal: int
    hsync_pos: bool
    vsync_pos: bool
    interlaced: bool = False

    @property
    def refresh_hz(self) -> float:
        return self.clock_mhz * 1e6 / (self.htotal * self.vtotal)

    def xorg(self) -> str:
        flags = ("+hsync" if self.hsync_pos else "-hsync") + " " + ("+vsync" if self.vsync_pos else "-vsync")
        if self.interlaced:
            flags += " Interlace"
        return (f'Modeline "{self.name}"  {self.clock_mhz:.2f}  {self.hdisplay} {self.hsync_start} {self.hsync_end} '
                f"{self.htotal}  {self.vdisplay} {self.vsync_start} {self.vsync_end} {self.vtotal} {flags}")


def cvt(width: int, height: int, refresh: float = 60.0, reduced: bool = True, interlaced: bool = False) -> Modeline:
    """Compute a CVT v1.1 mode.  ``reduced=True`` mirrors ``cvt -r``."""
    if width <= 0 or height <= 0 or refresh <= 0:
        raise ValueError("width, height and refresh must be positive")
    hpix = (width // CELL_GRAN) * CELL_GRAN
    vlines = height // 2 if interlaced else height
    field_rate = refresh * 2 if interlaced else refresh
    interlace = 0.5 if interlaced else 0.0
    vsync = _vsync_for_aspect(width, height)
    if reduced:
        h_period_est = ((1_000_000.0 / field_rate) - RB_MIN_V_BLANK) / (vlines + interlace)
        vbi_lines = int(RB_MIN_V_BLANK / h_period_est) + 1
        rb_min_vbi = RB_V_FPORCH + vsync + MIN_V_BPORCH
        act_vbi = max(vbi_lines, rb_min_vbi)
        total_v = act_vbi + vlines + interlace
        total_pix = RB_H_BLANK + hpix
        clock = CLOCK_STEP * math.floor((field_rate * total_v * total_pix / 1_000_000.0) / CLOCK_STEP)
        hsync_end = hpix + RB_H_BLANK // 2
        hsync_start = hsync_end - RB_H_SYNC
        vsync_start = height + RB_V_FPORCH
        vsync_end = vsync_start + vsync
        name = f"{width}x{height}R" + ("i" if interlaced else "")
        return Modeline(name, clock, hpix, hsync_start, hsync_end, total_pix, height, vsync_start, vsync_end,
                        int(total_v * (2 if interlaced else 1)), True, False, interlaced)
    h_period_est = ((1.0 / field_rate) - MIN_VSYNC_BP / 1_000_000.0) / (vlines + MIN_V_PORCH + interlace) * 1_000_000.0
    vsync_bp = int(MIN_VSYNC_BP / h_period_est) + 1
    if vsync_bp < vsync + MIN_V_PORCH:
        vsync_bp = vsync + MIN_V_PORCH
    total_v = vlines + vsync_bp + interlace + MIN_V_PORCH
    ideal_duty = C_PRIME - (M_PRIME * h_period_est / 1000.0)
    if ideal_duty < 20:
        ideal_duty = 20
    h_blank = int(hpix * ideal_duty / (100.0 - ideal_duty) / (2 * CELL_GRAN)) * (2 * CELL_GRAN)
    total_pix = hpix + h_blank
    clock = CLOCK_STEP * math.floor((total_pix / h_period_est) / CLOCK_STEP)
    h_sync = int(H_SYNC_PER * total_pix / CELL_GRAN) * CELL_GRAN
    hsync_end = hpix + h_blank // 2
    hsync_start = hsync_end - h_sync
    vsync_start = height + MIN_V_PORCH
    vsync_end = vsync_start + vsync
    name = f"{width}x{height}_{refresh:.2f}" + ("i" if interlaced else "")
    return Modeline(name, clock, hpix, hsync_start, hsync_end, total_pix, height, vsync_start, vsync_end,
                    int(total_v * (2 if interlaced else 1)), False, True, interlaced)


def main(argv: list[str] | None = None) -> None:
    """``python -m mxdesk.display.cvt [-r] W H [R]`` -- prints like ``cvt``."""
    import sys

    args = list(sys.argv[1:] if argv is None else argv)
    reduced = "-r" in args or "--reduced" in args
    args = [a for a in args if not a.startswith("-")]
    w, h = int(args[0]), int(args[1])
    r = float(args[2]) if len(args) > 2 else 60.0
    m = cvt(w, h, r, reduced=reduced)
    print(f"# {w}x{h} {m.refresh_hz:.2f} Hz ({'CVT RB' if reduced else 'CVT'}) hsync: "
          f"{m.clock_mhz * 1000 / m.htotal:.2f} kHz; pclk: {m.clock_mhz:.2f} MHz")
    print(m.xorg())


if __name__ == "__main__":
    main()
