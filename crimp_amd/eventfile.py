"""Event-file ingestion without astropy.

A minimal FITS binary-table reader sufficient for the X-ray event files CRIMP
consumes, restating the parts of CRIMP v2.3.0 ``eventfile.py`` on the ToA path:
  * ``readEF``              header keywords, MJDREF = MJDREFI + MJDREFF or MJDREF (:72-146)
  * ``readGTI``             GTI START/STOP -> MJD                              (:188-236)
  * ``build_time_energy_df`` TIME/86400 + MJDREF and PI -> keV per telescope (:238-280)
  * ``filtenergy``          inclusive energy cut (pandas ``between``)         (:282-298)
  * ``filttime``            inclusive time cut                                (:300-316)
  * ``addphasecolEF``       PHASE column from calcphase on the device, the EVENTS table rewritten in place
                            (and optionally a non-barycentred file's) (:319-375); ``main`` = ``addphasecolumn`` (:378)
The conversions keep the reference's operation order (``TIME / 86400 + MJDREF``,
``PI * 0.01`` for NICER/SWIFT) so the MJDs are bit-identical to the astropy path.
"""
import argparse
import os
import re

import numpy as np

# column keywords of a binary table header card (TTYPEn ... TDIMn): the new column's cards follow the last of them
_COLKEY = re.compile(r"T(TYPE|FORM|UNIT|ZERO|SCAL|DISP|NULL|DIM)\d+")

_CODES = {"L": ("u1", 1), "B": ("u1", 1), "I": (">i2", 2), "J": (">i4", 4), "K": (">i8", 8), "E": (">f4", 4),
          "D": (">f8", 8), "A": ("S1", 1)}


def _parse_card_value(v):
    v = v.strip()
    if v.startswith("'"):
        return v[1:v.rfind("'")].strip()
    if v in ("T", "F"):
        return v == "T"
    try:
        return int(v)
    except ValueError:
        try:
            return float(v.replace("D", "E"))
        except ValueError:
            return v


def read_fits(path):
    """List of (header dict, data bytes view offset, data size) for every HDU."""
    buf = np.fromfile(path, dtype=np.uint8)
    raw = buf.tobytes()
    pos, hdus = 0, []
    while pos + 2880 <= len(raw):
        hdr = {}
        done = False
        while not done:
            block = raw[pos:pos + 2880].decode("ascii", errors="replace")
            pos += 2880
            for i in range(0, 2880, 80):
                card = block[i:i + 80]
                key = card[:8].strip()
                if key == "END":
                    done = True
                    break
                if card[8:10] == "= ":
                    val = card[10:]
                    # strip a trailing comment outside quotes
                    if val.strip().startswith("'"):
                        q = val.find("'", val.find("'") + 1)
                        while q + 1 < len(val) and val[q + 1] == "'":
                            q = val.find("'", q + 2)
                        val = val[:q + 1]
                    else:
                        val = val.split("/")[0]
                    hdr[key] = _parse_card_value(val)
            if pos >= len(raw):
                break
        naxis = int(hdr.get("NAXIS", 0))
        size = 0
        if naxis:
            size = abs(int(hdr.get("BITPIX", 8))) // 8
            for a in range(1, naxis + 1):
                size *= int(hdr.get("NAXIS%d" % a, 0))
            size += int(hdr.get("PCOUNT", 0))
        hdus.append((hdr, pos, size))
        pos += ((size + 2879) // 2880) * 2880
    return raw, hdus


def read_table(raw, hdr, start):
    """Columns of a BINTABLE HDU as numpy arrays (TZERO/TSCAL applied like astropy)."""
    width, nrow = int(hdr["NAXIS1"]), int(hdr["NAXIS2"])
    rows = np.frombuffer(raw, dtype=np.uint8, count=width * nrow, offset=start).reshape(nrow, width)
    cols, off = {}, 0
    for c in range(1, int(hdr["TFIELDS"]) + 1):
        form = str(hdr["TFORM%d" % c]).strip()
        i = 0
        while i < len(form) and form[i].isdigit():
            i += 1
        rep = int(form[:i]) if i else 1
        code = form[i]
        name = str(hdr.get("TTYPE%d" % c, "COL%d" % c)).strip()
        if code == "X":  # bit array -> bool[rep] per row, as astropy returns it
            nbytes = (rep + 7) // 8
            bits = np.unpackbits(rows[:, off:off + nbytes], axis=1)[:, :rep].astype(bool)
            cols[name] = bits.ravel() if rep == 1 else bits
            off += nbytes
            continue
        if code == "L":  # logical 'T'/'F' bytes -> bool
            lg = rows[:, off:off + rep] == ord("T")
            cols[name] = lg.ravel() if rep == 1 else lg
            off += rep
            continue
        dt, sz = _CODES[code]
        nbytes = sz * rep
        blob = rows[:, off:off + nbytes].copy()
        off += nbytes
        if code == "A":
            arr = blob.view("S%d" % rep).ravel()
        else:
            arr = blob.view(dt)
            arr = arr.ravel() if rep == 1 else arr.reshape(nrow, rep)
            arr = arr.astype(arr.dtype.newbyteorder("=")) if arr.dtype.byteorder == ">" else arr
            zero = hdr.get("TZERO%d" % c)
            scale = hdr.get("TSCAL%d" % c)
            if zero is not None or scale is not None:
                arr = arr * (1.0 if scale is None else float(scale)) + (0.0 if zero is None else float(zero))
        cols[name] = arr
    return cols


class EvtFileOps:
    """Event-file operations on the ToA path (eventfile.py:33)."""

    def __init__(self, evtFile):
        self.evtFile = evtFile
        self.time_energy_df = None
        self._raw, self._hdus = read_fits(evtFile)

    def _hdu(self, name):
        for hdr, start, _ in self._hdus:
            if str(hdr.get("EXTNAME", "")).strip() == name:
                return hdr, start
        raise KeyError("no %s extension in %s" % (name, self.evtFile))

    def readEF(self):
        hdr, _ = self._hdu("EVENTS")
        if "MJDREFI" in hdr:
            mjdref = hdr["MJDREFI"] + hdr["MJDREFF"]
        elif "MJDREF" in hdr:
            mjdref = hdr["MJDREF"]
        else:
            raise KeyError("No reference time in event file, need either MJDREFI or MJDREF keywords")
        return {"TELESCOPE": hdr.get("TELESCOP"), "INSTRUME": hdr.get("INSTRUME"), "OBS_ID": hdr.get("OBS_ID"),
                "TSTART": hdr.get("TSTART"), "TSTOP": hdr.get("TSTOP"), "LIVETIME": hdr.get("LIVETIME"),
                "ONTIME": hdr.get("ONTIME"), "TIMESYS": hdr.get("TIMESYS"), "MJDREF": mjdref,
                "TIMEZERO": hdr.get("TIMEZERO"), "DATEOBS": hdr.get("DATE-OBS"), "DETNAME": hdr.get("DETNAM"),
                "DATATYPE": hdr.get("DATATYPE"), "CCDSRC": hdr.get("CCDSRC")}

    def readGTI(self):
        kw = self.readEF()
        name = "GTI"
        if kw["TELESCOPE"] == "XMM":
            ccd = int(kw["CCDSRC"])
            name = ("STDGTI0%d" % ccd) if ccd < 10 else ("STDGTI%d" % ccd)
        hdr, start = self._hdu(name)
        cols = read_table(self._raw, hdr, start)
        gti = np.vstack((cols["START"], cols["STOP"])).T
        return kw, gti / 86400 + kw["MJDREF"]

    def build_time_energy_df(self):
        import pandas as pd
        kw = self.readEF()
        hdr, start = self._hdu("EVENTS")
        cols = read_table(self._raw, hdr, start)
        tel = kw["TELESCOPE"]
        if tel == "GLAST":
            df = pd.DataFrame(np.vstack((cols["TIME"], cols["PHA"])).T, columns=["TIME", "PHA"])
        else:
            df = pd.DataFrame(np.vstack((cols["TIME"], cols["PI"])).T, columns=["TIME", "PI"])
            if tel in ("NICER", "SWIFT"):
                df["PI"] *= 0.01
            elif tel == "NuSTAR":
                df["PI"] = (df["PI"] * 0.04) + 1.6
            elif tel == "XMM":
                df["PI"] *= 0.001
            elif tel == "IXPE":
                df["PI"] *= 0.04
        df["TIME"] = df["TIME"] / 86400 + kw["MJDREF"]
        self.time_energy_df = df
        return self

    def filtenergy(self, eneLow, eneHigh):
        if self.time_energy_df is None:
            raise Exception("TIME ENERGY dataframe is empty - please run build_time_energy_df method first ")
        if "PI" not in self.time_energy_df.columns:
            raise Exception("NO PI column name to filter against ")
        mask = self.time_energy_df["PI"].between(eneLow, eneHigh)
        self.time_energy_df = self.time_energy_df.loc[mask].copy()
        return self

    def filttime(self, t_start=None, t_end=None):
        if self.time_energy_df is None:
            raise Exception("TIME ENERGY dataframe is empty - please run build_time_energy_df method first ")
        lo = -np.inf if t_start is None else t_start
        hi = np.inf if t_end is None else t_end
        mask = self.time_energy_df["TIME"].between(lo, hi)
        self.time_energy_df = self.time_energy_df.loc[mask].copy()
        return self

    def addphasecolEF(self, timMod, nonBaryEvtFile=None):
        """PHASE column (cycle-folded phase of TIME / 86400 + MJDREF under ``timMod``, calcphase.py:152-176 on the
        device) appended to the EVENTS table of this file, and to that of ``nonBaryEvtFile`` when given
        (eventfile.py:319-375). Returns the header keywords (readEF)."""
        from .calcphase import calcphase
        kw = self.readEF()
        hdr, start = self._hdu("EVENTS")
        cols = read_table(self._raw, hdr, start)
        timeMJD = cols["TIME"] / 86400 + kw["MJDREF"]
        _, folded = calcphase(timeMJD, timMod)
        add_column(self.evtFile, "EVENTS", "PHASE", np.asarray(folded, dtype=np.float64))
        if nonBaryEvtFile is not None:
            add_column(nonBaryEvtFile, "EVENTS", "PHASE", np.asarray(folded, dtype=np.float64))
        self._raw, self._hdus = read_fits(self.evtFile)
        return kw

    def read_fpmsel(self):
        """NICER FPM_SEL extension condensed to selected / on detector counts per time stamp
        (eventfile.py:149-183): DataFrame TIME (MJD), TOTFPMSEL, TOTFPMON."""
        import pandas as pd
        kw = self.readEF()
        if kw["TELESCOPE"] != "NICER":
            raise ValueError("No FPM selection is possible for non-NICER observations")
        hdr, start = self._hdu("FPM_SEL")
        cols = read_table(self._raw, hdr, start)
        time = cols["TIME"] / 86400 + kw["MJDREF"]
        sel = np.asarray(cols["FPM_SEL"]).reshape(len(time), -1).sum(axis=1).astype(np.float64)
        on = np.asarray(cols["FPM_ON"]).reshape(len(time), -1).sum(axis=1).astype(np.float64)
        table = pd.DataFrame({"TIME": time, "FPM_SEL": list(cols["FPM_SEL"]), "FPM_ON": list(cols["FPM_ON"])})
        condensed = pd.DataFrame(np.vstack((time, sel, on)).T, columns=["TIME", "TOTFPMSEL", "TOTFPMON"])
        return table, condensed


def _card(k, v):
    if isinstance(v, str):
        return ("%-8s= '%-8s'" % (k, v)).ljust(80)
    if isinstance(v, bool):
        return ("%-8s= %20s" % (k, "T" if v else "F")).ljust(80)
    return ("%-8s= %20s" % (k, repr(v) if isinstance(v, float) else v)).ljust(80)


def _block(cards):
    s = "".join(cards) + "END".ljust(80)
    s = s.ljust(((len(s) + 2879) // 2880) * 2880)
    return s.encode("ascii")


def write_fits(path, tables, primary=None):
    """Write BINTABLE extensions: ``tables`` is a list of (extname, [(col, tform, array)], {keyword: value}).
    Supports D/E/J/I/B/K scalars or vectors and L (bool) vectors -- enough for test inputs."""
    out = [_block([_card("SIMPLE", True), _card("BITPIX", 8), _card("NAXIS", 0), _card("EXTEND", True)]
                  + [_card(k, v) for k, v in (primary or {}).items()])]
    codes = {"D": ">f8", "E": ">f4", "J": ">i4", "I": ">i2", "B": "u1", "K": ">i8", "L": "S1"}
    for extname, cols, kws in tables:
        n = len(cols[0][2])
        fields = []
        for name, tform, arr in cols:
            rep = int(tform[:-1] or 1)
            code = tform[-1]
            fields.append((name, codes[code], (rep,)) if rep > 1 else (name, codes[code]))
        rec = np.zeros(n, dtype=fields)
        for name, tform, arr in cols:
            a = np.asarray(arr)
            rec[name] = np.where(a, b"T", b"F") if tform[-1] == "L" else a
        cards = [_card("XTENSION", "BINTABLE"), _card("BITPIX", 8), _card("NAXIS", 2),
                 _card("NAXIS1", rec.dtype.itemsize), _card("NAXIS2", n), _card("PCOUNT", 0), _card("GCOUNT", 1),
                 _card("TFIELDS", len(cols)), _card("EXTNAME", extname)]
        for i, (name, tform, _) in enumerate(cols, start=1):
            cards += [_card("TTYPE%d" % i, name), _card("TFORM%d" % i, tform)]
        cards += [_card(k, v) for k, v in kws.items()]
        data = rec.tobytes()
        out += [_block(cards), data + b"\0" * (((len(data) + 2879) // 2880) * 2880 - len(data))]
    with open(path, "wb") as fh:
        fh.write(b"".join(out))


def write_events_fits(path, time, pi, mjdrefi, mjdreff, telescope="NICER"):
    """Write a minimal EVENTS (TIME 1D, PI 1I) FITS file -- used by the tests to round-trip the reader."""
    def card(k, v, quote=False):
        vs = ("'%-8s'" % v) if quote else str(v)
        return ("%-8s= %20s" % (k, vs) if not quote else "%-8s= %s" % (k, vs)).ljust(80)

    def block(cards):
        s = "".join(cards) + "END".ljust(80)
        s = s.ljust(((len(s) + 2879) // 2880) * 2880)
        return s.encode("ascii")
    prim = block([card("SIMPLE", "T"), card("BITPIX", 8), card("NAXIS", 0), card("EXTEND", "T")])
    n = len(time)
    ext = block([card("XTENSION", "BINTABLE", True), card("BITPIX", 8), card("NAXIS", 2), card("NAXIS1", 10),
                 card("NAXIS2", n), card("PCOUNT", 0), card("GCOUNT", 1), card("TFIELDS", 2),
                 card("EXTNAME", "EVENTS", True), card("TTYPE1", "TIME", True), card("TFORM1", "1D", True),
                 card("TTYPE2", "PI", True), card("TFORM2", "1I", True), card("TELESCOP", telescope, True),
                 card("MJDREFI", int(mjdrefi)), card("MJDREFF", repr(float(mjdreff)))])
    rec = np.zeros(n, dtype=[("TIME", ">f8"), ("PI", ">i2")])
    rec["TIME"] = time
    rec["PI"] = pi
    data = rec.tobytes()
    data += b"\0" * (((len(data) + 2879) // 2880) * 2880 - len(data))
    with open(path, "wb") as fh:
        fh.write(prim + ext + data)


def _header_cards(raw, hstart, dstart):
    """The 80-character cards of the header in raw[hstart:dstart] (END card and padding excluded)."""
    text = raw[hstart:dstart].decode("ascii", errors="replace")
    cards = [text[i:i + 80] for i in range(0, len(text), 80)]
    return cards[:next(i for i, c in enumerate(cards) if c[:8].strip() == "END")]


def add_column(path, extname, name, values):
    """Append a double-precision column to a BINTABLE extension of a FITS file in place (the astropy
    Table.add_column + fits.update of eventfile.py:345-353): each row gets 8 big-endian bytes, the header gets
    NAXIS1 += 8, TFIELDS += 1, TTYPEn / TFORMn = 'D'; every other HDU is copied byte for byte. A table with a
    heap keeps it (THEAP moved with the main table). Like astropy, refuses a name the table already has."""
    raw, hdus = read_fits(path)
    out, found = [], False
    pos = 0  # each header starts where the previous HDU's (padded) data ends
    for hdr, dstart, dsize in hdus:
        hstart = pos
        cards = _header_cards(raw, hstart, dstart)
        dend = dstart + ((dsize + 2879) // 2880) * 2880
        if str(hdr.get("EXTNAME", "")).strip() != extname or found:
            out.append(raw[hstart:dend])
            pos = dend
            continue
        found = True
        width, nrow, nf = int(hdr["NAXIS1"]), int(hdr["NAXIS2"]), int(hdr["TFIELDS"])
        names = [str(hdr.get("TTYPE%d" % c, "")).strip() for c in range(1, nf + 1)]
        if name in names:
            raise ValueError("Duplicate column names: %s" % name)
        vals = np.asarray(values, dtype=">f8").reshape(-1)
        if vals.size != nrow:
            raise ValueError("Inconsistent data column lengths: %d rows, %d values" % (nrow, vals.size))
        rows = np.frombuffer(raw, dtype=np.uint8, count=width * nrow, offset=dstart).reshape(nrow, width)
        newrows = np.concatenate([rows, vals.view(np.uint8).reshape(nrow, 8)], axis=1)
        pcount = int(hdr.get("PCOUNT", 0))
        heap = raw[dstart + width * nrow:dstart + width * nrow + pcount] if pcount else b""
        new = []
        for c in cards:
            k = c[:8].strip()
            if k == "NAXIS1":
                c = _card("NAXIS1", width + 8)
            elif k == "TFIELDS":
                c = _card("TFIELDS", nf + 1)
            elif k == "THEAP":
                c = _card("THEAP", int(hdr["THEAP"]) + 8 * nrow)
            new.append(c)
        # the new column's keywords go after the last existing column keyword
        last = max(i for i, c in enumerate(new) if _COLKEY.match(c[:8]))
        new[last + 1:last + 1] = [_card("TTYPE%d" % (nf + 1), name), _card("TFORM%d" % (nf + 1), "D")]
        data = newrows.tobytes() + heap
        out.append(_block(new))
        out.append(data + b"\0" * (((len(data) + 2879) // 2880) * 2880 - len(data)))
        pos = dend
    if not found:
        raise KeyError("no %s extension in %s" % (extname, path))
    out.append(raw[pos:])
    tmp = path + ".tmp%d" % os.getpid()
    with open(tmp, "wb") as fh:
        fh.write(b"".join(out))
    os.replace(tmp, path)


def main(argv=None):
    """addphasecolumn CLI (eventfile.py:378-390)."""
    parser = argparse.ArgumentParser(description="Create and append event file with Phase column")
    parser.add_argument("evtFile", help="Name of (X-ray) fits event file", type=str)
    parser.add_argument("timMod", help="Timing model for phase folding, e.g., a .par file", type=str)
    parser.add_argument("-ne", "--nonBaryEvtFile", help="Name of non-barycentered event file", type=str,
                        default=None)
    args = parser.parse_args(argv)
    EvtFileOps(args.evtFile).addphasecolEF(args.timMod, args.nonBaryEvtFile)


if __name__ == "__main__":
    main()
