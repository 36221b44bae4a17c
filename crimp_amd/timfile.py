"""ToA phase shifts -> Tempo2/PINT .tim wire format, CRIMP v2.3.0
``timfile.py:25-233``: ``readtimfile``, ``PulseToAs`` (time filter, writer with the
``FORMAT 1`` header and one leading space per data line) and ``phshiftTotimfile``."""
import argparse

import numpy as np
import pandas as pd

from .ephemIntegerRotation import ephemIntegerRotation


def readtimfile(timfile, comment="C", skiprows=1):
    df = pd.read_csv(timfile, sep=r"\s+", comment=comment, skiprows=skiprows, header=None, engine="python", dtype=str)
    fixed = {0: "template", 1: "frequency", 2: "pulse_ToA", 3: "pulse_ToA_err", 4: "time_ref"}
    df = df.rename(columns=fixed)
    for c in ("frequency", "pulse_ToA", "pulse_ToA_err"):
        df[c] = pd.to_numeric(df[c], errors="coerce")
    if df.shape[1] <= 5:
        return df[list(fixed.values())]
    rows = []
    for _, r in df.iloc[:, 5:].iterrows():
        toks = [t for t in r.tolist() if pd.notna(t)]
        d, j = {}, 0
        while j < len(toks):
            if isinstance(toks[j], str) and toks[j].startswith("-"):
                key = toks[j].lstrip("-")
                d[key + "_flag"] = toks[j]
                d[key] = toks[j + 1] if j + 1 < len(toks) else None
                j += 2
            else:
                j += 1
        rows.append(d)
    extras = pd.DataFrame(rows, index=df.index)
    if "pn" in extras.columns:
        extras["pn"] = pd.to_numeric(extras["pn"], errors="coerce").astype("Int64")
    return pd.concat([df[list(fixed.values())], extras], axis=1)


class PulseToAs:
    def __init__(self, pulsetoas):
        self._original = pulsetoas.copy()
        self.df = pulsetoas.copy()

    def reset(self):
        self.df = self._original.copy()
        return self

    def time_filter(self, t_start=None, t_end=None, inplace=True):
        mask = self.df["pulse_ToA"].between(-np.inf if t_start is None else t_start,
                                            np.inf if t_end is None else t_end)
        if inplace:
            self.df = self.df.loc[mask].copy()
            return self
        return self.df.loc[mask].copy()

    def writetimfile(self, timfilename, clobber=False):
        assert isinstance(clobber, bool), "Clobber must be of type boolean"
        self.df.to_csv(timfilename + ".tim", sep=" ", index=False, header=False, mode="w" if clobber else "x")
        with open(timfilename + ".tim", "r+") as fh:
            lines = fh.readlines()
            fh.seek(0)
            fh.truncate()
            fh.write("FORMAT 1\n")
            fh.writelines(" " + ln for ln in lines)


def phshiftTotimfile(ToAs, timMod, timfile="residuals", tempModPP="ppTemplateMod", inst="Xray", addpn=False,
                     clobber=False):
    d = pd.read_csv(ToAs, sep=r"\s+", comment="#")
    mids = d["ToA_mid"].to_numpy()
    dph = d["phShift"].to_numpy() / (2 * np.pi)
    dph_err = np.hypot(d["phShift_LL"].to_numpy() / (2 * np.pi), d["phShift_UL"].to_numpy() / (2 * np.pi)) / np.sqrt(2)
    n = len(mids)
    toa = np.zeros(n)
    err_us = np.zeros(n)
    pn = np.zeros(n)
    for i, tm in enumerate(mids):
        e = ephemIntegerRotation(tm, timMod)
        toa[i] = e["Tmjd_intRotation"] + (dph[i] * (1 / e["freq_intRotation"])) / 86400
        err_us[i] = (dph_err[i] * (1 / e["freq_intRotation"])) * 1.0e6
        pn[i] = e["ph_intRotation"]
    out = {"template": np.full(n, tempModPP), "Frequency": np.full(n, 700), "TOA": np.round(toa, 12),
           "TOA_err": np.round(err_us, 5), "timeunit": np.full(n, "@"), "flag_instrument": np.full(n, "-i"),
           "instrument": inst}
    if addpn:
        pn -= np.min(pn)
        out["pulsenumberflag"] = np.full(n, "-pn")
        out["pulsenumber"] = np.round(pn).astype(np.int64)
    tab = pd.DataFrame.from_dict(out)
    PulseToAs(tab).writetimfile(timfile, clobber=clobber)
    return tab


def main(argv=None):
    p = argparse.ArgumentParser(description="Convert a phase-shift text file into a .tim file")
    p.add_argument("ToAs", type=str)
    p.add_argument("timMod", type=str)
    p.add_argument("-tf", "--timfile", type=str, default="residuals")
    p.add_argument("-tp", "--tempModPP", type=str, default="ppTemplateMod")
    p.add_argument("-in", "--inst", type=str, default="Xray")
    p.add_argument("-ap", "--addpn", default=False, action=argparse.BooleanOptionalAction)
    p.add_argument("-cl", "--clobber", default=False, action=argparse.BooleanOptionalAction)
    a = p.parse_args(argv)
    phshiftTotimfile(a.ToAs, a.timMod, a.timfile, a.tempModPP, a.inst, a.addpn, a.clobber)


if __name__ == "__main__":
    main()
