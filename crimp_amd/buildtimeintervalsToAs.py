"""ToA interval construction: the ``timeintervalsfortoas`` step that feeds
``measureToAs``, restating CRIMP v2.3.0 ``buildtimeintervalsToAs.py``.

  * ``timeintervalsToAs``       :64-312  GTI bunches split at gaps > waitTimeCutoff (:119-151),
                                         ``totCtsEachToA``-count slices of each bunch's photons
                                         (:169-257), exact exposure from the GTIs clipped to the slice's
                                         first/last photon, zero-exposure slices skipped, ``{:0.9f}``
                                         rows written then re-read (the rounding that later drops
                                         boundary photons in ``measureToAs``), merging (:262), NICER
                                         FPM-selection rate correction (:268-300), ``to_csv`` (:305)
  * ``merge_adjacent_intervals`` :315-365
  * ``main``                    :368-407 (CLI ``timeintervalsfortoas``; ``python -m`` here)

Host-side, sequential over bunches: one pass over sorted photon times with a binary search per
bunch instead of the reference's full-array mask per bunch, same output rows.
"""
import argparse

import numpy as np
import pandas as pd

from .eventfile import EvtFileOps
from .logging_utils import configure_logging, get_logger

logger = get_logger(__name__)

COLS = ["ToA_tstart", "ToA_tend", "ToA_lenInt", "ToA_exposure", "Events", "ct_rate"]


def _bunches(gtiList, waitTimeCutoff):
    """GTI bunches with no internal gap above waitTimeCutoff (buildtimeintervalsToAs.py:119-151):
    rows [tstart, tend, exposure (days), lenInt]."""
    wait = np.append(gtiList[1:, 0] - gtiList[:-1, 1], 0)
    exp_each = gtiList[:, 1] - gtiList[:, 0]
    cuts = np.flatnonzero(wait > waitTimeCutoff) + 1
    edges = np.concatenate(([0], cuts, [gtiList.shape[0]])).astype(int)
    rows = []
    for a, b in zip(edges[:-1], edges[1:]):
        seg = gtiList[a:b]
        rows.append((seg[0, 0], seg[-1, 1], np.sum(exp_each[a:b]), seg[-1, 1] - seg[0, 0]))
    return np.array(rows, dtype=np.float64).reshape(-1, 4)


def _exposure(gtiList, t_first, t_last):
    """Exposure (days) of a photon slice: GTIs ending after its first photon and starting before its
    last, the first start / last stop clipped to those photons (:176-187)."""
    g = gtiList[gtiList[:, 1] > t_first, :]
    g = g[g[:, 0] < t_last, :]
    g[0, 0] = t_first
    g[-1, -1] = t_last
    return np.sum(g[:, 1] - g[:, 0])


def _row(t, expo):
    return ('{:0.9f}'.format(t[0]) + '\t' + '{:0.9f}'.format(t[-1]) + '\t' + '{:0.9f}'.format(t[-1] - t[0]) + '\t'
            + '{:0.9f}'.format(expo * 86400) + '\t' + str(len(t)) + '\t'
            + '{:0.9f}'.format(len(t) / (expo * 86400)) + '\n')


def timeintervalsToAs(evtFile, totCtsEachToA=1000, waitTimeCutoff=1.0, eneLow=0.5, eneHigh=10,
                      min_counts=None, max_wait=None, outputFile="timIntToAs", correxposure=False):
    """START/END times of each ToA (buildtimeintervalsToAs.py:64). Writes ``outputFile``_bunches.txt
    and ``outputFile``.txt; returns the cleaned interval DataFrame."""
    if min_counts is None:
        min_counts = int(totCtsEachToA / 2)
    if max_wait is None:
        max_wait = waitTimeCutoff
    logger.info('\n Running timeintervalsToAs with input parameters: \n evtFile: %s\n totCtsEachToA: %s'
                '\n waitTimeCutoff: %s\n eneLow: %s\n eneHigh: %s\n min_counts: %s\n max_wait: %s'
                '\n outputFile: %s\n', evtFile, totCtsEachToA, waitTimeCutoff, eneLow, eneHigh, min_counts, max_wait,
                outputFile)

    EF = EvtFileOps(evtFile)
    evtFileKeyWords, gtiList = EF.readGTI()
    TIME = EF.build_time_energy_df().filtenergy(eneLow=eneLow, eneHigh=eneHigh).time_energy_df['TIME'].to_numpy()

    bunches = _bunches(gtiList, waitTimeCutoff)
    with open(outputFile + "_bunches.txt", "w+") as f:
        f.write('ToABunch_tstart \t ToABunch_tend \t ToABunch_exp \t ToABunch_lenInt\n')
        for b in bunches:
            f.write(str(b[0]) + '\t' + str(b[1]) + '\t' + str(b[2] * 86400) + '\t' + str(b[3]) + '\n')

    # the reference masks TIME per bunch (:169-170); for time-ordered events a binary search gives the
    # same contiguous run, otherwise fall back to the mask
    ordered = TIME.size < 2 or bool(np.all(TIME[1:] >= TIME[:-1]))
    with open(outputFile + ".txt", "w+") as f:
        f.write('ToA_tstart \t ToA_tend \t ToA_lenInt \t ToA_exposure \t Events \t ct_rate\n')
        for b in bunches:
            if ordered:
                lo, hi = np.searchsorted(TIME, b[0], "left"), np.searchsorted(TIME, b[1], "right")
                tb = TIME[lo:hi]
            else:
                tb = TIME[(TIME >= b[0]) & (TIME <= b[1])]
            nbr = int(np.ceil(len(tb) / totCtsEachToA))
            for nn in range(nbr):
                t = tb[nn * totCtsEachToA:] if nn == nbr - 1 else tb[nn * totCtsEachToA:(nn + 1) * totCtsEachToA]
                expo = _exposure(gtiList, t[0], t[-1])
                if expo == 0:
                    logger.warning(f"At {t[0]} MJD: exposure = 0 likely caused by a single timestamp "
                                   f"in interval - skipping")
                    continue
                f.write(_row(t, expo))

    timInt_toas = pd.read_csv(outputFile + ".txt", sep=r'\s+')
    timInt_toas = merge_adjacent_intervals(timInt_toas, min_counts, max_wait)
    nbrToATOT = len(timInt_toas)

    if evtFileKeyWords["TELESCOPE"] == 'NICER':
        logger.warning("\n If NICER event files were generaed with HEASOFT version 6.32+,\n it is advisable to "
                       "correct for the number of selected FPMs with the flag -ce for accurate\n measurement of "
                       "count rates\n")
        if correxposure is True:
            _, fpm = EF.read_fpmsel()
            for pp in range(nbrToATOT):
                a, b = timInt_toas['ToA_tstart'][pp], timInt_toas['ToA_tend'][pp]
                sel = fpm.loc[(fpm['TIME'] >= a) & (fpm['TIME'] <= b)]
                nbr_sel_det = np.sum(sel['TOTFPMSEL'])
                exp_nbr_det = 52 * timInt_toas['ToA_exposure'][pp]
                timInt_toas.at[pp, 'ct_rate'] *= exp_nbr_det / nbr_sel_det
        else:
            logger.info('\n No correction of exposure according to number of detectors_selected per ToA '
                        'interval\n This should not be an issue assuming HEASOFT 6.31- was used to reduce NICER '
                        'data\n')
    elif evtFileKeyWords["TELESCOPE"] == 'NuSTAR':
        logger.warning("\n If NuSTAR event files are merged for detectors FPMA and FPMB, then resulting count "
                       "rates  will be a factor of 2 smaller.\n")

    print('Total number of time intervals that define the TOAs: {}'.format(nbrToATOT))
    timInt_toas.to_csv(outputFile + ".txt", sep='\t', index=True, index_label='ToA')
    logger.info('\n End of timeintervalsToAs run\n Total number of time intervals that define each ToA: %d',
                nbrToATOT)
    return timInt_toas


def merge_adjacent_intervals(df, events_max, dtstart_max_days):
    """Merge row j into the running segment when Events[j] < events_max and
    ToA_tstart[j] - segment ToA_tend < dtstart_max_days (buildtimeintervalsToAs.py:315-365)."""
    if df.empty:
        return pd.DataFrame(columns=COLS)
    out = []
    cur = df.iloc[0].copy()
    for i in range(1, len(df)):
        row = df.iloc[i]
        if row['Events'] < events_max and (row['ToA_tstart'] - cur['ToA_tend']) < dtstart_max_days:
            expo = cur['ToA_exposure'] + row['ToA_exposure']
            events = cur['Events'] + row['Events']
            cur['ToA_tend'] = row['ToA_tend']
            cur['ToA_lenInt'] = row['ToA_tend'] - cur['ToA_tstart']
            cur['ToA_exposure'] = expo
            cur['Events'] = events
            cur['ct_rate'] = events / expo if expo != 0 else float('nan')
        else:
            out.append(cur[COLS].copy())
            cur = row.copy()
    out.append(cur[COLS].copy())
    return pd.DataFrame(out, columns=COLS).reset_index(drop=True)


def main(argv=None):
    p = argparse.ArgumentParser(description="Creating time intervals for individual ToAs - saving info to .txt file")
    p.add_argument("evtFile", help="Fits event file", type=str)
    p.add_argument("-tc", "--totCtsEachToA", help="Desired number of counts per ToA", type=int, default=1000)
    p.add_argument("-wt", "--waitTimeCutoff", help="Do not allow any gap in GTI larger than this (in days)",
                   type=float, default=1)
    p.add_argument("-el", "--eneLow", help="Low energy filter in event file, default=0.5", type=float, default=0.5)
    p.add_argument("-eh", "--eneHigh", help="High energy filter in event file, default=10", type=float, default=10)
    p.add_argument("-mc", "--min_counts", type=int, default=None,
                   help="min counts < which merge time interval with previous ones, default = totCtsEachToA / 2")
    p.add_argument("-mw", "--max_wait", type=float, default=None,
                   help="max wait < which merge time interval with previous ones, default = waitTimeCutoff")
    p.add_argument("-of", "--outputFile", type=str, default='timIntToAs',
                   help="name of .txt output file that defines ToAs. Also name of .log file (default = timIntToAs)")
    p.add_argument("-ce", "--correxposure", default=False, action=argparse.BooleanOptionalAction,
                   help="Flag to correct exposure/rate according to selected FPMs, default = False")
    p.add_argument("-v", "--verbose", action="count", default=0, help="WARNING if absent, -v: INFO, -vv: DEBUG")
    a = p.parse_args(argv)
    configure_logging(console_level=("WARNING", "INFO", "DEBUG")[min(a.verbose, 2)],
                      file_path=f"{a.outputFile}.log", file_level="INFO", force=True)
    timeintervalsToAs(a.evtFile, a.totCtsEachToA, a.waitTimeCutoff, a.eneLow, a.eneHigh, a.min_counts, a.max_wait,
                      a.outputFile, a.correxposure)


if __name__ == '__main__':
    main()
