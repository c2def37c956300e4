"""Per-launch HBM traffic of one kernel from two rocprofv3 --pmc passes.

    python tools/pmc_summary.py --fetch DIR --write DIR --kernel roi_align_fwd_buf \
        [--calib-fetch DIR --calib-bytes N] --out profiles/roi_align_pmc.json

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (MI355X_MICROARCH.md, HBM section).  The
guide's x2 FETCH correction is calibrated only for 16-B/lane streaming reads; this kernel
issues 8-B gathers, so the FETCH scale is measured on a known-byte launch of the SAME kernel
(tools/bench_roi_align.py --calib) when --calib-fetch is given: scale = known bytes / FETCH.
"""
import argparse, csv, glob, json, os


def counter_rows(d, name):
    rows = []
    for p in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(p)):
            if r['Counter_Name'] == name:
                rows.append(r)
    return rows


def per_launch(d, name, kernel):
    vals = [float(r['Counter_Value']) for r in counter_rows(d, name) if kernel in r['Kernel_Name']]
    if not vals:
        raise SystemExit('no {} rows for kernel matching {!r} under {}'.format(name, kernel, d))
    return sum(vals) / len(vals), len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--fetch', required=True)
    ap.add_argument('--write', required=True)
    ap.add_argument('--kernel', required=True)
    ap.add_argument('--calib-fetch', nargs='*', default=[])
    ap.add_argument('--calib-kernel')
    ap.add_argument('--calib-bytes', nargs='*', type=float, default=[])
    ap.add_argument('--out', required=True)
    a = ap.parse_args()
    fkb, nf = per_launch(a.fetch, 'FETCH_SIZE', a.kernel)
    # the full dispatched name (template arguments included): bench.py uses this figure only
    # while the kernel it dispatches is this same instantiation
    names = sorted({r['Kernel_Name'] for r in counter_rows(a.fetch, 'FETCH_SIZE') if a.kernel in r['Kernel_Name']})
    wkb, nw = per_launch(a.write, 'WRITE_SIZE', a.kernel)
    import datetime
    res = {'kernel': a.kernel, 'kernel_names': names, 'measured': datetime.datetime.now().isoformat(timespec='seconds'),
           'fetch_kib_per_launch': fkb, 'write_kib_per_launch': wkb,
           'launches_fetch_pass': nf, 'launches_write_pass': nw}
    scale, how = 1.0, 'raw FETCH_SIZE (uncalibrated access width)'
    if a.calib_fetch:
        cal = []
        for d, nbytes in zip(a.calib_fetch, a.calib_bytes):
            ckb, _ = per_launch(d, 'FETCH_SIZE', a.calib_kernel or a.kernel)
            cal.append({'dir': d, 'known_bytes': nbytes, 'fetch_kib': ckb, 'scale': nbytes / (ckb * 1024.0)})
        scales = [c['scale'] for c in cal]
        res['calibration'] = cal
        if max(scales) / min(scales) < 1.1:  # both access paths agree: apply their mean
            scale = sum(scales) / len(scales)
            how = 'FETCH_SIZE x {:.3f}: mean of known-byte calibration launches {}'.format(
                scale, ['{:.3f}'.format(x) for x in scales])
        else:
            how = 'raw FETCH_SIZE: calibration launches disagree ({})'.format(['{:.3f}'.format(x) for x in scales])
    res['fetch_scale'] = scale
    res['fetch_correction'] = how
    res['hbm_bytes_per_launch'] = fkb * 1024.0 * scale + wkb * 1024.0
    json.dump(res, open(a.out, 'w'), indent=1)
    print(json.dumps(res))


if __name__ == '__main__':
    main()
