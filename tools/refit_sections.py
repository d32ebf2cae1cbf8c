"""Host time of each section of ObservationStore._refit at n observations (GPU box): the method's body
restated with perf_counter stamps between its sections, medians over 200 refits of one new row each.
    python tools/refit_sections.py [n]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from hpbandster_amd import _native as N
    from hpbandster_amd import kde
    from hpbandster_amd import synthetic as S
    dev = torch.device("cuda", 0)
    nobs = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    reps = 220
    X = S.make_observations(nobs + reps, 24, 8, 4)
    losses = S.make_losses(nobs + reps)
    D = 32
    store = kde.ObservationStore(D, S.var_type_string(24, 8), device=dev, capacity=2 * (nobs + reps))
    store.add(X[:nobs], losses[:nobs])
    store.refit(D + 1)
    L = N.lib()
    names = ["enter", "stage", "sizes", "alloc", "native_sync", "unpack", "models"]
    rows = []
    for r in range(reps):
        store.add(X[nobs + r], losses[nobs + r])
        t = [time.perf_counter()]
        n = store.nh
        sizes = kde.split_sizes(n, D, D + 1)
        self = store
        with N.on_device(dev, None):
            X_host, lh = self._Xh[:n], self._lh[:n]
            n_good, n_bad = sizes
            n_new = n - self.n
            self._reserve(n)
            sh = kde._raw_stream(dev)
            t.append(time.perf_counter())
            staged = np.empty(n_new * (D + 1), dtype=np.float64)
            staged[:n_new * D] = X_host[self.n:].reshape(-1)
            staged[n_new * D:] = lh[self.n:]
            t.append(time.perf_counter())
            ob = int(L.hbx_kde_refit_out_bytes(n, D))
            sb = int(L.hbx_kde_refit_scratch_bytes(n, D))
            pb = int(L.hbx_kde_param_bytes())
            tgf = int(L.hbx_kde_table_floats(n_good, self.dc_pad, self.du_pad))
            tbf = int(L.hbx_kde_table_floats(n_bad, self.dc_pad, self.du_pad))
            t.append(time.perf_counter())
            a_ob, a_sb, a_pb, a_tg = (ob + 255) & ~255, (sb + 255) & ~255, (pb + 255) & ~255, (4 * tgf + 255) & ~255
            blk = torch.empty(a_ob + a_sb + 2 * a_pb + a_tg + 4 * tbf, dtype=torch.uint8, device=dev)
            p0 = blk.data_ptr()
            p_scr = p0 + a_ob
            pg = kde._DevSlice(blk, p_scr + a_sb, pb)
            pbad = kde._DevSlice(blk, pg._ptr + a_pb, pb)
            tg = kde._DevSlice(blk, pbad._ptr + a_pb, tgf)
            tb = kde._DevSlice(blk, tg._ptr + a_tg, tbf)
            ah = np.empty(ob, dtype=np.uint8)
            t.append(time.perf_counter())
            N.check(L.hbx_kde_refit_sync(N.ptr(self.X_dev), N.ptr(self.loss_dev), n, D, N.ptr(self.vt),
                                         staged.ctypes.data, n_new, n_good, n_bad,
                                         kde.bandwidth_factor(n_good, D), kde.bandwidth_factor(n_bad, D),
                                         pg._ptr, tg._ptr, tgf, pbad._ptr, tb._ptr, tbf, p0, p_scr, sb, sh,
                                         ah.ctypes.data))
            t.append(time.perf_counter())
            order_h = ah[:8 * n].view(np.int64)
            o = 8 * n
            bw_gh = ah[o:o + 8 * D].view(np.float64)
            bw_bh = ah[o + 8 * D:o + 16 * D].view(np.float64)
            nl_gh = ah[o + 16 * D:o + 20 * D].view(np.int32)
            nl_bh = ah[o + 20 * D:o + 24 * D].view(np.int32)
            info_g = ah[o + 24 * D:o + 24 * D + 32].view(np.int32)
            info_b = ah[o + 24 * D + 32:o + 24 * D + 64].view(np.int32)
            if (nl_gh < 0).any() or (nl_bh < 0).any():
                raise N.HbxError("bad codes")
            self.n = n
            order = blk[:8 * n].view(torch.int64)
            t.append(time.perf_counter())
            good = kde.DeviceKDE(self.X_dev, order[:n_good], self.var_type, bw_gh, nl_gh, (X_host, order_h[:n_good]),
                                 prepared=(pg, tg, info_g))
            bad = kde.DeviceKDE(self.X_dev, order[n - n_bad:], self.var_type, bw_bh, nl_bh,
                                (X_host, order_h[n - n_bad:]), prepared=(pbad, tb, info_b))
            pair = kde.KDEPair(good, bad)
            pair._keep = (blk,)
            t.append(time.perf_counter())
        if r >= 20:
            rows.append(np.diff(t))
    med = np.median(np.array(rows), axis=0) * 1e6
    res = {k: round(float(v), 2) for k, v in zip(names, med)}
    res["total_us"] = round(float(med.sum()), 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
