"""Where a 400-observation refit's host time goes (GPU box): cProfile over 200 ObservationStore.refit calls
(one new row each), the top entries by own time.  python tools/refit_profile.py [n]"""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from hpbandster_amd import kde
    from hpbandster_amd import synthetic as S
    dev = torch.device("cuda", 0)
    nobs = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    reps = 200
    X = S.make_observations(nobs + reps, 24, 8, 4)
    losses = S.make_losses(nobs + reps)
    store = kde.ObservationStore(32, S.var_type_string(24, 8), device=dev, capacity=2 * (nobs + reps))
    store.add(X[:nobs], losses[:nobs])
    store.refit(33)
    for r in range(20):  # warm
        store.add(X[nobs + r], losses[nobs + r])
        store.refit(33)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for r in range(20, reps):
        store.add(X[nobs + r], losses[nobs + r])
        store.refit(33)
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
