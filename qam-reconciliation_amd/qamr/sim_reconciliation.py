"""SNR-sweep CLI, the GPU counterpart of sims/sim_reconciliation.py (arguments and
CSV schema of sim_reconciliation.py:27-102, README.md:107-145).

    PYTHONPATH=qam-reconciliation_amd python -m qamr.sim_reconciliation EDGEFILE \\
        [--out out.csv] [--maxiter 50] [--ferr-count-min 100] [--alpha 1.0] \\
        [--simloops 5000] [--snr 0 5] [--nsnr 11] [--bps 2] [--hard | --direct] \\
        [--configuration-base] [--batch 4096] [--seed 0]

Instead of one OS process per SNR point (parfor), every SNR point runs batched
on the GPU(s); launched under torchrun, each rank takes its share of every
batch and the BER/FER counters are all-reduced over RCCL (qamr.dist).
"""
from __future__ import annotations

import argparse
import sys

import numpy as np


def main(argv=None):
    p = argparse.ArgumentParser(prog="decode", description="Evaluate BER for LDPC codes vs Raw BER")
    p.add_argument("edgefile", help="CSV with a 'vid' and a 'cid' columns representing an edge per line")
    p.add_argument("--out", default="out.csv")
    p.add_argument("--maxiter", default=50, type=int, help="Maximum number of iterations for the decoder")
    p.add_argument("--ferr-count-min", default=100, type=int, help="Minimum number of frame errors for early exit")
    p.add_argument("--alpha", type=float, default=1.0, help="Extra multiplicative coefficient for the LLR")
    p.add_argument("--simloops", default=5000, type=int, help="Number of frames per SNR point")
    p.add_argument("--snr", type=float, nargs=2, default=[0, 5], help="Initial and final SNR [dB]")
    p.add_argument("--nsnr", type=int, default=11, help="Number of equally spaced SNR [dB] points")
    p.add_argument("--bps", type=int, default=2, help="Bit Per Symbol (=log_2(PAM Order))")
    p.add_argument("--hard", action="store_true", help="Simulate hard reverse reconciliation")
    p.add_argument("--direct", action="store_true", help="Simulate the soft direct reconciliation, overrides '--hard'")
    p.add_argument("--configuration-base", action="store_true",
                   help="Instead of the Alternating configuration, use the Base configuration")
    p.add_argument("--batch", type=int, default=4096, help="frames per GPU per batch")
    p.add_argument("--seed", type=int, default=0)
    args = p.parse_args(argv)

    from . import dist
    from .codes import load_edge_csv
    from .decoder import Decoder
    from .sim import Simulator

    world, rank, local = dist.init()
    vid, cid = load_edge_csv(args.edgefile)  # counts row skipped (sim_reconciliation.py:60)
    dec = Decoder(vid, cid, device=local)
    mode = "direct" if args.direct else ("hard" if args.hard else "softening")
    sim = Simulator(dec, args.bps, mode, args.maxiter, args.alpha, args.batch,
                    configuration_base=args.configuration_base, device=local)
    rows = []
    for snr in np.linspace(args.snr[0], args.snr[1], args.nsnr):
        rows.append(sim.run_snr(float(snr), args.simloops, args.ferr_count_min, args.seed))
        if rank == 0:
            print("EsN0dB=%.3f ber=%.6g fer=%.6g iters=%.3f" % rows[-1], flush=True)
    if rank == 0:
        with open(args.out, "w") as fh:  # pandas DataFrame.to_csv layout (sim_reconciliation.py:96-102)
            fh.write(",EsN0dB,ber,fer,iters\n")
            for i, r in enumerate(rows):
                fh.write(f"{i},{r[0]!r},{r[1]!r},{r[2]!r},{r[3]!r}\n")
    dist.finalize()
    return rows


if __name__ == "__main__":
    sys.exit(0 if main() is not None else 1)
