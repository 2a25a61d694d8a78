"""Comm-stream slack in a serialised slab-group kernel trace (scripts/slab_trace.py N): per group step,
the end of the last comm-stream dispatch (ρ halo, boundary force passes, the next step's sends, bookkeeping) against the
end of the last interior force pass on the compute stream, and the boundary passes' mean duration.
usage: comm_slack.py run_kernel_trace.csv NSLABS [STEPS]"""
import csv
import re
import sys

f, nsl = sys.argv[1], int(sys.argv[2])
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
ev = []
for r in csv.DictReader(open(f)):
    k = re.sub(r"<[^>]*>", "", r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sph::", "")).strip()
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k, r["Stream_Id"]))
ev.sort()
dens = [i for i, e in enumerate(ev) if e[2] == "k_density_tiled"]
main = ev[dens[-1]][3]   # the compute stream (every density pass runs there)
# the comm streams: those running the halo kernels (an interior pass on its own CU-masked stream, SPH_INTERIOR_CU_EXCLUDE,
# is neither the compute stream nor a comm stream)
comm_streams = {e[3] for e in ev if e[2] in ("k_slab_unpack_rho2", "k_slab_pack2", "k_slab_rec", "k_slab_lag")} - {main}
starts = dens[::nsl]     # the first density pass of each group step
slack, bnd = [], []
for a, b in zip(starts[-steps - 1:-1], starts[-steps:]):
    w = ev[a:b]
    inter = [e for e in w if e[2] == "k_force_tiled" and e[3] not in comm_streams]
    comm = [e for e in w if e[3] in comm_streams]
    if not inter or not comm:
        continue
    slack.append((max(e[1] for e in inter) - max(e[1] for e in comm)) / 1e3)
    bnd += [(e[1] - e[0]) / 1e3 for e in comm if e[2] == "k_force_tiled"]
slack.sort()
print({"steps": len(slack), "slack_us_min": round(slack[0], 1), "slack_us_median": round(slack[len(slack) // 2], 1),
       "boundary_pass_us_mean": round(sum(bnd) / max(len(bnd), 1), 1)})
