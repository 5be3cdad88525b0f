"""Summarise tools/gpu_variants.sh logs: value, ms/step and the T1 stage times per variant."""
import glob
import json
import os

for f in sorted(glob.glob("gpurun_out/var_*.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            s = d["stages_ms"]
            print("%-10s %8.1f Mpix/s %7.2f ms  enc_t1 %6.2f (cm %5.2f mq %5.2f)  dec_t1 %6.2f (coder %6.2f)  dwt %5.2f/%5.2f" % (
                os.path.basename(f)[4:-4], d["value"], d["ms_per_step"], s["enc_t1_ms"], s["enc_t1_cm_ms"],
                s["enc_t1_coder_ms"], s["dec_t1_ms"], s["dec_t1_coder_ms"], s["enc_dwt_ms"], s["dec_dwt_ms"]))
