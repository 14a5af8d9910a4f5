"""Turn one tools/evidence_configs.sh run (gpurun_out/cfg) into the round's committed evidence:

usage: python tools/evidence_collect.py gpurun_out/cfg rNN

  profiles/<rNN>_bench_mlp3.json              bench.py --config mlp3 line (BASELINE config 2)
  profiles/<rNN>_bench_dnn5.json              bench.py --config dnn5 line (BASELINE config 3 network)
  profiles/<rNN>_configs_4_5.json             tools/rbm_bench.py (config 4) + tools/rnn_bench.py (config 5)
  profiles/<rNN>_mlp3_kernel_trace_stats.txt  rocprofv3 --kernel-trace --stats summary of the MLP3 step
  profiles/<rNN>_rbm256_kernel_stats.txt      the same for the bunch-256 RBM step
"""
import csv
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def last_json(path):
    return json.loads([l for l in open(path).read().splitlines() if l.startswith("{")][-1])


def stats_txt(csv_path, header):
    rows = list(csv.DictReader(open(csv_path)))
    out = [header]
    for r in rows:
        out.append(f"  {r['Name'][:96]:96s} n={int(r['Calls']):6d} avg={float(r['AverageNs']) / 1e3:9.2f}us "
                   f"tot={float(r['TotalDurationNs']) / 1e6:9.2f}ms {float(r['Percentage']):6.2f}%")
    return "\n".join(out) + "\n"


def main():
    src, tag = sys.argv[1], sys.argv[2]
    prof = os.path.join(REPO, "profiles")
    for cfg in ("mlp3", "dnn5"):
        with open(os.path.join(prof, f"{tag}_bench_{cfg}.json"), "w") as f:
            json.dump(last_json(os.path.join(src, f"bench_{cfg}.json")), f, indent=1)
    rnn = [l.strip() for n in ("rnn135.txt", "rnn4000.txt") for l in open(os.path.join(src, n))
           if l.startswith("RNN ")]
    conf = {"rbm": [last_json(os.path.join(src, "rbm256.json")), last_json(os.path.join(src, "rbm1024.json"))],
            "rnn": rnn,
            "source": "python3 tools/rbm_bench.py 256 2000 10 / 1024 1000 4; python3 tools/rnn_bench.py 4 135 / "
                      "2 4000 (one MI355X, tools/evidence_configs.sh)"}
    with open(os.path.join(prof, f"{tag}_configs_4_5.json"), "w") as f:
        json.dump(conf, f, indent=1)
    with open(os.path.join(prof, f"{tag}_mlp3_kernel_trace_stats.txt"), "w") as f:
        f.write(stats_txt(os.path.join(src, "prof_mlp3", "mlp3_kernel_stats.csv"),
                          "rocprofv3 --kernel-trace --stats -- python3 bench.py --config mlp3 --no-cpu-baseline "
                          "--steps 300 --kernel-timing 0 (config 2, 598:1024:135, bunch 1024)"))
    with open(os.path.join(prof, f"{tag}_rbm256_kernel_stats.txt"), "w") as f:
        f.write(stats_txt(os.path.join(src, "prof_rbm256", "rbm_kernel_stats.csv"),
                          "rocprofv3 --kernel-trace --stats -- python3 tools/rbm_bench.py 256 500 1 (config 4, "
                          "Gauss-Bernoulli 440->2048 CD-1, bunch 256)"))
    print(json.dumps(conf, indent=1))


if __name__ == "__main__":
    main()
