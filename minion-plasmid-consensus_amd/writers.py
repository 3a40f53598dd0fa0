"""Step 7 writers of the reference (:446-463), fed by the device call arrays.

consensus  ">consensus\\n" + called bases + "\\n"
chromat    "pos\\tbase\\tcount" header, two lines per call (top, second) using the
           pre-GTF bases; pos is the 1-based index in the consensus
accuracies "pos\\taccuracy" header, str(100 * (count / total)) per call
"""
import numpy as np


def consensus_text(calls):
    return ">consensus\n" + bytes(calls["base"]).decode("ascii") + "\n"


def chromat_text(calls):
    c1 = bytes(calls["chrom1"]).decode("ascii")
    c2 = bytes(calls["chrom2"]).decode("ascii")
    cnt = calls["count"].tolist()
    cnt2 = calls["count2"].tolist()
    out = ["pos\tbase\tcount\n"]
    for i in range(len(cnt)):
        out.append("%d\t%s\t%d\n%d\t%s\t%d\n" % (i + 1, c1[i], cnt[i], i + 1, c2[i], cnt2[i]))
    return "".join(out)


def accuracies_text(calls):
    # 100 * (count / total): the division of two ints < 2^53 is the correctly
    # rounded IEEE quotient in both Python and numpy, then one f64 multiply;
    # str() of a Python float is the shortest round-trip repr (:431, :463).
    cnt = np.asarray(calls["count"], dtype=np.float64)
    tot = np.asarray(calls["total"], dtype=np.float64)
    acc = (100.0 * (cnt / tot)).tolist() if len(cnt) else []
    out = ["pos\taccuracy\n"]
    out.extend("{}\t{}\n".format(i + 1, a) for i, a in enumerate(acc))
    return "".join(out)


def write_outputs(calls, consensus_path, chromat_path, accuracies_path):
    with open(consensus_path, "w") as f:
        f.write(consensus_text(calls))
    with open(chromat_path, "w") as f:
        f.write(chromat_text(calls))
    with open(accuracies_path, "w") as f:
        f.write(accuracies_text(calls))
