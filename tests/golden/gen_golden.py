"""Generate tests/golden/reference_kats.json from the reference's OWN fixtures.

Run here (where /root/reference exists); the JSON is committed and is all the
GPU box sees.  Contents are data only:

  * LOG_TABLE / EXP_TABLE values, parsed from the array literals of
    rs/src/main/java/com/backblaze/erasure/Galois.java:59-93,103-170
    (GaloisTest.java:114-127 checks the generated tables against them);
  * the JUnit known-answer values of GaloisTest.java:139-149,
    MatrixTest.java:178-236 and ReedSolomonTest.java:44-70 (transcribed as
    numbers with the line they come from);
  * LP-block.jpg is copied next to this script as a binary input fixture
    (the input file of SampleEncoder / LRCErasureCodeExample, configs 1 and 3).

The SURVEY.md A.4 cross-check digests (sha256, first 16 hex chars) are kept
as independent expected values for the oracle restatement.  gen_clay42_maps.py then
derives the Clay(4,2) e=1 / e=4 repair maps and the encode map in closed form from the
pair-transform and RS equations alone (clay42_closed_form.json).
"""
import sys
import json
import re
import shutil
from pathlib import Path

REF = Path("/root/reference")
HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))


def parse_java_array(text: str, name: str):
    m = re.search(name + r"\s*=\s*new\s+\w+\s*\[\]\s*\{(.*?)\};", text, re.S)
    body = re.sub(r"//[^\n]*", "", m.group(1))
    return [int(x) for x in re.findall(r"-?\d+", body)]


def main():
    galois = (REF / "rs/src/main/java/com/backblaze/erasure/Galois.java").read_text()
    log_table = parse_java_array(galois, "LOG_TABLE")
    exp_table = [x & 0xFF for x in parse_java_array(galois, "EXP_TABLE")]
    assert len(log_table) == 256 and len(exp_table) == 510

    kats = {
        "source": "krishnarb3/repair-pipelining reference JUnit fixtures (see gen_golden.py)",
        "galois": {
            "generating_polynomial": 29,  # Galois.java:43
            "log_table": log_table,  # Galois.java:59-93
            "exp_table": exp_table,  # Galois.java:103-170
            "polynomials": [29, 43, 45, 77, 95, 99, 101, 105, 113, 135, 141, 169, 195, 207, 231, 245],  # GaloisTest.java:122-126
            "multiply": [[3, 4, 12], [7, 7, 21], [23, 45, 41]],  # GaloisTest.java:142-144
            "exp": [[2, 2, 4], [5, 20, 235], [13, 7, 43]],  # GaloisTest.java:146-148
        },
        "matrix": {
            "times": {"a": [[1, 2], [3, 4]], "b": [[5, 6], [7, 8]], "out": [[11, 22], [19, 42]]},  # MatrixTest.java:178-193
            "invert": [
                {"m": [[56, 23, 98], [3, 100, 200], [45, 201, 123]],
                 "inv": [[175, 133, 33], [130, 13, 245], [112, 35, 126]]},  # MatrixTest.java:195-212
                {"m": [[1, 0, 0, 0, 0], [0, 1, 0, 0, 0], [0, 0, 0, 1, 0], [0, 0, 0, 0, 1], [7, 7, 6, 6, 1]],
                 "inv": [[1, 0, 0, 0, 0], [0, 1, 0, 0, 0], [123, 123, 1, 122, 122], [0, 0, 1, 0, 0],
                         [0, 0, 0, 1, 0]]},  # MatrixTest.java:214-236
            ],
        },
        "reed_solomon": {
            "rs55_data": [[0, 1], [4, 5], [2, 3], [6, 7], [8, 9]],  # ReedSolomonTest.java:49-53
            "rs55_parity": [[12, 13], [10, 11], [14, 15], [90, 91], [94, 95]],  # ReedSolomonTest.java:60-64
            "simple_data": [[0, 1], [1, 2], [1, 3], [2, 4], [3, 5]],  # ReedSolomonTest.java:77-83
            "java_random_0_first_int": -1155484576,  # java.util.Random(0).nextInt(), JDK spec
        },
        "survey_digests": {  # SURVEY.md A.4 (independent scratch restatement)
            "sample_encoder_lp_block": ["2e8b90f242ad5e5e", "1ca28fd347c8f45c", "06612d2264623d1c",
                                        "31dd1a42d88f0a8a", "39ba02564b5690c2", "80a23f293ebbe80e"],
            "lrc_local_parities_3_7_11_15": ["f23bb7dbc50dbb35", "a30e8d810e7a3634", "4928da6b22ac792e",
                                             "990ae96c7d8c24b6"],
            "clay42_first_bytes": "27bcc8696e7acfe1",
            "clay42_parity_node4": ["9bc2689f1cbc257c", "8b2d979463427dd7", "95a4bd3b84785a22", "435d5a797493c7c1",
                                    "0d99ba63a7c4e38a", "afd5400af04da1b6", "80554b8f10c391f3", "f7020624a58e9d39"],
            "clay42_parity_node5": ["20465b8f567eeaba", "21a0e19c7e98ce2a", "a979b43f29e1a119", "06f047fbada00313",
                                    "0b3dc98a5e0e9b9a", "572f4048cb4ab2fd", "23bf57e46ba680a1", "c79001f38abab1e7"],
        },
        "rs_parity_rows": {  # SURVEY.md A.1 (derived from ReedSolomon.buildMatrix)
            "2,2": [[3, 2], [2, 3]],
            "3,1": [[1, 1, 1]],
            "4,2": [[27, 28, 18, 20], [28, 27, 20, 18]],
            "12,4": [[175, 180, 150, 140, 245, 232, 196, 216, 27, 28, 18, 20],
                     [180, 175, 140, 150, 232, 245, 216, 196, 28, 27, 20, 18],
                     [150, 140, 175, 180, 196, 216, 245, 232, 18, 20, 27, 28],
                     [140, 150, 180, 175, 216, 196, 232, 245, 20, 18, 28, 27]],
            "17,3_row0": [148, 148, 115, 115, 221, 221, 48, 48, 227, 227, 238, 238, 87, 87, 81, 81, 1],
        },
    }
    (HERE / "reference_kats.json").write_text(json.dumps(kats, indent=1) + "\n")
    shutil.copyfile(REF / "LP-block.jpg", HERE / "LP-block.jpg")
    print("wrote", HERE / "reference_kats.json", "and LP-block.jpg")
    # the closed-form Clay(4,2) maps (an independent pin of the planner and the oracle)
    import gen_clay42_maps
    gen_clay42_maps.main()


if __name__ == "__main__":
    main()
