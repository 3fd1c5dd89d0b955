"""Mid-vector text format of load_model_and_save_vector.py:108-152 (host side, no GPU)."""
import numpy as np

from dssm_amd.export import append_mid_vectors, mid_vector_line, read_mid_vectors


def test_mid_vector_line_format():
    v = np.array([0.0, 0.123456789, 1e-5, 0.0001, 0.00012345, 2.5, 12.3456789, -0.5], np.float32)
    # float32 -> Python float str, cut to 6 chars; 0.0, <= 1e-4 and negatives dropped
    exp = ",".join(["1:" + str(float(np.float32(0.123456789)))[:6],
                    "4:" + str(float(np.float32(0.00012345)))[:6],
                    "5:2.5", "6:" + str(float(np.float32(12.3456789)))[:6]])
    assert mid_vector_line("刘 德 华", v) == "刘德华\t" + exp
    assert mid_vector_line("a b", np.zeros(4, np.float32)) == "ab\t"


def test_append_and_read_back(tmp_path):
    p = tmp_path / "y_mid_vector.txt"
    Y = np.array([[0.5, 0.0, 0.25], [0.0, 0.0, 0.0]], np.float32)
    assert append_mid_vectors(str(p), ["x y", "z"], Y) == 2
    append_mid_vectors(str(p), ["w"], Y[:1])  # 'a+': appends
    rows = list(read_mid_vectors(str(p)))
    assert rows == [("xy", {0: 0.5, 2: 0.25}), ("z", {}), ("w", {0: 0.5, 2: 0.25})]
