"""Configuration mirroring semantic_matching/dssm/config.py:5-34 (same attribute names), plus the
fields the MI355X path needs (layer widths beyond two, compute dtype, sparse capacity)."""
from __future__ import annotations


class Config(object):
    def to_string(self):
        print("conf params: ")
        for key, val in self.__dict__.items():
            print(str(key) + ": " + str(val))

    def __init__(self, verbose: bool = False, **overrides):
        # reference defaults (config.py:13-32)
        self.vocab_path = '../../data/vocab.txt'
        self.file_train = '../../data/dataset_20190508_20190514_2w.txt'
        self.file_vali = '../../data/dataset_vali_20190515_20190515_5k.txt'
        self.query_BS = 400
        self.L1_N = 100
        self.L2_N = 100
        self.learning_rate = 0.01
        self.num_epoch = 10
        self.summaries_dir = './Summaries/'
        self.gpu = 0
        self.NEG = 4
        self.query_mid_vector_file = r'output/y_mid_vector.txt'
        self.doc_pos_y_mid_vector_file = r'output/doc_pos_y_mid_vector.txt'
        self.doc_neg_y_mid_vector_file = r'output/doc_neg_y_mid_vector.txt'
        # MI355X path additions
        self.L3_N = None            # third FC layer (the DSSM paper / BASELINE config 2 shape)
        self.compute_dtype = "bf16"  # "bf16" (perf) or "fp32" (parity)
        self.max_nnz_per_row = 96    # sparse capacity per input row (synthetic generator clips at 96)
        self.seed = 0
        for k, v in overrides.items():
            setattr(self, k, v)
        if verbose:
            self.to_string()

    @property
    def widths(self):
        w = [self.L1_N, self.L2_N]
        if self.L3_N:
            w.append(self.L3_N)
        return w
