"""TEST INFRASTRUCTURE ONLY: a Python restatement of the reference's text pre-processing, used to
check libdssm.so's native data path (dssm_amd/feed.py).  Never imported by the product.

pre_process follows /root/reference/utils/utils.py:424-437 line for line (the regexes are the
reference's); the vectorizer check uses scikit-learn's CountVectorizer with the reference's
arguments (new_dssm.py:37) directly.
"""
import re

_URL = re.compile(r'http[s]?://(?:[a-zA-Z]|[0-9]|[$-_@.&+]|[!*\(\),]|(?:%[0-9a-fA-F][0-9a-fA-F]))+')


def pre_process(line):
    """utils/utils.py:424-437."""
    if line is None:
        return line
    line = line.strip()
    urls = re.findall(_URL, line)
    if len(urls) != 0:
        line = line.replace(urls[0], "")
        for index in range(len(urls)):
            line = line.replace(urls[index], "")
    line = re.sub(u"([^一-龥0-9A-Za-z])", "", line)
    return line


def char_split(text):
    """get_data_set_comment's `" ".join([i for i in prefix])` (utils/utils.py:391-396)."""
    return " ".join([i for i in text])
