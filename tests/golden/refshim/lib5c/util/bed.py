import re


def parse_feature_from_string(s):
    m = re.match(r'(\w+):(\d+)-(\d+)', s)
    return {'chrom': m.group(1), 'start': int(m.group(2)),
            'end': int(m.group(3))}
