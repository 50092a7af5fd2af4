"""Read requests by size per launch (tools/pmc_req.sh): TCC_EA0_RDREQ (all), _32B (32-byte
requests) and TCC_BUBBLE (128-byte requests, as counted), per bench probe name, with the byte
estimates they imply: 'fetch_size' is rocprofv3's FETCH_SIZE formula, 'bytes_if_wide_128'
counts every request that is not a 32-byte one as 128 B (the gfx950 reading of FETCH_SIZE's
½ for wide streaming reads, MI355X_MICROARCH.md § HBM)."""
import json
import sys

sys.path.insert(0, __file__.rsplit('/', 1)[0])
from pmc_traffic import dispatches, per_name  # noqa: E402


def main(d, out_path):
    c = {k: per_name(dispatches(d, k)) for k in ('TCC_EA0_RDREQ_sum', 'TCC_EA0_RDREQ_32B_sum', 'TCC_BUBBLE_sum')}
    res = {}
    for k in sorted(c['TCC_EA0_RDREQ_sum']):
        rq, r32, bb = (c[n].get(k, 0.0) for n in ('TCC_EA0_RDREQ_sum', 'TCC_EA0_RDREQ_32B_sum', 'TCC_BUBBLE_sum'))
        res[k] = {'rdreq': rq, 'rdreq_32b': r32, 'bubble_128b': bb,
                  'fetch_size_bytes': 128 * bb + 64 * (rq - bb - r32) + 32 * r32,
                  'bytes_if_wide_128': 32 * r32 + 128 * (rq - r32),
                  'frac_32b': r32 / rq if rq else None}
    json.dump(res, open(out_path, 'w'), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
