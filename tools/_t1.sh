timeout -k 10 300 python3 -u -m pytest tests -x -q -m gpu -k "k_step_goal or local_shard or smoke" --timeout 180 --timeout-method thread -p no:cacheprovider 2>&1 | tail -5
