set -e
timeout -k 10 400 python -u -m pytest tests/test_abstracts.py tests/test_events.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gputest.log 2>&1
