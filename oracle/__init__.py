"""oracle — TEST INFRASTRUCTURE ONLY: CPU restatement of the reference's
GraphExecutor (graph_oracle.cpp) and Histogram (histogram.py), the checker of
the HIP path.  Never imported by the product (fantoch_amd/)."""
