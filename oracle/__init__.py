"""Test-infrastructure oracle (CPU restatement of the Go sst/ path). Never imported by the product."""
