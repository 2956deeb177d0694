"""commefficient_amd: communication-efficient federated SGD, MI355X-native."""
